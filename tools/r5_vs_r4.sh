# round-5 tree vs the round-4 HEAD tree (build_ab/r4tree, its own library), same box, alternating,
# the same steady-state window for both
set -o pipefail
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 50 --warmup 8"
for rep in 1 2 3; do
  a=$(timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
  b=$(cd build_ab/r4tree && timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
  echo "rep $rep r5 $a   r4 $b"
done
