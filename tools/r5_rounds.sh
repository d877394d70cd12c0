# whole-tree A/B of the round HEADs (round 3, round 4) and this tree, same box, steady-state window
set -o pipefail
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 50 --warmup 8"
run() { (cd $1 && timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'])"); }
for rep in 1 2 3; do
  for t in build_ab/t_34389e9 build_ab/t_4021a98 .; do
    v=$(run $t) || exit 1
    echo "rep $rep $t $v"
  done
done
