# default bench window (10 timed steps, 3 warmup) vs longer windows, same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras"
for rep in 1 2; do
  for args in "--steps 10 --warmup 3" "--steps 30 --warmup 3" "--steps 50 --warmup 8"; do
    v=$(timeout -k 10 300 python3 bench.py $B $args 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
    echo "rep $rep [$args] $v"
  done
done
