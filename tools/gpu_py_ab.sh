# Same-box A/B of a Python-level knob: bench step rate with ENV=0 / ENV=1 alternating, each in
# its own process.  Usage: bash tools/gpu_py_ab.sh URED_GRAD_VIEWS [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$1
N=${2:-3}
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-breakdown --no-extras --steps 30"
for rep in $(seq $N); do
  for x in 0 1; do
    r=$(env $V=$x timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
    echo "rep $rep $V=$x $r it/s"
  done
done
