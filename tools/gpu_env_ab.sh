# Same-box A/B of an environment setting: bench step rate without / with `VAR=VALUE`, alternating,
# each in its own process.  Usage: bash tools/gpu_env_ab.sh VAR VALUE [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$1; X=$2; N=${3:-3}
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 30"
for rep in $(seq $N); do
  a=$(timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], 'gemm_ms', d['gemm_all']['ms_per_step'])") || exit 1
  echo "rep $rep default $a"
  b=$(env $V=$X timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], 'gemm_ms', d['gemm_all']['ms_per_step'])") || exit 1
  echo "rep $rep $V=$X $b"
done
