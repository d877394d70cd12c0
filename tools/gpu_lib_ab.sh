# Whole-step A/B of two library builds: bench step rate with the in-tree library (A) and with
# URED_LIB=<lib> (B), alternating, each in its own process. Usage: bash tools/gpu_lib_ab.sh <lib.so> [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$1
N=${2:-3}
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 30"
for rep in $(seq $N); do
  a=$(timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], 'gemm_ms', d['gemm_all']['ms_per_step'], 'dgrad', d['gemm_variants']['gemm2_kernel<false, true, 0, 0, 2, 2, 2>']['ms'])") || exit 1
  echo "rep $rep A in-tree $a"
  b=$(URED_LIB=$L timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], 'gemm_ms', d['gemm_all']['ms_per_step'], 'dgrad', d['gemm_variants']['gemm2_kernel<false, true, 0, 0, 2, 2, 2>']['ms'])") || exit 1
  echo "rep $rep B $L $b"
done
