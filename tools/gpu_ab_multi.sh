# Same-box A/B/C... of bench variants, alternating, each run in its own process.
# Each argument is one variant: "ENV=VAL ... -- --bench-flag ..." (either side may be empty).
# Usage: bash tools/gpu_ab_multi.sh "" "URED_WGRAD_STREAM=0 --" "-- --deform-overlap"   (REPS=3 default)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 30"
N=${REPS:-3}
for rep in $(seq $N); do
  for v in "$@"; do
    envs="${v%%--*}"; flags=""
    [[ "$v" == *--* ]] && flags="${v#*--}"
    r=$(env $envs timeout -k 10 200 python3 bench.py $B $flags 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], 'gemm_ms', d['gemm_all']['ms_per_step'])") || exit 1
    echo "rep $rep [${v:-default}] $r"
  done
done
