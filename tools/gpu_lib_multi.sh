# Same-box A/B/C... of library builds: bench step rate with each URED_LIB, alternating, each run in
# its own process ("" = the in-tree library).  Usage: REPS=3 bash tools/gpu_lib_multi.sh "" build_ab/x.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 30"
for rep in $(seq ${REPS:-3}); do
  for L in "$@"; do
    r=$(URED_LIB=$L timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], 'gemm_ms', d['gemm_all']['ms_per_step'])") || exit 1
    echo "rep $rep [${L:-in-tree}] $r"
  done
done
