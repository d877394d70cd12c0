# Isolated GEMM rates (tools/gemm_bench.py --step) with the in-tree library and with URED_LIB=<lib>,
# alternating A B A B in separate processes.  Usage: bash tools/ab_lib_gemm.sh <lib.so>
set -o pipefail
cd $GRAFT_REPO_ROOT
for m in A B A B; do
  if [ $m = A ]; then L=""; else L=$1; fi
  echo "== $m ${L:-in-tree}"; URED_LIB=$L timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --step 2>&1 | grep -v amdgpu.ids | grep -v '^{' || exit 1
done
