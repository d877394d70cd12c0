# Isolated GEMM rates (tools/gemm_bench.py --step) with the in-tree library (A) and with each
# URED_LIB=<lib> given (B, C, ...), alternating A B [C ...] A B [C ...] in separate processes.
# Usage: bash tools/ab_lib_gemm.sh <lib.so> [<lib2.so> ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  echo "== A in-tree"; timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --step 2>&1 | grep -v amdgpu.ids | grep -v '^{' || exit 1
  tag=B
  for L in "$@"; do
    echo "== $tag $L"; URED_LIB=$L timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --step 2>&1 | grep -v amdgpu.ids | grep -v '^{' || exit 1
    tag=$(echo $tag | tr 'A-Y' 'B-Z')
  done
done
