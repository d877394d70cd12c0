# node GEMM v4 with three resident workgroups per CU: node tests, DeformNet A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
URED_LIB=build_ab/n4wg3.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_node_gpu.py tests/test_attn_gpu.py 2>&1 | tail -1 || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | grep deformnet | sed "s/^/wg2 /" || exit 1
  URED_LIB=build_ab/n4wg3.so timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | grep deformnet | sed "s/^/wg3 /" || exit 1
done
