# node GEMM v3 (buffer-load ring) vs v1: node/attn/grad-view tests, DeformNet graph timing, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_node_gpu.py tests/test_attn_gpu.py tests/test_grad_views_gpu.py > gpurun_out/r5n_tests.log 2>&1 || { tail -30 gpurun_out/r5n_tests.log; exit 1; }
tail -3 gpurun_out/r5n_tests.log
for r in 1 2; do
  timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | tail -2 | sed "s/^/v3 /" || exit 1
  URED_LIB=build_ab/nodev1.so timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | tail -2 | sed "s/^/v1 /" || exit 1
done
bash tools/gpu_lib_ab.sh build_ab/nodev1.so 3
