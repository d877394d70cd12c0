# node BatchNorm rows cached in registers: node / attention / train-step tests, DeformNet A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_node_gpu.py tests/test_attn_gpu.py tests/test_grad_views_gpu.py tests/test_train_step_gpu.py tests/test_syncbn_gpu.py > gpurun_out/r5b2_tests.log 2>&1 || { tail -30 gpurun_out/r5b2_tests.log; exit 1; }
tail -1 gpurun_out/r5b2_tests.log
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | grep deformnet | sed "s/^/cached /" || exit 1
  URED_LIB=build_ab/nbn0.so timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | grep deformnet | sed "s/^/loops /" || exit 1
done
