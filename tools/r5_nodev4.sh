# node GEMM v4 (URED_NODE_RING half-chunks in flight, float4 for k-contiguous operands) vs v1 and vs a
# 2-deep ring: node / attention / grad-view / train-step tests, DeformNet graph timing, phases, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_node_gpu.py tests/test_attn_gpu.py tests/test_grad_views_gpu.py tests/test_train_step_gpu.py > gpurun_out/r5w_tests.log 2>&1 || { tail -30 gpurun_out/r5w_tests.log; exit 1; }
tail -1 gpurun_out/r5w_tests.log
for r in 1 2; do
  timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | grep deformnet | sed "s/^/v4 ring4 /" || exit 1
  URED_LIB=build_ab/ring2.so timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | grep deformnet | sed "s/^/v4 ring2 /" || exit 1
  URED_LIB=build_ab/nodev1.so timeout -k 10 120 python3 tools/deformnet_bench.py --graph --iters 100 2>&1 | grep deformnet | sed "s/^/v1 /" || exit 1
done
echo "== v4 phase 288x1536x512"; URED_LIB=build_ab/nts4.so timeout -k 10 120 python3 tools/node_phase.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== v4 phase 288x1024x1024"; URED_LIB=build_ab/nts5.so timeout -k 10 120 python3 tools/node_phase.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/gpu_lib_ab.sh build_ab/nodev1.so 3
