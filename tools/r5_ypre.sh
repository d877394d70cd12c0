# BN-backward Yp prefetch in the last K-step: MLP/train-step tests, phase timing with and without,
# whole-step A/B against the URED_BNBWD_YPRE=0 build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_gpu.py tests/test_train_step_gpu.py > gpurun_out/r5y_tests.log 2>&1 || { tail -30 gpurun_out/r5y_tests.log; exit 1; }
tail -2 gpurun_out/r5y_tests.log
echo "== phase, prefetch on"; URED_LIB=build_ab/ts.so timeout -k 10 300 python3 tools/gemm_phase.py 2>&1 | grep -v "^{" | grep -v amdgpu.ids || exit 1
echo "== phase, prefetch off"; URED_LIB=build_ab/ts0.so timeout -k 10 300 python3 tools/gemm_phase.py 2>&1 | grep -v "^{" | grep -v amdgpu.ids || exit 1
bash tools/gpu_lib_ab.sh build_ab/ypre0.so 3
