# BN-backward epilogue G stores through an LDS image as 16-B rows (VST): bounds-checked debug build on
# the MLP tests, MLP / train-step / full-size tests, phase timing with and without, whole-step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
URED_LIB=build_ab/dbg.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_gpu.py > gpurun_out/r5v_dbg_tests.log 2>&1 || { tail -30 gpurun_out/r5v_dbg_tests.log; exit 1; }
tail -1 gpurun_out/r5v_dbg_tests.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_gpu.py tests/test_train_step_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r5v_tests.log 2>&1 || { tail -30 gpurun_out/r5v_tests.log; exit 1; }
tail -1 gpurun_out/r5v_tests.log
echo "== phase, VST"; URED_LIB=build_ab/ts.so timeout -k 10 300 python3 tools/gemm_phase.py 2>&1 | grep -E "epi|launch span|K-loop|whole" || exit 1
echo "== phase, 4-B stores"; URED_LIB=build_ab/ts0.so timeout -k 10 300 python3 tools/gemm_phase.py 2>&1 | grep -E "epi|launch span|K-loop|whole" || exit 1
bash tools/gpu_lib_ab.sh build_ab/vst0.so 3
