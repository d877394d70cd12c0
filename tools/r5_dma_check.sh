# Round 5: the LDS-DMA on the compiler builtin. MLP/PointNet parity with the in-tree build, isolated
# GEMM A/B of the DMA forms (asm vs builtin, issue points), whole-step A/B, and the debug-bounds
# build (device traps on an out-of-range LDS-DMA destination or epilogue store) on the MLP tests and
# the single-process config-5 step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_mlp_gpu.py tests/test_pointnet_gpu.py > gpurun_out/r5a_mlp.log 2>&1 || { tail -30 gpurun_out/r5a_mlp.log; exit 1; }
tail -3 gpurun_out/r5a_mlp.log
bash tools/ab_lib_gemm.sh build_ab/asm_s1.so build_ab/bi_s2.so build_ab/bi_s0.so > gpurun_out/r5a_gemm_ab.log 2>&1 || { tail -30 gpurun_out/r5a_gemm_ab.log; exit 1; }
bash tools/gpu_lib_ab.sh build_ab/asm_s1.so 2 > gpurun_out/r5a_step_ab.log 2>&1 || { tail -30 gpurun_out/r5a_step_ab.log; exit 1; }
cat gpurun_out/r5a_step_ab.log
URED_LIB=build_ab/dbg.so timeout -k 10 400 $T tests/test_mlp_gpu.py "tests/test_fullsize_gpu.py::test_config5_train_step_4096_points" > gpurun_out/r5a_dbg.log 2>&1 || { tail -30 gpurun_out/r5a_dbg.log; exit 1; }
tail -3 gpurun_out/r5a_dbg.log
