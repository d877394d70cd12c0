# Round 5: cross-process probe (tools/xproc.sh) with the current GEMM (prologue VALU interleaved with
# the fp32 MFMAs, DMA ahead of them) and with the DMA among the MFMAs (s1il) as load; then the
# whole-step A/B of the two issue points.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=r5i LIBS="cur:cur cur:s1il" bash tools/xproc.sh 2>&1 | tee gpurun_out/r5i_xproc.log
bash tools/gpu_lib_ab.sh build_ab/s1il.so 3 > gpurun_out/r5i_step_ab.log 2>&1 || exit 1
cat gpurun_out/r5i_step_ab.log
