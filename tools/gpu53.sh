# BN-backward epilogue: all 64 Yp values issued at once (tree) vs the two-half form (build_ab/ybase.so):
# GEMM tests, then gemm_bench and bench interleaved on the same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py tests/test_train_step_gpu.py tests/test_pointnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -1 gpurun_out/t_sub.log
for m in tree alt; do
  if [ $m = alt ]; then export URED_LIB=$R/build_ab/ybase.so; else unset URED_LIB; fi
  timeout -k 10 200 python tools/gemm_bench.py --iters 10 > gpurun_out/gb_$m.log 2>&1 || { echo "gb fail $m"; tail gpurun_out/gb_$m.log; exit 1; }
done
unset URED_LIB
for m in tree alt; do echo $m; grep -v "^{" gpurun_out/gb_$m.log | grep -v amdgpu.ids; done
ALT=ybase bash tools/gpu48.sh
