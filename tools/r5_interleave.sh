# Round 5: prologue interleaved with the MFMAs (URED_GEMM_INTERLEAVE), tail k-chunks zero-filled by the DMA.
# Parity tests, whole-step A/B vs the non-interleaved build, per-shape GEMM breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r5h}
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_mlp_gpu.py tests/test_pointnet_gpu.py tests/test_edge_gpu.py tests/test_train_step_gpu.py tests/test_fullsize_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash tools/gpu_lib_ab.sh ${AB:-build_ab/noil.so} 3 > gpurun_out/${TAG}_step_ab.log 2>&1 || { tail -20 gpurun_out/${TAG}_step_ab.log; exit 1; }
cat gpurun_out/${TAG}_step_ab.log
timeout -k 10 300 python3 bench.py --steps 5 --no-extras --no-cpu-baseline --no-all-slots-rate --no-k16-rate --shapes-out gpurun_out/${TAG}_shapes.json > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
