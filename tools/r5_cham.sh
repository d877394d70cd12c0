# Round 5: NN / chamfer-shim tests (ured_nn_bwd_set), the reference-API chamfer call's wall time vs
# its summed kernel time (rocprofv3 kernel trace), and a kernel trace of the current step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_nn_gpu.py tests/test_chamfer_shim_gpu.py > gpurun_out/r5c_nn.log 2>&1 || { tail -30 gpurun_out/r5c_nn.log; exit 1; }
tail -2 gpurun_out/r5c_nn.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5c_cham -o cham --output-format csv -- python3 $R/tools/chamfer_api_trace.py --iters 200 > $R/gpurun_out/r5c_cham.log 2>&1 || { tail -20 $R/gpurun_out/r5c_cham.log; exit 1; }
cd $R
tail -1 gpurun_out/r5c_cham.log
find gpurun_out/r5c_cham -name "*kernel_stats.csv" | head -1 | xargs cat
find gpurun_out/r5c_cham -name "*kernel_trace.csv" -delete
bash tools/prof_step.sh r5c 20 > gpurun_out/r5c_prof.log 2>&1 || { tail -20 gpurun_out/r5c_prof.log; exit 1; }
tail -32 gpurun_out/r5c_prof.log
