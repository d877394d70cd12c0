# edge-layer streaming kernels at 1024 threads: edge tests + GEMM/step tests, bench A/B vs the v1
# GEMM path (build_ab/dsmall0.so), kernel-trace profile of the tree
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_edge_gpu.py tests/test_mlp_gpu.py tests/test_train_step_gpu.py tests/test_pointnet_gpu.py tests/test_inference_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/t_sub.log | tail -30; exit 1; }
grep -c PASSED gpurun_out/t_sub.log
ALT=dsmall0 bash tools/gpu48.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ds3_prof -o step --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 20 > $R/gpurun_out/ds3_prof.log 2>&1 || { echo "prof failed"; exit 1; }
find $R/gpurun_out/ds3_prof -name "*kernel_trace.csv" -delete
