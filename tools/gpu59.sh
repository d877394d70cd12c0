# streaming K<=4 edge-layer kernels (dgrad + BN-backward, forward + BN stats; tree) vs the v1 GEMM
# path (build_ab/dsmall0.so): GEMM tests, bench interleaved, then a kernel-trace profile of the tree
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py tests/test_train_step_gpu.py tests/test_pointnet_gpu.py tests/test_graph_gpu.py tests/test_inference_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -1 gpurun_out/t_sub.log
ALT=dsmall0 bash tools/gpu48.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ds2_prof -o step --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 20 > $R/gpurun_out/ds2_prof.log 2>&1 || { echo "prof failed"; exit 1; }
find $R/gpurun_out/ds2_prof -name "*kernel_trace.csv" -delete
