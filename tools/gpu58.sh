# streaming K<=4 dgrad + BN-backward kernel (tree) vs the v1 GEMM path (build_ab/dsmall0.so):
# MLP / train-step / PointNet tests, then bench interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py tests/test_train_step_gpu.py tests/test_pointnet_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -1 gpurun_out/t_sub.log
ALT=dsmall0 bash tools/gpu48.sh
