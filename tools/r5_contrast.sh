# contrastive loss kernels with lane-parallel dots / wave-split vector-matrix products: loss-head,
# step, DP and full-size tests; the kernels' in-step durations; whole-step A/B vs the previous form
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_losshead_gpu.py tests/test_losses_gpu.py tests/test_train_step_gpu.py tests/test_dp_gpu.py tests/test_graph_dp_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r5c2_tests.log 2>&1 || { tail -30 gpurun_out/r5c2_tests.log; exit 1; }
tail -1 gpurun_out/r5c2_tests.log
bash tools/gpu_lib_ab.sh build_ab/ct0.so 3
