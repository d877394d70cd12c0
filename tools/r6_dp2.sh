# data-parallel graph tests + bench's N = 2 gloo path, outputs kept
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6h}
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_graph_dp_gpu.py tests/test_nccl_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "rank [01]:|nccl world|passed|failed" gpurun_out/${TAG}_tests.log | tail -8
TAG=$TAG bash tools/bench2_gloo.sh
