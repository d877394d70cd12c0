# Data-parallel / graph-replay checks on one box (gloo world 2 on the one GPU, RCCL world 1), then
# the default bench line. Usage: TAG=... bash tools/dp_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6dp}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_graph_dp_gpu.py tests/test_nccl_gpu.py tests/test_dp_gpu.py tests/test_graph_gpu.py \
    tests/test_bench_gpu.py > gpurun_out/${TAG}_dp_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_dp_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_dp_tests.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d.get('all_slots_iters_s'), d.get('k16_iters_s'), d.get('side_rates_mode'), d['roofline']['frac'])"
