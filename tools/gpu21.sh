# HIP graph with unique sources: graph tests, step tests, bench eager vs graph
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_train_step_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate > gpurun_out/bench_eager.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --graph > gpurun_out/bench_graph.log 2>&1
echo "rc=$?" >> gpurun_out/bench_graph.log
