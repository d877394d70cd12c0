set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_graph_gpu.py -x -q > gpurun_out/pytest_graph.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph > gpurun_out/bench_eager.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "rc=$?" >> gpurun_out/bench.log
