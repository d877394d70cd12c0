# unique-source encoding: step parity tests + bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_train_step_gpu.py tests/test_mlp_gpu.py tests/test_graph_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
echo "rc=$?" >> gpurun_out/bench.log
