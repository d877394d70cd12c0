# fused NN forward: GPU tests (whole suite), NN micro-benchmark (fused vs two-pass), short bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_nn.log 2>&1 || { tail -30 gpurun_out/t_nn.log; exit 1; }
tail -3 gpurun_out/t_nn.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 300 python tools/nn_bench.py --iters 30 > gpurun_out/nn_bench.log 2>&1 || { tail -20 gpurun_out/nn_bench.log; exit 1; }
grep -v "^{" gpurun_out/nn_bench.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
