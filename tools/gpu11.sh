set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_p1.log 2>&1 && \
URED_GEMM_PERSIST=0 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_p0.log 2>&1 && \
timeout -k 10 300 python tools/gemm_sweep.py > gpurun_out/sweep.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --shapes-out gpurun_out/shapes.json > gpurun_out/bench.log 2>&1
echo "rc=$?" >> gpurun_out/bench.log
