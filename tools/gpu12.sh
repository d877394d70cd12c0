set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_p1.log 2>&1 && \
timeout -k 10 300 python tools/gemm_sweep.py > gpurun_out/sweep.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --shapes-out gpurun_out/shapes.json > gpurun_out/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step -o step --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_step.log 2>&1
echo "rc=$?" >> $R/gpurun_out/bench.log
