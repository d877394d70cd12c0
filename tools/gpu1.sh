set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests/test_nn_gpu.py -x -q > gpurun_out/t_nn.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t_nn.log
timeout -k 10 300 python tools/nn_bench.py > gpurun_out/nnb.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_nn -o nn --output-format csv -- python3 $R/tools/nn_bench.py --iters 10 > $R/gpurun_out/prof_nn.log 2>&1
echo done
