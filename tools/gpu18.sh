# torch profiler + rocprofv3 kernel stats of the unique-source step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/torch_prof.py --steps 2 > gpurun_out/torch_prof.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_k -o k --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-all-slots-rate > $R/gpurun_out/prof_k.log 2>&1
echo "rc=$?" >> $R/gpurun_out/prof_k.log
