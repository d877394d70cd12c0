# rocprofv3 kernel stats of the current step (eager, 5 steps, no extras)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s -o s --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-all-slots-rate --no-breakdown > $R/gpurun_out/prof_s.log 2>&1
echo "rc=$?" >> $R/gpurun_out/prof_s.log
