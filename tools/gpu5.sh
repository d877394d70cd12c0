set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t_all.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step2 -o step --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-breakdown > $R/gpurun_out/prof_step2.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/prof_step2.log
