set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests/test_train_step_gpu.py -x -q > gpurun_out/t_step.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t_step.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step -o step --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_step.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/prof_step.log
