set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests/test_train_step_gpu.py -x -q > gpurun_out/t_step.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t_step.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
