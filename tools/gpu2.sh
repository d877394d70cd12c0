set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests/test_mlp_gpu.py -x -q > gpurun_out/t_mlp.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t_mlp.log
