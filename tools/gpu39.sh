# skinny wgrad v2: its tests, then whole GPU suite, then kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_mlp_gpu.py -x -q --timeout 100 --timeout-method thread -k skinny > gpurun_out/t_sk.log 2>&1 || { tail -30 gpurun_out/t_sk.log; exit 1; }
tail -1 gpurun_out/t_sk.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
bash tools/gpu38.sh
