# graphed inference: its tests, then the inference rate (eager vs graph)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inference_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_inf.log 2>&1 || { tail -40 gpurun_out/t_inf.log; exit 1; }
tail -3 gpurun_out/t_inf.log
timeout -k 10 200 python tools/infer_bench.py --iters 30 > gpurun_out/inf.txt 2>&1 || { tail -20 gpurun_out/inf.txt; exit 1; }
grep "^{" gpurun_out/inf.txt
