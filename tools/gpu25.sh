# two-stream step: tests + bench (overlap on / off)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
rm -f gpurun_out/cmp.txt
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_train_step_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_2s.log 2>&1 || exit 1
for m in "" "--no-overlap" "" "--no-overlap" "--graph"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --steps 30 $m > gpurun_out/b.log 2>&1 || exit 1
  echo "$m $(tail -1 gpurun_out/b.log | cut -c1-200)" >> gpurun_out/cmp.txt
done
