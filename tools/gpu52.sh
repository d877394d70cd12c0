# FlatAdam: train-step tests, whole GPU suite, bench x2 (flat vs torch Adam A/B on the same box)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_train_step_gpu.py tests/test_graph_gpu.py tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/t_sub.log | tail -30; exit 1; }
grep -c PASSED gpurun_out/t_sub.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
rm -f gpurun_out/cmp.txt
for m in 1 0 1 0; do
  URED_FLAT_ADAM=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 40 > gpurun_out/b.log 2>&1 || { echo "FAIL $m"; tail -20 gpurun_out/b.log; exit 1; }
  echo "flat=$m $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" >> gpurun_out/cmp.txt
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 40 --graph > gpurun_out/b.log 2>&1 || { echo "FAIL graph"; tail -20 gpurun_out/b.log; exit 1; }
echo "graph $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" >> gpurun_out/cmp.txt
cat gpurun_out/cmp.txt
