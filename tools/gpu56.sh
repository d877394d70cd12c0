# few-tile weight-gradient split depth A/B (URED_WGRAD_FEW_MIN_K 128 / 512 / 1024), bench interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
URED_WGRAD_FEW_MIN_K=1024 timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -1 gpurun_out/t_sub.log
rm -f gpurun_out/ab.txt
for m in 128 512 1024 128 512 1024; do
  URED_WGRAD_FEW_MIN_K=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-extras --steps 30 --shapes-out gpurun_out/shw_$m.json > gpurun_out/b.log 2>&1 || { echo "FAIL $m"; tail -20 gpurun_out/b.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" >> gpurun_out/ab.txt
done
cat gpurun_out/ab.txt
