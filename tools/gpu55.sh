# few-tile split-K slice length A/B (URED_SPLITK_KMIN 128 / 64 / 32): mlp tests at 32, then bench interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
URED_SPLITK_KMIN=32 timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py tests/test_train_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -1 gpurun_out/t_sub.log
rm -f gpurun_out/ab.txt
for m in 128 32 64 128 32 64; do
  URED_SPLITK_KMIN=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-extras --steps 30 --shapes-out gpurun_out/sh_$m.json > gpurun_out/b.log 2>&1 || { echo "FAIL $m"; tail -20 gpurun_out/b.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" >> gpurun_out/ab.txt
done
cat gpurun_out/ab.txt
