# few-tile weight gradients: more, shorter splits (FEW_WGS/FEW_MIN_K/FEW_MAX) vs the current 512/128/256
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
run() { URED_WGRAD_FEW_WGS=$2 URED_WGRAD_FEW_MIN_K=$3 URED_WGRAD_FEW_MAX=$4 timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-extras --steps 30 --shapes-out gpurun_out/shx_$1.json > gpurun_out/b.log 2>&1 || { echo "FAIL $1"; tail -20 gpurun_out/b.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" >> gpurun_out/ab.txt; }
URED_WGRAD_FEW_WGS=1024 URED_WGRAD_FEW_MIN_K=32 URED_WGRAD_FEW_MAX=1024 timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -1 gpurun_out/t_sub.log
rm -f gpurun_out/ab.txt
for i in 1 2; do
  run cur 512 128 256 && run w1024k64 1024 64 512 && run w1024k32 1024 32 1024 && run w2048k32 2048 32 1024 || exit 1
done
cat gpurun_out/ab.txt
