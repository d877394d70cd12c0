# GEMM variant A/B: GPU mlp/train tests, then bench with the per-variant breakdown x2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py tests/test_train_step_gpu.py tests/test_pointnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -1 gpurun_out/t_sub.log
rm -f gpurun_out/cmp.txt
for m in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-extras --steps 30 > gpurun_out/b.log 2>&1 || { echo "FAIL $m"; tail -20 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d["gemm_variants"]; print(d["value"], d["ms_per_step"], {k[13:]: (x["ms"], x["tflops"]) for k,x in list(v.items())[:4]})' >> gpurun_out/cmp.txt
done
cat gpurun_out/cmp.txt
