# BLAS backend A/B for the small torch GEMMs
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
rm -f gpurun_out/cmp.txt
for m in "" "--blas rocblas" "--blas hipblaslt" "" "--blas rocblas"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 30 $m > gpurun_out/b.log 2>&1 || { echo "FAIL $m"; tail -20 gpurun_out/b.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" >> gpurun_out/cmp.txt
done
cat gpurun_out/cmp.txt
