# group_colsum widening: GPU suite, colsum trace, bench x2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
KT=group_colsum,splitk_reduce bash tools/gpu40.sh > gpurun_out/kt_print.log 2>&1 || { tail -20 gpurun_out/kt_print.log; exit 1; }
cd $R
rm -f gpurun_out/cmp.txt
for m in "" ""; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 40 $m > gpurun_out/b.log 2>&1 || { echo "FAIL $m"; tail -20 gpurun_out/b.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" >> gpurun_out/cmp.txt
done
cat gpurun_out/cmp.txt
