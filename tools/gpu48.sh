# same-box A/B of a build_ab/<name>.so variant against the in-tree library: bench x2 each, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
ALT=${ALT:-ybase}
rm -f gpurun_out/ab.txt
for m in tree alt tree alt; do
  if [ $m = alt ]; then export URED_LIB=$R/build_ab/$ALT.so; else unset URED_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-extras --steps 30 > gpurun_out/b.log 2>&1 || { echo "FAIL $m"; tail -20 gpurun_out/b.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d["gemm_variants"]; print(d["value"], d["ms_per_step"], {k[13:]: (x["ms"], x["tflops"]) for k,x in list(v.items())[:3]})')" >> gpurun_out/ab.txt
done
cat gpurun_out/ab.txt
