# final profile set r1y + the default bench (with CPU baseline) + smoke
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_prof.sh r1y > gpurun_out/prof_r1y.log 2>&1 || { tail -20 gpurun_out/prof_r1y.log; exit 1; }
cp gpurun_out/r1y_pmc_summary.json profiles/
cd $R
timeout -k 10 400 python bench.py > gpurun_out/bench_r1y.log 2>&1 || { tail -20 gpurun_out/bench_r1y.log; exit 1; }
tail -1 gpurun_out/bench_r1y.log | cut -c1-300
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
