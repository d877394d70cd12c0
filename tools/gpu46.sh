# profile set r1z: kernel stats + FETCH/WRITE passes, clock pass, SQ pass, default bench (CPU baseline), smoke
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
bash tools/gpu_prof.sh r1z > gpurun_out/prof_r1z.log 2>&1 || { tail -20 gpurun_out/prof_r1z.log; exit 1; }
cd $R && cp gpurun_out/r1z_pmc_summary.json profiles/
bash tools/gpu41.sh > gpurun_out/clk_print.log 2>&1 || { tail -20 gpurun_out/clk_print.log; exit 1; }
cd $R && cp gpurun_out/clock_summary.json gpurun_out/r1z_clock_summary.json && cp gpurun_out/r1z_clock_summary.json profiles/
bash tools/gpu42.sh > gpurun_out/sq_print.log 2>&1 || { tail -20 gpurun_out/sq_print.log; exit 1; }
cd $R && cp gpurun_out/sq_summary.json gpurun_out/r1z_sq_summary.json && cp gpurun_out/r1z_sq_summary.json profiles/
timeout -k 10 400 python bench.py > gpurun_out/bench_r1z.log 2>&1 || { tail -20 gpurun_out/bench_r1z.log; exit 1; }
tail -1 gpurun_out/bench_r1z.log | cut -c1-400
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
