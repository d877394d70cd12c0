# GPU-box profile of the default bench: rocprofv3 kernel-trace stats, then separate FETCH_SIZE and
# WRITE_SIZE PMC passes (MI355X_MICROARCH.md: one TCC counter group per pass), then the per-kernel
# HBM-traffic summary. Usage: bash tools/gpu_prof.sh <tag>   (outputs under gpurun_out/<tag>_*)
set -o pipefail
T=${1:-r1}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o step --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-breakdown --no-extras --steps 20 > $R/gpurun_out/${T}_prof.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $R/gpurun_out/${T}_prof.log; exit 1; }
tail -1 $R/gpurun_out/${T}_prof.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/${T}_pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-all-slots-rate --no-k16-rate --no-extras > $R/gpurun_out/${T}_pmc_fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; tail -20 $R/gpurun_out/${T}_pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/${T}_pmc_write -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-all-slots-rate --no-k16-rate --no-extras > $R/gpurun_out/${T}_pmc_write.log 2>&1 || { echo "write pass failed rc=$?"; tail -20 $R/gpurun_out/${T}_pmc_write.log; exit 1; }
cd $R
python3 tools/pmc_summary.py gpurun_out/${T}_prof gpurun_out/${T}_pmc_fetch gpurun_out/${T}_pmc_write gpurun_out/${T}_pmc_summary.json gpurun_out/${T}_prof.log
# the trace CSVs are large; keep only the stats and counter summaries (the check above read them)
find gpurun_out/${T}_prof gpurun_out/${T}_pmc_fetch gpurun_out/${T}_pmc_write -name "*kernel_trace.csv" -delete
ls -R gpurun_out | head -40
