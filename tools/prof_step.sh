# GPU-box profile of the headline step (bench.py config 2 without the side measurements):
#   1. rocprofv3 --kernel-trace --stats           -> <tag>_stats/ (stats CSV) + the bench line under it
#   2. rocprofv3 --kernel-trace (no --stats)      -> per-kernel stats computed by tools/trace_stats.py
# The bench's own roofline.avg_launch_ms (HIP events) is printed by both runs for comparison.
# Usage: bash tools/prof_step.sh <tag> [steps]
set -o pipefail
T=${1:-r2}
K=${2:-20}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-breakdown --no-extras --steps $K"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_stats -o step --output-format csv -- python3 $R/bench.py $B > $R/gpurun_out/${T}_stats.log 2>&1 || { echo "stats run failed rc=$?"; tail -20 $R/gpurun_out/${T}_stats.log; exit 1; }
tail -1 $R/gpurun_out/${T}_stats.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_trace -o step --output-format csv -- python3 $R/bench.py $B > $R/gpurun_out/${T}_trace.log 2>&1 || { echo "trace run failed rc=$?"; tail -20 $R/gpurun_out/${T}_trace.log; exit 1; }
tail -1 $R/gpurun_out/${T}_trace.log
cd $R
# all launches, and only the timed steps (bench default, graph replay: 1 GEMM-timer eager step + 4 warmup steps (eager + capture) + K replayed steps)
python3 tools/trace_stats.py gpurun_out/${T}_trace gpurun_out/${T}_trace_stats.csv --top 60 > gpurun_out/${T}_trace_top.txt
python3 tools/trace_stats.py gpurun_out/${T}_trace gpurun_out/${T}_trace_timed_stats.csv --tail $K/$((K + 5)) --top 60 > gpurun_out/${T}_trace_timed_top.txt
python3 tools/trace_stats.py gpurun_out/${T}_stats gpurun_out/${T}_stats_timed_stats.csv --tail $K/$((K + 5)) --top 5 > /dev/null
# one replayed step's kernel sequence (durations, gaps) for the tail breakdown
python3 tools/trace_seq.py gpurun_out/${T}_trace > gpurun_out/${T}_seq.txt 2>&1 || true
find gpurun_out/${T}_stats gpurun_out/${T}_trace -name "*kernel_trace.csv" -delete
head -30 gpurun_out/${T}_trace_top.txt
