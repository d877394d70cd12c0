# kernel stats only (default bench step)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ks -o step --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 20 > $R/gpurun_out/ks.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $R/gpurun_out/ks.log; exit 1; }
tail -1 $R/gpurun_out/ks.log | cut -c1-200
find $R/gpurun_out/ks -name "*kernel_trace.csv" -delete
