# edge-layer streaming kernels (256 threads): the whole GPU suite, then a kernel-trace profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/t_all.log | tail -30; exit 1; }
tail -1 gpurun_out/t_all.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ds4_prof -o step --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 20 > $R/gpurun_out/ds4_prof.log 2>&1 || { echo "prof failed"; exit 1; }
find $R/gpurun_out/ds4_prof -name "*kernel_trace.csv" -delete
