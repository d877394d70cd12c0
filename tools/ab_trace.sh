# A/B of two libured_hip.so builds on one command by kernel time: rocprofv3 kernel traces of
# `<cmd>` with the in-tree library and with URED_LIB=<lib>; per-kernel totals side by side.
# Usage: bash tools/ab_trace.sh <lib.so> <tag> <python args...>
set -o pipefail
LIB=$1; TAG=$2; shift 2
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_A -o t --output-format csv -- python3 "$@" > $R/gpurun_out/${TAG}_A.log 2>&1 || exit 1
URED_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_B -o t --output-format csv -- python3 "$@" > $R/gpurun_out/${TAG}_B.log 2>&1 || exit 1
cd $R
echo "== A (in-tree)"; python3 tools/trace_stats.py gpurun_out/${TAG}_A --top 12
echo "== B ($LIB)"; python3 tools/trace_stats.py gpurun_out/${TAG}_B --top 12
find gpurun_out/${TAG}_A gpurun_out/${TAG}_B -name "*kernel_trace.csv" -delete
