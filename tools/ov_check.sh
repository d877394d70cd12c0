set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-breakdown --no-extras --steps 20"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ov_trace -o step --output-format csv -- python3 $R/bench.py $B > $R/gpurun_out/ov_trace.log 2>&1 || exit 1
cd $R
python3 tools/trace_stats.py gpurun_out/ov_trace --top 8
python3 tools/trace_stats.py gpurun_out/ov_trace --top 8 --exclusive
python3 - <<'PY'
import sys; sys.path.insert(0, "tools")
import trace_stats as t
rows = t.load("gpurun_out/ov_trace")
k = "gemm2_kernel<false, true, 0, 0, 2>"
ov = []
for i in range(1, len(rows)):
    if k in rows[i][0]:
        ov.append((rows[i][1] - rows[i-1][2], rows[i][2]-rows[i][1], rows[i-1][0][:60]))
import statistics
print("start - prev_end (ns): median", statistics.median(o[0] for o in ov), "min", min(o[0] for o in ov), "max", max(o[0] for o in ov))
print(ov[:30])
PY
find gpurun_out/ov_trace -name "*kernel_trace.csv" -delete
