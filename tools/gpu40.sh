# kernel trace of the default bench step; keep per-launch rows of the kernels named in $KT
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o step --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 5 --warmup 2 > $R/gpurun_out/kt.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $R/gpurun_out/kt.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, glob, os
f = glob.glob("gpurun_out/kt/**/*kernel_trace.csv", recursive=True)[0]
keys = os.environ.get("KT", "bn_bwd_apply").split(",")
out = open("gpurun_out/kt_sel.csv", "w")
w = None
for r in csv.DictReader(open(f)):
    if any(k in r["Kernel_Name"] for k in keys):
        if w is None:
            w = csv.DictWriter(out, fieldnames=list(r)); w.writeheader()
        w.writerow(r)
PY
find gpurun_out/kt -name "*kernel_trace.csv" -delete
