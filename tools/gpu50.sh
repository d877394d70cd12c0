# default bench with extras (no CPU baseline) + inference tool for comparison
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/b_ext.log 2>&1 || { tail -20 gpurun_out/b_ext.log; exit 1; }
tail -1 gpurun_out/b_ext.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"]); print(d["inference"]); print(d["chamfer_vs_published"]); print(d["chamfer"])'
