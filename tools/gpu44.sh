# wgrad split-K sweep (workgroup target x min points per split)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
rm -f gpurun_out/sweep.txt
for cfg in "512 512" "1024 512" "512 256" "512 1024" "256 512" "512 512" "1024 512"; do
  set -- $cfg
  URED_WGRAD_WGS=$1 URED_WGRAD_MIN_K=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --no-extras --steps 40 > gpurun_out/b.log 2>&1 || { echo "FAIL $cfg"; tail -20 gpurun_out/b.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/sweep.txt
done
cat gpurun_out/sweep.txt
