set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/prof_inflation.py > $R/gpurun_out/infl_bare.json 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/infl_trace -o t --output-format csv -- python3 $R/tools/prof_inflation.py > $R/gpurun_out/infl_prof.json 2>&1 || exit 1
cd $R
cat gpurun_out/infl_bare.json; grep '^{' gpurun_out/infl_prof.json
python3 tools/trace_stats.py gpurun_out/infl_trace --top 4
find gpurun_out/infl_trace -name "*kernel_trace.csv" -delete
