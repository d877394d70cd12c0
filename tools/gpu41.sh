# effective clock per kernel (GRBM_GUI_ACTIVE pass) on the default bench step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/clk -o pmc --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-breakdown --no-all-slots-rate --no-extras > $R/gpurun_out/clk.log 2>&1 || { echo "clk pass failed rc=$?"; tail -20 $R/gpurun_out/clk.log; exit 1; }
cd $R
python3 tools/clock_summary.py gpurun_out/clk gpurun_out/clock_summary.json
find gpurun_out/clk -name "*.csv" -delete
