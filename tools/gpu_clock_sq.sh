# GPU-box counter passes of the default bench step for the bench's roofline extras:
#   1. GRBM_GUI_ACTIVE                              -> <tag>_clock_summary.json (held clock per kernel)
#   2. SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE   -> <tag>_sq_summary.json (MFMA-busy fraction)
# One counter group per pass (MI355X_MICROARCH.md). Usage: bash tools/gpu_clock_sq.sh <tag>
set -o pipefail
T=${1:-r2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="--steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-all-slots-rate --no-k16-rate --no-extras"
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/${T}_clk -o pmc --output-format csv -- python3 $R/bench.py $B > $R/gpurun_out/${T}_clk.log 2>&1 || { echo "clock pass failed rc=$?"; tail -20 $R/gpurun_out/${T}_clk.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/${T}_sq -o pmc --output-format csv -- python3 $R/bench.py $B > $R/gpurun_out/${T}_sq.log 2>&1 || { echo "sq pass failed rc=$?"; tail -20 $R/gpurun_out/${T}_sq.log; exit 1; }
cd $R
python3 tools/clock_summary.py gpurun_out/${T}_clk gpurun_out/${T}_clock_summary.json
python3 tools/sq_summary.py gpurun_out/${T}_sq gpurun_out/${T}_sq_summary.json gemm2 node_gemm bn_bwd_apply nn_fused
find gpurun_out/${T}_clk gpurun_out/${T}_sq -name "*.csv" -delete
