# SQ counters (issue/wait/MFMA-busy/LDS) + GRBM clock of the default bench step's kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/sq -o pmc --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-breakdown --no-all-slots-rate --no-extras > $R/gpurun_out/sq.log 2>&1 || { echo "sq pass failed rc=$?"; tail -20 $R/gpurun_out/sq.log; exit 1; }
cd $R
python3 tools/sq_summary.py gpurun_out/sq gpurun_out/sq_summary.json gemm2 bn_bwd
find gpurun_out/sq -name "*.csv" -delete
