set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_v2.log 2>&1 && \
URED_GEMM_V1=1 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_v1.log 2>&1
echo "rc=$?" >> gpurun_out/gemm_v1.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc_gemm -o g --output-format csv -- python3 $R/tools/gemm_bench.py --iters 3 > $R/gpurun_out/pmc_gemm.log 2>&1
echo "rc=$?" >> $R/gpurun_out/pmc_gemm.log
