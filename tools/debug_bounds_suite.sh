# The single-process GPU test suite on the bounds-checked debug build (-DURED_DEBUG_BOUNDS=1:
# device-side checks of the GEMM LDS-DMA ranges and epilogue stores, the node GEMM's raw-buffer
# loads and stores, and the data-dependent indices of the NN / loss / EMD kernels; a violation
# traps). Build it first on the CPU side: bash tools/build_ab.sh debug_bounds -DURED_DEBUG_BOUNDS=1
# The multi-process files (they start their own ranks) are left out.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6dbg}
test -f build_ab/debug_bounds.so || { echo "build_ab/debug_bounds.so missing"; exit 1; }
URED_LIB=$GRAFT_REPO_ROOT/build_ab/debug_bounds.so timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider \
    --ignore=tests/test_bench_gpu.py --ignore=tests/test_dp_configs_gpu.py --ignore=tests/test_dp_gpu.py \
    --ignore=tests/test_graph_dp_gpu.py --ignore=tests/test_nccl_gpu.py --ignore=tests/test_syncbn_gpu.py \
    --ignore=tests/test_train_main_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
