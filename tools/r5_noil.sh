# GEMM without the round-5 prologue interleave / branch-free prologue (the narrow-tile commit's K loop)
# vs HEAD's interleaved K loop (build_ab/il.so): MLP / PointNet / edge / step / full-size tests, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_mlp_gpu.py tests/test_pointnet_gpu.py tests/test_edge_gpu.py tests/test_train_step_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r5u_tests.log 2>&1 || { tail -30 gpurun_out/r5u_tests.log; exit 1; }
tail -1 gpurun_out/r5u_tests.log
bash tools/gpu_lib_ab.sh build_ab/il.so 4
