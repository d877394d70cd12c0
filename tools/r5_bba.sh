# BN-backward apply tile width (float4 columns per block row): step A/B of 32 and 64 vs 16
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_lib_ab.sh build_ab/cq32.so 3 || exit 1
bash tools/gpu_lib_ab.sh build_ab/cq64.so 3
