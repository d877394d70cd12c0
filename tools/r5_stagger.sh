# co-resident block stagger (blocks 256..511 start half a tile late): phase timing + step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== phase, stagger"; URED_LIB=build_ab/tsstg.so timeout -k 10 300 python3 tools/gemm_phase.py 2>&1 | grep -v "^{" | grep -v amdgpu.ids || exit 1
bash tools/gpu_lib_ab.sh build_ab/stg2.so 3 || exit 1
bash tools/gpu_lib_ab.sh build_ab/stg4.so 2
