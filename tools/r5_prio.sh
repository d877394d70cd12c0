# s_setprio around the MFMA cluster, re-checked on the final K loop: step A/B vs URED_GEMM_PRIO=0
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_lib_ab.sh build_ab/prio0.so 4
