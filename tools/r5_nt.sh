# non-temporal Yp loads (and G stores) in the BN-backward dgrad epilogue: whole-step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_lib_ab.sh build_ab/ntyp.so 3 || exit 1
bash tools/gpu_lib_ab.sh build_ab/ntboth.so 3
