# DMA issue point on the final K loop: in-tree (2: behind the fragment reads, ahead of the MFMAs) vs
# 0 (before the fragment reads, also ahead of the MFMAs) and 1 (among the MFMAs, round 4's placement)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_lib_ab.sh build_ab/sp0.so 3 || exit 1
bash tools/gpu_lib_ab.sh build_ab/sp1.so 2
