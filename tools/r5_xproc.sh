# Round 5: the cross-process probe (tools/xproc.sh) on the final round-4 DMA form (asm, issue points
# among the MFMAs), the builtin DMA at the same points, and the builtin DMA ahead of the MFMAs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=r5x LIBS="bi_s1:asm_s1 bi_s1:bi_s1 bi_s1:bi_s2 bi_s1:asm_s1" bash tools/xproc.sh 2>&1 | tee gpurun_out/r5x_xproc.log
