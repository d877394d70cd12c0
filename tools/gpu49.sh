# inference A/B: current tree vs the r1y worktree (build_ab/r1y), same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for t in cur r1y cur r1y; do
  if [ $t = cur ]; then D=$R; else D=$R/build_ab/r1y; fi
  echo "== $t" >> gpurun_out/inf.txt
  (cd $D && timeout -k 10 200 python tools/infer_bench.py --iters 30) >> gpurun_out/inf.txt 2>&1 || { echo "FAIL $t"; tail -20 gpurun_out/inf.txt; exit 1; }
done
grep -v "^W\|amdgpu.ids" gpurun_out/inf.txt
