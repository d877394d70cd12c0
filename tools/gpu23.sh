# eager vs graph (bucket 1 / 8), 30 steps each
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for m in "" "--graph" "--graph --graph-bucket 8" "" "--graph"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-breakdown --steps 30 $m > gpurun_out/b.log 2>&1 || exit 1
  echo "$m $(tail -1 gpurun_out/b.log | cut -c1-200)" >> gpurun_out/cmp.txt
done
