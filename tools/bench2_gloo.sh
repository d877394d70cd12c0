# bench.py's N = 2 path (gloo, both ranks on the box's one GPU) with its full output kept
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6g}
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --batch 4 --no-extras \
    --no-cpu-baseline --no-breakdown --no-all-slots-rate --no-k16-rate --no-loader-rate \
    > gpurun_out/${TAG}_bench2.out 2> gpurun_out/${TAG}_bench2.err; rc=$?
echo "bench2 rc=$rc"; tail -2 gpurun_out/${TAG}_bench2.out
grep -n -A25 "Traceback" gpurun_out/${TAG}_bench2.err | head -80
exit $rc
