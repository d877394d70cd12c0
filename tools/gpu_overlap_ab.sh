# Step rate with and without the optional side streams (source branch / DeformNet+losses),
# alternating, each in its own process.  Usage: bash tools/gpu_overlap_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-breakdown --no-extras --steps 30"
for rep in 1 2; do
  for f in "" "--overlap" "--deform-overlap" "--overlap --deform-overlap"; do
    r=$(timeout -k 10 200 python3 bench.py $B $f 2>/dev/null | tail -1 | python3 -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
    echo "rep $rep [${f:-none}] $r it/s"
  done
done
