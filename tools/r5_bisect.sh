# round-5 step-rate bisection: the bench (steady-state window) of HEAD and of whole-tree checkouts of
# this round's code commits (build_ab/t_<sha>, each with its own library), same box, two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 50 --warmup 8"
run() { (cd $1 && timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'])"); }
for rep in 1 2; do
  for t in build_ab/r4tree build_ab/t_03c12db build_ab/t_ccd3f97 build_ab/t_3bf9b5a build_ab/t_6159309 build_ab/t_d854e98 .; do
    v=$(run $t) || exit 1
    echo "rep $rep $t $v"
  done
done
