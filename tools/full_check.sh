# Full check on one box: the whole GPU suite once (-x, multi-process rehearsals last), smoke,
# the default bench line, then (AB=<lib.so>) a whole-step A/B of the in-tree library against
# that build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6a}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline'])"
if [ -n "$AB" ]; then bash tools/gpu_lib_ab.sh $AB 3 > gpurun_out/${TAG}_step_ab.log 2>&1 || { tail -20 gpurun_out/${TAG}_step_ab.log; exit 1; }; cat gpurun_out/${TAG}_step_ab.log; fi
