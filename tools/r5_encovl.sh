# target encoder on a side stream (engine/train.py _encoders): step / graph / DP tests, then whole-step
# A/B against URED_ENCODER_OVERLAP=0, alternating processes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_train_step_gpu.py tests/test_graph_gpu.py tests/test_fullsize_gpu.py tests/test_losshead_gpu.py tests/test_nccl_gpu.py tests/test_graph_dp_gpu.py tests/test_dp_gpu.py > gpurun_out/r5o_tests.log 2>&1 || { tail -30 gpurun_out/r5o_tests.log; exit 1; }
tail -1 gpurun_out/r5o_tests.log
B="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --steps 30"
for rep in 1 2 3; do
  a=$(timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'])") || exit 1
  b=$(URED_ENCODER_OVERLAP=0 timeout -k 10 200 python3 bench.py $B 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'])") || exit 1
  echo "rep $rep overlap $a  no-overlap $b"
done
