# NN fused-plan A/B + NN tests on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_nn.log 2>&1 || { tail -30 gpurun_out/t_nn.log; exit 1; }
tail -1 gpurun_out/t_nn.log
rm -f gpurun_out/nnab.txt
for v in t4k; do
  timeout -k 10 200 python tools/nn_seg_ab.py 2>/dev/null | tail -1 >> gpurun_out/nnab.txt || { echo "fail $v"; exit 1; }
done
cat gpurun_out/nnab.txt
