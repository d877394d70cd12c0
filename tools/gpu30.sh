# pseudo-label table, retrieval metrics, inference extras
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pseudo_labels.py tests/test_retrieval_metrics.py tests/test_inference_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_f23.log 2>&1 || { tail -40 gpurun_out/t_f23.log; exit 1; }
tail -3 gpurun_out/t_f23.log
