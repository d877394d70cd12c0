set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/graph_diag.py > gpurun_out/graph_diag.txt 2>&1
echo "rc=$?" >> gpurun_out/graph_diag.txt
