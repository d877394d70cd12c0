set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/step_parts.py > gpurun_out/step_parts.txt 2>&1
echo "rc=$?" >> gpurun_out/step_parts.txt
