# torch.profiler op view of the config-2 step (which torch ops launch the small kernels)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/torch_prof.py --steps 2 > gpurun_out/torch_prof.txt 2>&1
echo "rc=$?" >> gpurun_out/torch_prof.txt
