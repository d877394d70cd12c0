set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/torch_prof.py > gpurun_out/torch_prof.txt 2>&1 || { echo tp fail; tail gpurun_out/torch_prof.txt; exit 1; }
timeout -k 10 300 python tools/step_parts.py > gpurun_out/step_parts.txt 2>&1 || { echo sp fail; tail gpurun_out/step_parts.txt; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --shapes-out gpurun_out/shapes_u.json > gpurun_out/bench_shapes.log 2>&1 || { echo b fail; exit 1; }
echo done
