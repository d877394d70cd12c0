# GPU-box check: gpu tests, smoke, bench (graph replay, the default, + eager). Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python bench.py --eager --no-cpu-baseline --no-all-slots-rate > gpurun_out/bench_eager.log 2>&1 || { echo "bench eager failed"; tail -30 gpurun_out/bench_eager.log; exit 1; }
tail -1 gpurun_out/bench_eager.log
