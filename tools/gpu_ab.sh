set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in old packed; do
  URED_LIB=$PWD/build_ab/lib_$v.so timeout -k 10 200 python tools/gemm_bench.py --iters 10 > gpurun_out/ab_$v.log 2>&1 || { echo "fail $v"; tail gpurun_out/ab_$v.log; exit 1; }
done
timeout -k 10 200 python tools/gemm_bench.py --iters 10 > gpurun_out/ab_scalar.log 2>&1 || { echo "fail scalar"; exit 1; }
for v in old packed scalar; do echo $v; grep -v "^{" gpurun_out/ab_$v.log | grep -v amdgpu.ids; done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate > gpurun_out/bench_ab.log 2>&1 || { echo bench fail; tail gpurun_out/bench_ab.log; exit 1; }
tail -1 gpurun_out/bench_ab.log | cut -c1-400
