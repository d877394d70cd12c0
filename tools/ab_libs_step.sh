# Same-box A/B of library builds: isolated GEMM rates (tools/gemm_bench.py --step) and the default
# bench's step rate, alternating the builds named in $LIBS (build_ab/<name>.so), $REPS rounds.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-abg}
for r in $(seq 1 ${REPS:-2}); do
for v in $LIBS; do
  URED_LIB=$PWD/build_ab/$v.so timeout -k 10 200 python tools/gemm_bench.py --step > gpurun_out/${TAG}_${v}_$r.log 2>&1 || exit 1
  echo "== $v $r"; grep -E "^step" gpurun_out/${TAG}_${v}_$r.log
done
done
for r in $(seq 1 ${REPS:-2}); do
for v in $LIBS; do
  URED_LIB=$PWD/build_ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras > gpurun_out/${TAG}_bench_${v}_$r.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('bench', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_bench_${v}_$r.log $v
done
done
