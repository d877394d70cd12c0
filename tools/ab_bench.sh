#!/bin/bash
# Same-box A/B of library builds in build_ab/: GEMM rates (tools/gemm_bench.py --step) and the
# default bench's step rate with the per-variant GEMM breakdown, alternating builds ($LIBS, in order).
TAG=${TAG:-ab}
set -o pipefail
for v in $LIBS; do
  echo "== $v"
  URED_LIB=$PWD/build_ab/$v.so timeout -k 10 200 python tools/gemm_bench.py --step > gpurun_out/${TAG}_gemm_$v.log 2>&1 || exit 1
  grep "^step" gpurun_out/${TAG}_gemm_$v.log
  URED_LIB=$PWD/build_ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras > gpurun_out/${TAG}_bench_$v.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('bench', d['value'], d['ms_per_step']); [print('   ', k, v) for k, v in list(d.get('gemm_variants', {}).items())[:10]]" gpurun_out/${TAG}_bench_$v.log
done
