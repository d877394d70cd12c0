#!/bin/bash
# A/B of the emulated-fp32 GEMM builds in build_ab/: poisoned-allocation determinism, 4-process
# contention determinism, and the step-shape GEMM rates. Output under gpurun_out/$TAG*.
TAG=${TAG:-r4i}
set -o pipefail
for v in $POISON; do for pv in nan 3e38; do
  echo "== poison $v $pv"
  URED_LIB=$PWD/build_ab/$v.so timeout -k 10 200 python tools/determinism.py --poison $pv > gpurun_out/${TAG}_poison_${v}_$pv.log 2>&1 || exit 1
  grep -h "deterministic\|differ\|layer-0" gpurun_out/${TAG}_poison_${v}_$pv.log | head -8
done; done
for v in $CONTEND; do
  echo "== contention $v"
  for i in 1 2 3 4; do URED_LIB=$PWD/build_ab/$v.so timeout -k 10 200 python tools/determinism.py > gpurun_out/${TAG}_c_${v}_$i.log 2>&1 & done
  wait
  grep -h "deterministic\|differ$\|layer-0" gpurun_out/${TAG}_c_${v}_*.log | sort | uniq -c
done
for v in $GEMM; do
  echo "== gemm $v"
  URED_LIB=$PWD/build_ab/$v.so timeout -k 10 200 python tools/gemm_bench.py --step > gpurun_out/${TAG}_gemm_$v.log 2>&1 || exit 1
  grep "^step" gpurun_out/${TAG}_gemm_$v.log
done
