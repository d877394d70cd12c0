#!/bin/bash
# tools/xproc.py: one checker process beside 3 GEMM load processes.
# LIBS: "checkerlib:loadlib[:loadenv]" pairs (build_ab/*.so names)
for pair in $LIBS; do
  IFS=: read cl ll le <<< "$pair"
  echo "== checker $cl, load $ll $le"
  for i in 1 2 3; do env $le URED_LIB=$PWD/build_ab/$ll.so timeout -k 10 120 python tools/xproc.py load --seconds 40 > gpurun_out/${TAG}_load_${ll}_$i.log 2>&1 & done
  sleep 8
  URED_LIB=$PWD/build_ab/$cl.so timeout -k 10 120 python tools/xproc.py check --seconds 25 2>&1 | grep check
  wait
done
