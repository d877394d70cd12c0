#!/bin/bash
# Same-box A/B of the node GEMM: node_bench shapes and the graph-replayed DeformNet fwd+bwd for the
# tree at build_ab/head (a copy of HEAD with its own library) and for this tree.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-abn}
for r in 1 2; do
  (cd build_ab/head && timeout -k 10 120 python tools/deformnet_bench.py --graph --iters 100) > gpurun_out/${TAG}_head_def_$r.log 2>&1 || exit 1
  timeout -k 10 120 python tools/deformnet_bench.py --graph --iters 100 > gpurun_out/${TAG}_new_def_$r.log 2>&1 || exit 1
  grep graph gpurun_out/${TAG}_head_def_$r.log gpurun_out/${TAG}_new_def_$r.log
done
(cd build_ab/head && timeout -k 10 120 python tools/node_bench.py) > gpurun_out/${TAG}_head_node.log 2>&1 || exit 1
timeout -k 10 120 python tools/node_bench.py > gpurun_out/${TAG}_new_node.log 2>&1 || exit 1
paste gpurun_out/${TAG}_head_node.log gpurun_out/${TAG}_new_node.log
