#!/bin/bash
# Same-box A/B of the default bench: the tree at build_ab/head (a copy of an earlier commit with
# its own built library) against this tree, alternating, $REPS rounds.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-abt}
REPS=${REPS:-2}
ARGS="--no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras"
for r in $(seq 1 $REPS); do
  (cd build_ab/head && timeout -k 10 300 python bench.py $ARGS) > gpurun_out/${TAG}_head_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_new_$r.log 2>&1 || exit 1
  for v in head new; do
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_${v}_$r.log $v
  done
done
