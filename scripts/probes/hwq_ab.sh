#!/bin/bash
# A/B of the 1-GPU bench at GPU_MAX_HW_QUEUES 4 (box default) / 8 / 16,
# interleaved so box drift hits all arms alike.  Output: gpurun_out/ab/.
set -o pipefail
mkdir -p gpurun_out/ab
for i in $(seq 1 "${1:-6}"); do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py > gpurun_out/ab/q${q}_$i.json 2>/dev/null || exit $?
  done
done
