#!/bin/bash
# RCCL communicators per rank x HIP hardware queues (GPU_MAX_HW_QUEUES) on the
# 1-GPU bench at RCCL unroll 4, interleaved, untimed sections off.
#   bash scripts/probes/hwq_comms_probe.sh [out_dir] [reps] ["queues comms"...]
set -u
OUT=${1:-gpurun_out/hwq_comms}
REPS=${2:-2}
shift 2 2>/dev/null
CFGS=("$@")
[ ${#CFGS[@]} -gt 0 ] || CFGS=("4 4" "8 4" "8 6" "8 8" "16 8")
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    q=$1 k=$2
    timeout -k 10 180 python bench.py --hw-queues "$q" --steps 20 --warmup 5 --comms "$k" --ipc-extra 0 \
      --ref-iters 0 --latency-iters 50 > "$OUT/q${q}_k${k}_$rep.json" 2> "$OUT/q${q}_k${k}_$rep.err"
    rc=$?
    echo "hwq=$q comms=$k rep=$rep rc=$rc $(python3 -c "import json; r=json.loads([l for l in open('$OUT/q${q}_k${k}_$rep.json') if l.startswith('{')][0]); print(r['value'], r['matrix_gbs_mean'], r['provenance']['env'].get('GPU_MAX_HW_QUEUES'))" 2>/dev/null)" | tee -a "$OUT/summary.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
