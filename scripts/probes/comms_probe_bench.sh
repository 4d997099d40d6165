#!/bin/bash
# RCCL communicators per rank (--comms K) on the driver-shaped 1-GPU bench,
# interleaved, REPS rounds, untimed sections off (one box).
#   bash scripts/probes/comms_probe_bench.sh [out_dir] [reps] [K...]
set -u
OUT=${1:-gpurun_out/comms_probe}
REPS=${2:-2}
shift 2 2>/dev/null
KS=${*:-2 3 4}
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for k in $KS; do
    timeout -k 10 180 python bench.py --steps 20 --warmup 5 --comms "$k" --ipc-extra 0 --ref-iters 0 \
      --latency-iters 50 > "$OUT/k${k}_$rep.json" 2> "$OUT/k${k}_$rep.err"
    rc=$?
    echo "comms=$k rep=$rep rc=$rc $(python3 -c "import json; r=json.loads([l for l in open('$OUT/k${k}_$rep.json') if l.startswith('{')][0]); print(r['value'], r['matrix_gbs_mean'], r['posting']['tuning_ms_per_step'])" 2>/dev/null)" | tee -a "$OUT/summary.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
