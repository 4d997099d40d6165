#!/bin/bash
# Messages per step x RCCL communicators on the 1-GPU bench (8 hardware
# queues, unroll 4), interleaved; prints value, device-time matrix and the
# host's posting time per step (host_post_ms_per_step vs ms_per_step).
#   bash scripts/probes/msgs_comms_probe.sh [out_dir] [reps] ["msgs comms"...]
set -u
OUT=${1:-gpurun_out/msgs_comms}
REPS=${2:-2}
shift 2 2>/dev/null
CFGS=("$@")
[ ${#CFGS[@]} -gt 0 ] || CFGS=("32 4" "32 8" "64 4" "64 8")
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    m=$1 k=$2
    timeout -k 10 180 python bench.py --msgs "$m" --comms "$k" --steps 20 --warmup 5 --ipc-extra 0 --ref-iters 0 \
      --latency-iters 50 > "$OUT/m${m}_k${k}_$rep.json" 2> "$OUT/m${m}_k${k}_$rep.err"
    rc=$?
    echo "msgs=$m comms=$k rep=$rep rc=$rc $(python3 -c "import json; r=json.loads([l for l in open('$OUT/m${m}_k${k}_$rep.json') if l.startswith('{')][0]); print(r['value'], r['matrix_gbs_mean'], r['ms_per_step'], r['host_post_ms_per_step'])" 2>/dev/null)" | tee -a "$OUT/summary.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
