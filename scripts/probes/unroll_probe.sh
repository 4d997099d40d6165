#!/bin/bash
# RCCL_UNROLL_FACTOR A/B on the 1-GPU bench (RCCL's kernel table is built for
# a few unroll factors; its INFO log reports the one in use, "RCCL Unroll
# Factor (pre-set): 1" on MI355X by default).  Settings are interleaved, REPS
# rounds, each the driver-shaped bench with the untimed sections off; RCCL's
# INFO log of every run is kept to show the factor it used.
#   bash scripts/probes/unroll_probe.sh [out_dir] [reps] [factors...]
set -u
OUT=${1:-gpurun_out/unroll}
REPS=${2:-2}
shift 2 2>/dev/null
FACTORS=${*:-default 2 4}
mkdir -p "$OUT/logs"
for rep in $(seq 1 "$REPS"); do
  for u in $FACTORS; do
    if [ "$u" = default ]; then envs=(P2P_UNUSED=1); else envs=(RCCL_UNROLL_FACTOR=$u); fi
    env "${envs[@]}" TMPDIR="$PWD/$OUT/logs" P2P_RCCL_LOG=keep timeout -k 10 180 python bench.py --steps 20 \
      --warmup 5 --ipc-extra 0 --ref-iters 0 --latency-iters 50 > "$OUT/u${u}_$rep.json" 2> "$OUT/u${u}_$rep.err"
    rc=$?
    used=$(grep -h "Unroll Factor" "$OUT"/logs/*.log 2>/dev/null | tail -1 | sed 's/.*NCCL INFO //')
    rm -f "$OUT"/logs/*.log
    echo "unroll=$u rep=$rep rc=$rc $(python3 -c "import json; r=json.loads([l for l in open('$OUT/u${u}_$rep.json') if l.startswith('{')][0]); print(r['value'], r['matrix_gbs_mean'], r['posting']['rccl_comms'])" 2>/dev/null) [$used]" | tee -a "$OUT/summary.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
