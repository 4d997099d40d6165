#!/bin/bash
# RCCL_UNROLL_FACTOR A/B on the 1-GPU bench (RCCL's kernel table is built for
# a few unroll factors; its INFO log reports the pre-set one, 1 on MI355X).
# Each setting runs the driver-shaped bench twice, untimed sections off.
#   bash scripts/unroll_probe.sh [out_dir]
set -u
OUT=${1:-gpurun_out/unroll}
mkdir -p "$OUT"
for u in default 2 4 1; do
  for rep in a b; do
    if [ "$u" = default ]; then envs=(P2P_UNUSED=1); else envs=(RCCL_UNROLL_FACTOR=$u); fi
    env "${envs[@]}" timeout -k 10 180 python bench.py --steps 20 --warmup 5 --ipc-extra 0 --ref-iters 0 \
      --latency-iters 50 > "$OUT/u${u}_$rep.json" 2> "$OUT/u${u}_$rep.err"
    rc=$?
    echo "unroll=$u rep=$rep rc=$rc $(python3 -c "import json,sys; r=json.loads(open('$OUT/u${u}_$rep.json').read().splitlines()[-1]); print(r['value'], r['matrix_gbs_mean'], r['posting']['rccl_comms'])" 2>/dev/null)" | tee -a "$OUT/summary.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
