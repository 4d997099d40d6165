#!/bin/bash
# Interleaved A/B of environment settings on the driver-shaped 1-GPU bench
# (untimed sections off).  Each setting is "NAME=VAL[,NAME=VAL...]" or
# "default"; REPS rounds over all settings, each round starting one setting
# later than the one before (so no setting always runs first on the box).
#   bash scripts/probes/bench_env_ab.sh <out_dir> <reps> <setting>...
set -u
OUT=$1
REPS=$2
shift 2
mkdir -p "$OUT"
settings=("$@")
n=${#settings[@]}
for rep in $(seq 1 "$REPS"); do
  for i in $(seq 0 $((n - 1))); do
    setting=${settings[$(((i + rep - 1) % n))]}
    envs=(P2P_UNUSED=1)
    [ "$setting" = default ] || IFS=, read -r -a envs <<< "$setting"
    tag=$(echo "$setting" | tr -c 'A-Za-z0-9_=' '_')
    env "${envs[@]}" timeout -k 10 180 python bench.py --steps 20 --warmup 5 --ipc-extra 0 --ref-iters 0 \
      --latency-iters 50 > "$OUT/${tag}_$rep.json" 2> "$OUT/${tag}_$rep.err"
    rc=$?
    echo "$setting rep=$rep rc=$rc $(python3 -c "import json; r=json.loads([l for l in open('$OUT/${tag}_$rep.json') if l.startswith('{')][0]); print(r['value'], r['matrix_gbs_mean'], r['posting']['rccl_comms'], r['posting']['tuning_ms_per_step'], 'first_step_ms', (r.get('rank0_step_ms') or [None])[0], 'bracket_ms', r.get('bracket_overhead_ms'), 'host_post_ms', r.get('host_post_ms_per_step'))" 2>/dev/null)" | tee -a "$OUT/summary.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
