#!/bin/bash
# 1-GPU bench at several step shapes (messages of 32 MiB per step x RCCL
# communicators), each run verified; one JSON line per run in
# gpurun_out/step_shape/.  Run on a GPU box from the repo root:
#   scripts/probes/step_shape_sweep.sh "8 32 128" "-1 2 3 4"
set -o pipefail
out=gpurun_out/step_shape
mkdir -p $out
for m in ${1:-8 32 128}; do
  for c in ${2:--1}; do
    timeout -k 10 200 python bench.py --msgs "$m" --comms "$c" --steps 20 --warmup 5 \
      > $out/m${m}_c${c}.json 2> $out/m${m}_c${c}.err || exit $?
    python - "$out/m${m}_c${c}.json" "$m" "$c" <<'EOF'
import json, sys
r = json.loads(open(sys.argv[1]).read())
print("msgs %s comms %s: value %.1f GB/s, ms/step %.4f, gpu p50 %.1f GB/s, posting %s, verify %s" % (
    sys.argv[2], sys.argv[3], r["value"], r["ms_per_step"], r["matrix_gbs_mean"],
    r["posting"]["rccl_comms"], r["verify_mismatches"]), flush=True)
EOF
  done
done
