#!/bin/bash
# One-command xGMI pair-cell tuning sweep (needs N >= 2 GPUs; refuses N = 1).
#   scripts/probes/xgmi_pair_sweep.sh [N] [extra args for scripts/xgmi_pair_sweep.py]
# Results: gpurun_out/xgmi_sweep/{rows.jsonl,summary.json}.  See the .py for the rows.
set -o pipefail
cd "$(dirname "$0")/.."
N=${1:-0}; shift || true
exec python3 scripts/xgmi_pair_sweep.py --np "$N" "$@"
