#!/bin/bash
# Scaling curve of the headline bench on one node: N = 1, 2, 4, 8 GPUs
# (whatever is visible), one torchrun launch per N, results appended as JSON
# lines, then a Markdown table (utils.report.scaling_table).
#
#   bash scripts/scaling.sh [out.jsonl] [extra bench.py args...]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-scaling.jsonl}
shift || true
# P2P_SCALING_GPUS: how many ranks to go up to (node_run.sh --rehearse: 4 ranks on one GPU).
NGPU=${P2P_SCALING_GPUS:-$(python3 -c "import torch; print(torch.cuda.device_count())")}
: > "$OUT"
for N in 1 2 4 8; do
  if [ "$N" -gt "$NGPU" ]; then break; fi
  PORT=$((29500 + RANDOM % 2000))
  if [ "$N" -eq 1 ]; then
    timeout -k 10 600 python3 bench.py --gpus 1 "$@" >> "$OUT"
  else
    timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
      --master-addr 127.0.0.1 --master-port "$PORT" bench.py --gpus "$N" "$@" >> "$OUT"
  fi
done
python3 - "$OUT" <<'PY'
import sys
from test_nccl_p2p_amd.utils.report import read_json_lines, scaling_table
print(scaling_table(read_json_lines(sys.argv[1])))
PY
