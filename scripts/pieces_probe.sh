#!/bin/bash
# RCCL self path: messages split into P ops (P2P_RCCL_PIECES) x communicators.
# Output: gpurun_out/pieces/.
set -o pipefail
mkdir -p gpurun_out/pieces
for p in 1 2 4; do
  P2P_RCCL_PIECES=$p timeout -k 10 200 python scripts/comms_probe.py --comms 1,2,4 > gpurun_out/pieces/p$p.txt 2>/dev/null || exit $?
done
