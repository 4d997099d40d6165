#!/bin/bash
# Debug helper for the IPC relay engine (run on a GPU box from the repo root):
# 4 processes on GPU 0 push random verified message groups through ipc:relay
# (tests/scripts/fuzz_session.py) with P2P_IPC_DEBUG=1, which prints every
# rank's per-group flag bookkeeping (who it writes to / receives from, the
# ready counters) to stderr.  Output: gpurun_out/rd2/.
set -o pipefail
mkdir -p gpurun_out/rd2
P2P_IPC_DEBUG=1 P2P_FUZZ_DEVICE=0 P2P_IPC_POOL=1G P2P_FUZZ_TIMEOUT=15 timeout -k 10 90 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port $((30000 + RANDOM % 1000)) tests/scripts/fuzz_session.py ipc:relay "${1:-15}" \
  > gpurun_out/rd2/relay.out 2> gpurun_out/rd2/relay.err
echo "rc=$?" > gpurun_out/rd2/rc.txt
