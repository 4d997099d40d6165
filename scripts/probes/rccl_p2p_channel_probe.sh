#!/bin/bash
# RCCL self send/recv under NCCL_MAX_P2P_NCHANNELS = 1 / 2 / 4 / 64, through build/p2p_matrix (--verify) at 1 and 4
# communicators and 1 MiB .. 256 MiB messages: which settings deliver every byte.  A run that delivers wrong
# bytes exits 2 and the probe goes on; any other failure ends it.  Output: gpurun_out/p2p_ch/.
set -uo pipefail
mkdir -p gpurun_out/p2p_ch
for nch in 64 1 2 4; do
  for k in 1 4; do
    name=nch${nch}_k${k}
    NCCL_MAX_P2P_NCHANNELS=$nch timeout -k 10 120 ./build/p2p_matrix --bootstrap local --mode self --sizes 1M,32M,256M \
      -n 16 --verify --no-compat --comms $k --json gpurun_out/p2p_ch/$name.json > gpurun_out/p2p_ch/$name.txt 2>&1
    rc=$?
    echo "$name rc=$rc" >> gpurun_out/p2p_ch/summary.txt
    if [ $rc -ne 0 ] && [ $rc -ne 2 ]; then exit $rc; fi
  done
done
exit 0
