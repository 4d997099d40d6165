#!/bin/bash
# bench.py (1 GPU) under RCCL's p2p-channel knobs around RCCL's defaults (64 p2p channels, 128 per peer, read from
# the NCCL_DEBUG=INFO run), at 4 communicators and, for the 128-channel setting, at 1 and 2.  One JSON line per
# config into gpurun_out/bench_env_ch/<name>.json.  Each run is time-limited.
set -o pipefail
mkdir -p gpurun_out/bench_env_ch
run() {
  name=$1; comms=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --comms "$comms" --ipc-extra 0 --ref-iters 0 --latency-iters 100 \
    > gpurun_out/bench_env_ch/$name.json 2> gpurun_out/bench_env_ch/$name.err
}
run default_info 4 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,P2P,TUNING &&
run pp32 4 NCCL_NCHANNELS_PER_PEER=32 &&
run pp64 4 NCCL_NCHANNELS_PER_PEER=64 NCCL_MAX_P2P_NCHANNELS=64 &&
run minp2p32 4 NCCL_MIN_P2P_NCHANNELS=32 &&
run minp2p64 4 NCCL_MIN_P2P_NCHANNELS=64 NCCL_MAX_P2P_NCHANNELS=64 &&
run maxnch64 4 NCCL_MAX_NCHANNELS=64 &&
run p2p128_k4 4 NCCL_MIN_P2P_NCHANNELS=128 NCCL_MAX_P2P_NCHANNELS=128 &&
run p2p128_k2 2 NCCL_MIN_P2P_NCHANNELS=128 NCCL_MAX_P2P_NCHANNELS=128 &&
run p2p128_k1 1 NCCL_MIN_P2P_NCHANNELS=128 NCCL_MAX_P2P_NCHANNELS=128 &&
run p2p128_k2_info 2 NCCL_MIN_P2P_NCHANNELS=128 NCCL_MAX_P2P_NCHANNELS=128 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT &&
run default_k1 1 P2P_NOOP=1 &&
run default_b 4 P2P_NOOP=1
