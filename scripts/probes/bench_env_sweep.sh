#!/bin/bash
# Runs bench.py (1 GPU) under several RCCL channel settings; one JSON line per
# config into gpurun_out/bench_env/<name>.json.  Each run is time-limited.
set -o pipefail
mkdir -p gpurun_out/bench_env
run() {
  name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 28 --warmup 7 > gpurun_out/bench_env/$name.json 2> gpurun_out/bench_env/$name.err
}
run default P2P_NOOP=1 &&
run pp64 NCCL_NCHANNELS_PER_PEER=64 NCCL_MIN_P2P_NCHANNELS=64 NCCL_MAX_P2P_NCHANNELS=64 &&
run all64 NCCL_NCHANNELS_PER_PEER=64 NCCL_MIN_P2P_NCHANNELS=64 NCCL_MAX_P2P_NCHANNELS=64 NCCL_MIN_NCHANNELS=64 NCCL_MAX_NCHANNELS=64 &&
run all128 NCCL_NCHANNELS_PER_PEER=128 NCCL_MIN_P2P_NCHANNELS=128 NCCL_MAX_P2P_NCHANNELS=128 NCCL_MIN_NCHANNELS=128 NCCL_MAX_NCHANNELS=128 &&
run simple64 NCCL_PROTO=Simple NCCL_NCHANNELS_PER_PEER=64 NCCL_MIN_P2P_NCHANNELS=64 NCCL_MAX_P2P_NCHANNELS=64 NCCL_MIN_NCHANNELS=64 NCCL_MAX_NCHANNELS=64
