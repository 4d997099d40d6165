#!/bin/bash
# bench.py (1 GPU) with 4 RCCL communicators under RCCL channel / protocol knobs; one JSON line per config into
# gpurun_out/bench_env_k4/<name>.json.  Each run is time-limited.
set -o pipefail
mkdir -p gpurun_out/bench_env_k4
run() {
  name=$1; shift
  env "$@" timeout -k 10 150 python bench.py --comms 4 --ipc-extra 0 --ref-iters 0 --latency-iters 100 \
    > gpurun_out/bench_env_k4/$name.json 2> gpurun_out/bench_env_k4/$name.err
}
run default_a P2P_NOOP=1 &&
run pp8 NCCL_NCHANNELS_PER_PEER=8 &&
run pp16 NCCL_NCHANNELS_PER_PEER=16 &&
run maxp2p16 NCCL_MAX_P2P_NCHANNELS=16 &&
run batch RCCL_P2P_BATCH_ENABLE=1 &&
run memcpy NCCL_P2P_USE_CUDA_MEMCPY=1 &&
run simple NCCL_PROTO=Simple &&
run default_b P2P_NOOP=1
