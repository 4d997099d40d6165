#!/bin/bash
# 8-byte RCCL latency (bench.py's host-posted and pre-posted p50, 1 GPU) under runtime / RCCL knobs that act on
# small-message cost: kernel arguments in device memory, RCCL's protocol, thread count and channel count.  One
# JSON line per config into gpurun_out/lat_knobs/<name>.json.  Each run is time-limited.
set -o pipefail
mkdir -p gpurun_out/lat_knobs
run() {
  name=$1; shift
  env "$@" timeout -k 10 150 python bench.py --ipc-extra 0 --ref-iters 0 --latency-iters 2000 \
    > gpurun_out/lat_knobs/$name.json 2> gpurun_out/lat_knobs/$name.err
}
run default_a P2P_NOOP=1 &&
run dev_kernarg HIP_FORCE_DEV_KERNARG=1 &&
run proto_ll NCCL_PROTO=LL &&
run nthreads64 NCCL_NTHREADS=64 &&
run nthreads128 NCCL_NTHREADS=128 &&
run p2p_nch1 NCCL_MAX_P2P_NCHANNELS=1 &&
run dev_kernarg_ll HIP_FORCE_DEV_KERNARG=1 NCCL_PROTO=LL &&
run default_b P2P_NOOP=1
