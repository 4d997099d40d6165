#!/bin/bash
# Runs the framework-free RCCL half-delivery reproducer (scripts/rccl_half_repro.cpp)
# over the VERDICT r2 cases, on both RCCLs of the image, one GPU:
#   NCCL_MAX_P2P_NCHANNELS=1 at 16 / 24 MiB, default channels at 1 GiB / 1 GiB + 16,
#   plus controls (the same bytes as two ops; memset pattern; Simple protocol)
#   and an INFO log of the self connection's channels.
# Exit 0 / 3 from the binary means "ran" (3: some delivery was wrong); anything
# else (fault, abort, time limit) ends the script at once.
#
#   make tools && bash scripts/probes/rccl_half_repro.sh [out_dir]
set -u
OUT=${1:-gpurun_out/half_repro}
mkdir -p "$OUT"
run() {  # run <name> <binary> [env...] -- args...
  local name=$1 bin=$2
  shift 2
  local envs=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  echo "== $name: ${envs[*]} $bin $*" | tee -a "$OUT/summary.log"
  env "${envs[@]}" timeout -k 10 90 "$bin" "$@" > "$OUT/$name.log" 2> "$OUT/$name.err"
  local rc=$?
  cat "$OUT/$name.log" >> "$OUT/summary.log"
  echo "rc=$rc" >> "$OUT/summary.log"
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then
    echo "stopping: $name exited $rc" | tee -a "$OUT/summary.log"
    tail -20 "$OUT/$name.err"
    exit $rc
  fi
}
: > "$OUT/summary.log"
for v in torch rocm; do
  bin=build/rccl_half_repro
  [ $v = rocm ] && bin=build/rccl_half_repro_rocm
  run ${v}_nch1 $bin NCCL_MAX_P2P_NCHANNELS=1 -- --sizes 16M,24M,32M
  run ${v}_nch1_memset $bin NCCL_MAX_P2P_NCHANNELS=1 -- --sizes 16M,24M --memset
  run ${v}_nch1_two_ops $bin NCCL_MAX_P2P_NCHANNELS=1 -- --sizes 24M,32M --ops 2
  run ${v}_nch1_simple $bin NCCL_MAX_P2P_NCHANNELS=1 NCCL_PROTO=Simple -- --sizes 24M
  run ${v}_nch2 $bin NCCL_MAX_P2P_NCHANNELS=2 -- --sizes 32M,48M
  run ${v}_default $bin P2P_UNUSED=1 -- --sizes 1G,1G+16 --iters 2
  run ${v}_default_two_ops $bin P2P_UNUSED=1 -- --sizes 1G+16,2G --ops 2
done
# RCCL's own account of the self connection: channels and transport.
run torch_info build/rccl_half_repro NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,P2P NCCL_DEBUG_FILE=$OUT/torch_info.nccl.%p.txt -- --sizes 1G+16
run torch_info_nch1 build/rccl_half_repro NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,P2P NCCL_MAX_P2P_NCHANNELS=1 NCCL_DEBUG_FILE=$OUT/torch_info_nch1.nccl.%p.txt -- --sizes 24M
echo "done" | tee -a "$OUT/summary.log"
