#!/bin/bash
# Round-3 evidence on one MI355X (each step time-limited; a fault, abort,
# crash or time limit ends the script, exit statuses 0-3 are results):
#   1. bench.py with 4 RCCL ranks on the one GPU (distinct hosts to RCCL, so its
#      NET transport): provenance.rccl_peers / matrix_transport per pair;
#   2. scripts/probes/chunk_cost.sh: one op vs 32 MiB ops on the self path;
#   3. scripts/probes/unroll_probe.sh: RCCL_UNROLL_FACTOR on the 1-GPU bench.
#   bash scripts/probes/r3_evidence.sh [out_dir]
O=${1:-gpurun_out/r3_evidence}
mkdir -p "$O"
: > "$O/status.txt"
exec 3>&1
step() {  # step <name> <ok codes regex> <cmd...>
  local name=$1 ok=$2
  shift 2
  "$@"
  local rc=$?
  # (the step's own redirections cover this function's output: report on fd 3)
  echo "$name rc=$rc" >> "$O/status.txt"
  echo "$name rc=$rc" >&3
  if ! [[ $rc =~ ^($ok)$ ]]; then
    echo "stopping after $name (rc=$rc)" >> "$O/status.txt"
    echo "stopping after $name (rc=$rc)" >&3
    exit "$rc"
  fi
}
PORT=$((20000 + RANDOM % 10000))
step emu4_bench "0|3" env P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 timeout -k 10 300 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $PORT \
  bench.py --gpus 4 --device 0 --size 4M --msgs 8 --sweep-max 64M --allpairs-size 64M --ring-size 16M \
  --ref-iters 16 --latency-iters 30 --ipc-extra 0 --timeout 60 --json-out "$O/emu4_bench.json" \
  > "$O/emu4_bench.out" 2> "$O/emu4_bench.err"
step chunk_cost "0" bash scripts/probes/chunk_cost.sh "$O/chunk_cost"
step unroll "0" bash scripts/probes/unroll_probe.sh "$O/unroll"
