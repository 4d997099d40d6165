#!/bin/bash
# Everything this framework measures on a multi-GPU MI355X node, in one command, each step time-limited and the
# first failure ending the run (the GPUs are never driven again after a fault):
#
#   1. the multi-GPU test tier (tests/test_multi_gpu.py: RCCL across GPUs in every mode, 4 communicators, the IPC
#      engines across xGMI, fuzz);
#   2. the reference's own run line, `mpirun -n N ./p2p_matrix` (compat matrices, result.txt);
#   3. the headline bench at N = 1, 2, 4, 8 and its scaling table (scripts/scaling.sh);
#   4. the xGMI pair-cell tuning sweep (scripts/xgmi_pair_sweep.py);
#   5. the framework-free RCCL reproducers across two GPUs: scripts/rccl_half_repro.cpp --devices 2 (where RCCL's
#      lost-second-half threshold lies on a real xGMI link, with RCCL's INFO log of the 2-GPU communicator), and
#      scripts/rccl_net_repro.cpp as two MPI ranks on GPUs 0 and 1 with RCCL's defaults and with
#      NCCL_NCHANNELS_PER_PEER=8 (which loses half of every message over RCCL's socket transport,
#      profiles/r4_node_rehearsal/).
#
#   bash scripts/node_run.sh [OUT_DIR] [--dry-run] [--rehearse]
#
# --rehearse runs the same steps on a one-GPU box, with 4 ranks on device 0, each rank its own RCCL host (RCCL's
# socket transport, not xGMI), benches at 32 messages per step under a 150 s deadline, the pair sweep emulated
# through RCCL, and no 2-GPU reproducer: it checks this script's steps end to end before a node run.
set -uo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/node
DRY=0
REHEARSE=0
for a in "$@"; do
  case "$a" in
    --dry-run) DRY=1 ;;
    --rehearse) REHEARSE=1 ;;
    *) OUT=$a ;;
  esac
done
MPIRUN=${P2P_MPIRUN:-/opt/conda/bin/mpirun}
NGPU=$(python3 -c "import torch; print(torch.cuda.device_count())")
N=$(( NGPU < 8 ? NGPU : 8 ))
[ "$DRY" = 1 ] && [ "$N" -lt 2 ] && N=8  # show the node commands anywhere
SWEEP_EMULATE=()
BENCH_EXTRA=()
if [ "$REHEARSE" = 1 ]; then
  N=4
  export P2P_REHEARSE_MULTI_GPU=$N P2P_DEVICE=0 P2P_FUZZ_DEVICE=0 P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo \
    NCCL_IB_DISABLE=1 P2P_SCALING_GPUS=$N
  SWEEP_EMULATE=(--emulate rccl --sizes 32M)
  BENCH_EXTRA=(--msgs 32 --deadline 150)
fi

step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "== $name (limit ${secs}s): $*"
  [ "$DRY" = 1 ] && return 0
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/summary.txt"
  if [ $rc -ne 0 ]; then
    echo "node_run: $name failed (rc=$rc); stopping, see $OUT/$name.log" >&2
    exit $rc
  fi
}

if [ "$N" -lt 2 ] && [ "$DRY" = 0 ] && [ "$REHEARSE" = 0 ]; then
  echo "node_run: needs >= 2 visible GPUs (found $NGPU); on one GPU use scripts/gpu_check.sh," \
       "scripts/emulated_node.sh and scripts/rccl_emulated_node.sh, or --rehearse" >&2
  exit 1
fi
mkdir -p "$OUT"
if [ "$DRY" = 0 ]; then
  make -j16 all > "$OUT/build.log" 2>&1 || { echo "node_run: build failed, see $OUT/build.log" >&2; exit 1; }
fi
step multi_gpu_tests 1800 python3 -u -m pytest tests/test_multi_gpu.py -m gpu -x -v --timeout 900 --timeout-method thread
step reference_run 600 "$MPIRUN" -n "$N" ./p2p_matrix --json "$OUT/reference_run.json"
[ "$DRY" = 0 ] && cp "$OUT/reference_run.log" "$OUT/result.txt"
step scaling 3600 bash scripts/scaling.sh "$OUT/scaling.jsonl" "${BENCH_EXTRA[@]}"
# (exit 2 = some row's bytes failed verification: a finding listed in
# xgmi_sweep/summary.json corrupt_rows, never a winner; the run goes on)
step pair_sweep 1200 bash -c 'python3 scripts/xgmi_pair_sweep.py "$@"; rc=$?; [ $rc -eq 2 ] && exit 0; exit $rc' _ \
  --np "$N" --out "$OUT/xgmi_sweep" "${SWEEP_EMULATE[@]}"
if [ "$REHEARSE" = 1 ]; then
  [ "$DRY" = 0 ] && cat "$OUT/summary.txt"
  exit 0
fi
# (exit 3 = some size came back wrong: a finding, not a failure of the step)
step rccl_repro_2gpu 300 env NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,P2P NCCL_DEBUG_FILE="$OUT/rccl_repro_2gpu.nccl.txt" \
  bash -c './build/rccl_half_repro --devices 2 --sizes 16M,32M,64M,128M,256M,512M,1G,1G+16; rc=$?; [ $rc -eq 3 ] && exit 0; exit $rc'
# (exit 3 = some message came back wrong: a finding, not a failure of the step)
for pp in default 8; do
  step "rccl_pair_repro_pp$pp" 300 env $([ "$pp" = default ] || echo NCCL_NCHANNELS_PER_PEER=$pp) NCCL_DEBUG=INFO \
    NCCL_DEBUG_SUBSYS=INIT,P2P NCCL_DEBUG_FILE="$OUT/rccl_pair_repro_pp$pp.nccl.%p.txt" \
    bash -c '"$0" -n 2 ./build/rccl_net_repro --sizes 1M,32M,1G --iters 2; rc=$?; [ $rc -eq 3 ] && exit 0; exit $rc' "$MPIRUN"
done
[ "$DRY" = 0 ] && cat "$OUT/summary.txt"
exit 0
