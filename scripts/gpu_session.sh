#!/bin/bash
# One GPU visit: the GPU tests that cover this round's changes, a 4-rank RCCL
# run on one GPU (NET transport, RCCL INFO logs kept), and the 1-GPU bench.
# Every step has its own time limit; a fault, abort, crash or time limit ends
# the script there (exit statuses 0-3 are results, anything else is not).
#   bash scripts/gpu_session.sh [out_dir] [pytest files...]
O=${1:-gpurun_out/session}
shift
TESTS=${*:-tests/test_rccl_gpu.py tests/test_binary_gpu.py tests/test_ipc_gpu.py}
mkdir -p "$O/tmp"
export P2P_TEST_LOG_DIR="$PWD/$O/testlogs"  # long bench runs inside tests stream their progress here
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
step pytest "0|1" timeout -k 10 900 python -u -m pytest --maxfail 5 -v --timeout 300 --timeout-method thread $TESTS -m gpu \
  > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
step emu4 "0|2|3" env P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 TMPDIR="$PWD/$O/tmp" \
  P2P_RCCL_LOG=keep timeout -k 10 180 /opt/conda/bin/mpirun -n 4 build/p2p_matrix --device 0 --mode pair,allpairs \
  --size 64M -n 4 --verify --json "$O/emu4.json" --timeout 60 > "$O/emu4.txt" 2> "$O/emu4.err"
step bench "0|3" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
