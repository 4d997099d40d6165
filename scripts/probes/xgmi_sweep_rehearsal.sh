#!/bin/bash
# bench.py's xGMI pair sweep section (--xgmi-sweep) rehearsed on one MI355X:
#   1. the GPU test that runs it emulated through the IPC engines (2 ranks on GPU 0);
#   2. the driver's N = 2 bench with both ranks on GPU 0 through real RCCL (each rank claims a host of its own,
#      P2P_RCCL_DISTINCT_HOSTS=1, so RCCL links them over loopback sockets), the sweep forced on: every RCCL
#      communicator / knob row and IPC row the node run would do, within the time the deadline leaves.
# Output: gpurun_out/xsw/.
set -o pipefail
mkdir -p gpurun_out/xsw
timeout -k 10 400 python -u -m pytest tests/test_ipc_gpu.py -k "two_ranks_ipc_push" -x -v --timeout 380 \
  --timeout-method thread > gpurun_out/xsw/pytest.log 2>&1 && \
P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port $((24000 + RANDOM % 4000)) bench.py --gpus 2 --steps 14 --warmup 7 --device 0 \
  --xgmi-sweep 1 --xgmi-sweep-sizes "${1:-32M}" \
  > gpurun_out/xsw/bench_rccl_n2.json 2> gpurun_out/xsw/bench_rccl_n2.err
