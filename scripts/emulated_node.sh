# bench.py at N = 8 and 4 with every rank on one MI355X (IPC transport): the N-rank code paths of the
# driver's multi-GPU run, on one GPU. N = 8 runs its comparisons in-process (8 + 8 processes would hit the box's
# 16-process limit).
set -o pipefail
mkdir -p gpurun_out/emu
export P2P_IPC_POOL=2G
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 8 --transport ipc --device 0 --sweep-max 1G --isolate 0 --json-out gpurun_out/emu/bench_ipc_n8.json > gpurun_out/emu/n8.out 2> gpurun_out/emu/n8.err && \
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 4 --transport ipc --device 0 --sweep-max 1G --json-out gpurun_out/emu/bench_ipc_n4.json > gpurun_out/emu/n4.out 2> gpurun_out/emu/n4.err
