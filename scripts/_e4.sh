mkdir -p gpurun_out/e4
rm -f gpurun_out/e4/*
P2P_IPC_POOL=1G P2P_FUZZ_DEVICE=0 P2P_FUZZ_TIMEOUT=20 timeout -k 5 45 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29564 tests/scripts/step_probe.py ipc:push tournament 32M 8 5 6 > gpurun_out/e4/d5.log 2>&1 &&
P2P_IPC_POOL=1G timeout -k 10 170 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 4 --steps 14 --warmup 7 --transport ipc --device 0 --sweep-max 64M --latency-iters 100 --deadline 160 --isolate 1 > gpurun_out/e4/bench.json 2> gpurun_out/e4/bench.err
