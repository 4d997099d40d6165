O=gpurun_out/emu8
mkdir -p $O
P2P_IPC_POOL=1G timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 8 --steps 14 --warmup 7 --transport ipc --device 0 --sweep-max 64M --latency-iters 100 --deadline 360 --isolate 0 > $O/b.json 2> $O/b.err
echo "rc=$?" >> $O/b.err
