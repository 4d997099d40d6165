# Relay pair cell 0 -> 1 (32 MiB, 16 iterations, verified) with 4 and 8 ranks on one GPU, at the box's default
# hardware queues per process and at 1: does the 8-rank slowdown of the emulated node come from more queues than
# the hardware scheduler maps at once (profiles/r2_emulated/README.md)?  Run on the MI355X box.
set -o pipefail
mkdir -p gpurun_out/relay_probe
export P2P_IPC_POOL=1G
if [ "${1:-}" != bench ]; then
for n in 4 8; do
  for q in default 1; do
    if [ "$q" = default ]; then unset GPU_MAX_HW_QUEUES; else export GPU_MAX_HW_QUEUES=$q; fi
    echo "== ranks $n hwq $q" >> gpurun_out/relay_probe/summary.txt
    timeout -k 10 120 /opt/conda/bin/mpirun -n $n ./build/p2p_matrix --transport ipc --ipc-engine relay --device 0 \
      --mode pair --dir uni --cells 0:1 --size 32M -n 16 --verify --no-compat --timeout 60 \
      > gpurun_out/relay_probe/r${n}_q${q}.txt 2>&1 || exit 1
    grep -E "GB/s|verification|  0 " gpurun_out/relay_probe/r${n}_q${q}.txt | head -12 >> gpurun_out/relay_probe/summary.txt
  done
done
fi
unset GPU_MAX_HW_QUEUES
# Part 2: the relay engine as bench.py's timed transport, 8 ranks on one GPU (each rank a torch process), at the
# default hardware queues per process and at 2 (8 x 2 = 16 queues in all).
if [ "${1:-}" = bench ]; then
  for q in default 2; do
    if [ "$q" = default ]; then unset GPU_MAX_HW_QUEUES; else export GPU_MAX_HW_QUEUES=$q; fi
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port $((29770 + ${#q})) bench.py --gpus 8 --transport ipc:relay --device 0 --ipc-extra 0 --extras 0 --sweep 0 \
      --ref-iters 0 --steps 14 --warmup 7 > gpurun_out/relay_probe/bench_relay_q$q.json 2> gpurun_out/relay_probe/bench_relay_q$q.err || exit 1
  done
fi
