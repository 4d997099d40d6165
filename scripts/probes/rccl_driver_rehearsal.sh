# The driver's exact bench command (defaults, --steps 20 --warmup 5) at N = 2 and 4, every rank on one MI355X and
# RCCL between them over its socket transport (P2P_RCCL_DISTINCT_HOSTS=1): every section of the node run, through
# real RCCL, within the deadline. Output in gpurun_out/drv/.
set -o pipefail
mkdir -p gpurun_out/drv
export P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
for N in 2 4; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29930 + N)) bench.py --gpus $N --steps 20 --warmup 5 --device 0 \
    > gpurun_out/drv/n$N.json 2> gpurun_out/drv/n$N.err || exit 1
done
