# RCCL with several ranks on ONE MI355X: every rank claims a host of its own (P2P_RCCL_DISTINCT_HOSTS=1 sets
# NCCL_HOSTID per rank), so RCCL accepts ranks that share the GPU and connects them through its socket network
# transport on loopback. Not an xGMI measurement: it runs bench.py's and p2p_matrix's multi-rank RCCL paths
# (communicator candidates 1/2/4/8, tournament rounds, ring, all-pairs, ring token chain, latency matrix, pair
# sweep, reference-method matrix, verification of every timed delivery) through real RCCL where only one GPU
# exists. Sizes are cut to what loopback sockets move in seconds. Run on the box; output in gpurun_out/rccl_emu/.
set -o pipefail
mkdir -p gpurun_out/rccl_emu
export P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
N=${1:-4}
timeout -k 10 150 /opt/conda/bin/mpirun -n $N ./build/p2p_matrix --device 0 --mode pair,tournament,ring,allpairs \
  --size 4M -n 4 --verify --latency --latency-iters 50 --no-compat --timeout 60 \
  > gpurun_out/rccl_emu/cli_n$N.txt 2>&1 &&
timeout -k 10 150 /opt/conda/bin/mpirun -n $N ./build/p2p_matrix --device 0 --comms 4 --mode tournament,ring,allpairs \
  --size 4M -n 4 --verify --no-compat --timeout 60 > gpurun_out/rccl_emu/cli_n${N}_k4.txt 2>&1 &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port $((29870 + N)) bench.py --gpus $N --device 0 --size 4M --msgs 8 --sweep-max 64M --allpairs-size 64M \
  --ring-size 16M --ref-iters 16 --latency-iters 50 --ipc-extra 0 --timeout 60 --deadline 380 \
  --json-out gpurun_out/rccl_emu/bench_n$N.json > /dev/null 2> gpurun_out/rccl_emu/bench_n$N.err
