# Round 4: build/rccl_net_repro (raw HIP + RCCL + MPI, no framework code) on
# the configurations of profiles/r4_node_rehearsal/: two ranks on GPU 0, each
# its own RCCL host (socket transport), with RCCL's default channels, with
# NCCL_NCHANNELS_PER_PEER=8 (p2p_matrix lost half of every message), and with
# that plus NCCL_MIN_P2P_NCHANNELS=8 (p2p_matrix verified).
O=${1:-gpurun_out/r4_net_repro}
mkdir -p "$O"
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT
run() {  # name, env assignments..., --
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 120 env "${envs[@]}" NCCL_DEBUG_FILE="$PWD/$O/$name.nccl.%h.%p.txt" /opt/conda/bin/mpirun -n 2 \
    build/rccl_net_repro --distinct-hosts --device 0 --sizes 1M,32M --iters 2 > "$O/$name.json" 2> "$O/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -le 3 ] || exit $rc  # a crash or time limit ends the probe
}
run default P2P_PROBE=1 --
run per_peer8 NCCL_NCHANNELS_PER_PEER=8 --
run per_peer8_min8 NCCL_NCHANNELS_PER_PEER=8 NCCL_MIN_P2P_NCHANNELS=8 --
exit 0
