# Round-4 probe: the pair-sweep row NCCL_NCHANNELS_PER_PEER=8 lost half of every
# 32 MiB message between ranks on RCCL's socket transport (4 ranks on one GPU,
# node_run.sh --rehearse).  Re-run that cell at 8 iterations with RCCL's log
# kept, at 32 MiB and 16 MiB, with and without the knob; record the links
# record (op limits, channels connected) and the verification.
O=${1:-gpurun_out/r4_pp8}
mkdir -p "$O/tmp"
export P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 P2P_RCCL_LOG=keep TMPDIR="$PWD/$O/tmp"
run() {  # name, env..., -- args
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 120 env "${envs[@]}" /opt/conda/bin/mpirun -n 4 build/p2p_matrix --mode pair --cells 0-1 --dir both \
    -n 8 --no-compat --json "$O/$name.json" --timeout 60 --transport rccl --comms 1 --device 0 "$@" \
    > "$O/$name.txt" 2> "$O/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -le 3 ] || exit $rc  # a crash or time limit ends the probe
}
if [ "${2:-}" = "rule" ]; then
  # Which knob values lose data: per-peer channels vs the p2p channel count
  # (4 by default on the socket transport).
  run pp4_32m NCCL_NCHANNELS_PER_PEER=4 -- --sizes 32M
  run pp8_min8_32m NCCL_NCHANNELS_PER_PEER=8 NCCL_MIN_P2P_NCHANNELS=8 -- --sizes 32M
  run pp8_1m NCCL_NCHANNELS_PER_PEER=8 -- --sizes 1M
  run pp16_min8_32m NCCL_NCHANNELS_PER_PEER=16 NCCL_MIN_P2P_NCHANNELS=8 -- --sizes 32M
  exit 0
fi
run pp8_32m NCCL_NCHANNELS_PER_PEER=8 -- --sizes 32M
run pp8_16m NCCL_NCHANNELS_PER_PEER=8 -- --sizes 16M
run pp8_32m_norechunk NCCL_NCHANNELS_PER_PEER=8 P2P_RECHUNK=0 -- --sizes 32M
run default_32m P2P_RCCL_UNROLL=4 -- --sizes 32M
exit 0
