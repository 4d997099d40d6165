set -uo pipefail
mkdir -p gpurun_out/p2p_ch2
for spec in "1 8M,16M,24M" "2 32M,48M" "4 64M,96M" "8 128M,160M"; do
  set -- $spec
  nch=$1; sizes=$2
  P2P_RCCL_MAX_CHUNK=0 NCCL_MAX_P2P_NCHANNELS=$nch timeout -k 10 120 ./build/p2p_matrix --bootstrap local --mode self \
    --sizes $sizes -n 8 --verify --no-compat --json gpurun_out/p2p_ch2/nch$nch.json > gpurun_out/p2p_ch2/nch$nch.txt 2>&1
  rc=$?; echo "nch$nch rc=$rc" >> gpurun_out/p2p_ch2/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 2 ]; then exit $rc; fi
done
P2P_RCCL_MAX_CHUNK=16M timeout -k 10 150 python bench.py --comms 4 --ipc-extra 0 --ref-iters 0 > gpurun_out/p2p_ch2/bench_chunk16m.json 2> gpurun_out/p2p_ch2/bench_chunk16m.err &&
timeout -k 10 150 python bench.py --comms 4 --ipc-extra 0 --ref-iters 0 > gpurun_out/p2p_ch2/bench_default.json 2> gpurun_out/p2p_ch2/bench_default.err &&
P2P_RCCL_MAX_CHUNK=16M timeout -k 10 150 python bench.py --comms 4 --ipc-extra 0 --ref-iters 0 > gpurun_out/p2p_ch2/bench_chunk16m_b.json 2> gpurun_out/p2p_ch2/bench_chunk16m_b.err
