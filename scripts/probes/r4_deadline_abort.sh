# Round 4: bench.py's deadline watchdog while RCCL is busy.  The 8-rank
# rehearsal (profiles/r4_rehearsal/) hit the deadline during the posting
# tuning and 3 of 8 ranks died with SIGSEGV: the watchdog thread aborted the
# communicators while the main thread was inside RCCL.  Now the watchdog only
# requests the abort and the transports' waits perform it on their own
# thread.  Same situation here: 4 ranks on one GPU over RCCL's socket
# transport, 128 x 32 MiB per step, a 25 s deadline that lands in the tuning.
O=${1:-gpurun_out/r4_deadline}
mkdir -p "$O"
export P2P_RCCL_DISTINCT_HOSTS=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 4 --device 0 --deadline 25 --timeout 60 --ipc-extra 0 \
  > "$O/bench.json" 2> "$O/bench.err"
rc=$?
echo "torchrun rc=$rc"
grep -c "Signal 11" "$O/bench.err" | sed 's/^/SIGSEGV lines: /'
grep -E "exitcode|aborted|deadline" "$O/bench.err" | head -20
cat "$O/bench.json"
[ $rc -le 3 ] || [ $rc -eq 1 ] || exit $rc
exit 0
