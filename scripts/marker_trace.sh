# rocprofv3 marker + kernel trace of p2p_matrix with P2P_ROCTX=1 (roctx ranges around every timed phase) and the
# engine's own Chrome trace (--trace). Run on the MI355X box; output in gpurun_out/marker/.
set -o pipefail
export TMPDIR=/tmp && mkdir -p gpurun_out/marker
export P2P_ROCTX=1
# RCCL's own roctx ranges around its API calls (ncclSend / ncclRecv / ncclGroupEnd), next to the engine's phases.
export RCCL_LOG_ROCTX=1
timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/marker -o m -- \
  ./build/p2p_matrix --mode self --sizes 4M,64M -n 8 --verify --no-compat --trace gpurun_out/marker/chrome_trace.json \
  > gpurun_out/marker/stdout.txt 2> gpurun_out/marker/stderr.txt
