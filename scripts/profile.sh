#!/bin/bash
# rocprofv3 profiles of the flagship paths (run on the MI355X box, from the repo root).
# Kernel-trace/stats and PMC counters run in SEPARATE invocations (gpurun refuses
# --pmc together with the trace domains).  Outputs land in ${1:-gpurun_out/prof}/*;
# copy the summaries worth keeping into profiles/.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
# 1) kernel trace + stats of the bench (RCCL kernels + fill/verify)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench -- \
    python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_stdout.txt"
# 2) kernel trace + stats of the kernel microbench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kernels" -o kernels -- \
    python3 scripts/kernel_bench.py --sizes 256M,1G --reps 5 > "$OUT/kernels_stdout.txt"
# 3) counters on the kernel microbench (own pass): HBM bytes + LDS behaviour
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv \
    -d "$OUT/pmc_fetch" -o pmc -- python3 scripts/kernel_bench.py --sizes 1G --reps 2 > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_INSTS_VMEM_RD --kernel-trace --output-format csv \
    -d "$OUT/pmc_write" -o pmc -- python3 scripts/kernel_bench.py --sizes 1G --reps 2 > /dev/null
# 4) kernel trace + stats of the hand-written data plane (one process: IPC copy
#    kernel on the self path, device ping-pong kernel, fill / verify)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ipc" -o ipc -- \
    ./build/p2p_matrix --transport ipc --mode self --sizes 32M,1G -n 16 --verify --device-latency \
    --latency-iters 2000 --no-compat > "$OUT/ipc_stdout.txt"
echo "profiles done"
