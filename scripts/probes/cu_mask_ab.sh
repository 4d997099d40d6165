# A/B on one MI355X: RCCL self step with 4 communicators, their streams unmasked (default) or each owning 1/4 of
# the CUs (P2P_RCCL_CU_MASK=contig|stride), interleaved, $1 reps.  Run on the box; results in gpurun_out/cu_mask/.
set -o pipefail
mkdir -p gpurun_out/cu_mask
for rep in $(seq 1 "${1:-2}"); do
  for m in none contig stride; do
    if [ "$m" = none ]; then unset P2P_RCCL_CU_MASK; else export P2P_RCCL_CU_MASK=$m; fi
    timeout -k 10 200 python bench.py --comms 4 --ipc-extra 0 --ref-iters 0 --latency-iters 100 \
      > gpurun_out/cu_mask/${m}_${rep}.json 2> gpurun_out/cu_mask/${m}_${rep}.err || exit 1
  done
done
unset P2P_RCCL_CU_MASK
