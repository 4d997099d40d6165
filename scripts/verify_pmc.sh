#!/bin/bash
# rocprofv3 counters of the two verify stagings on one 1 GiB buffer
# (VERDICT r5 item 3): occupancy (SQ_WAVE_CYCLES over GRBM_GUI_ACTIVE), how
# much of each wave's life is spent waiting (SQ_WAIT_INST_ANY, SQ_WAIT_ANY),
# VALU / LDS activity, and HBM bytes.  One rocprofv3 pass per counter group
# (the hardware's per-block limits), each its own short process.  Outputs
# under ${1:-gpurun_out/verify_pmc}; summary via scripts/summarize_pmc.py.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/verify_pmc}
mkdir -p "$OUT"
PROG=(python3 scripts/verify_ab.py --sizes 1G --rounds 2 --reps 3 --grids 2048)
pass() {
  local name=$1
  shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o pmc -- \
      "${PROG[@]}" > "$OUT/$name.stdout" 2>&1
}
pass occupancy SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE
pass valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD
pass fetch FETCH_SIZE TA_BUSY_avr
python3 scripts/summarize_pmc.py $(find "$OUT" -name '*counter_collection.csv') > "$OUT/summary.txt"
echo "verify pmc done"
