# The driver's GPU tier on one MI355X box (`pytest -m gpu -x`, conftest's
# order: correctness, multi-GPU, perf floors last), with per-test progress,
# the 30 slowest durations and the perf floors' per-launch record under
# $OUT/testlogs/perf_floors.json; then, only if the tier ended without a
# crash or time limit (rc 0 or 1), the fill grid-shape probe.
#   bash scripts/gpu_tier.sh [out_dir]
OUT=${1:-gpurun_out/tier}
mkdir -p "$OUT"
export P2P_TEST_LOG_DIR="$PWD/$OUT/testlogs"
timeout -k 10 950 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=30 \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 60 build/fill_probe 1 > "$OUT/fill_probe.txt" 2>&1
echo "fill_probe rc=$?"
exit $rc
