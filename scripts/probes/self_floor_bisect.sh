# Which earlier tests slow the GPU tier's 4-communicator self-step floor?
# (~1800-1970 GB/s inside the tier against 2230-2450 in a fresh
# process, profiles/r5_tier1/.)  The floor test after each test file alone,
# every run in a fresh pytest process.
O=${1:-gpurun_out/floor_bisect}
mkdir -p "$O"
FLOOR=tests/test_zz_perf_floors_gpu.py::test_self_copy_rate_floors
for f in none tests/test_kernels_gpu.py tests/test_kernels_properties_gpu.py tests/test_rccl_gpu.py \
         tests/test_ipc_gpu.py tests/test_rccl_ranks_gpu.py tests/test_binary_gpu.py tests/test_examples.py; do
  name=$(basename "$f" .py)
  [ "$f" = none ] && f=""
  timeout -k 10 400 python -m pytest -q -p no:cacheprovider -m gpu --timeout 300 --timeout-method thread $f "$FLOOR" \
    > "$O/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(grep '^PERF' "$O/$name.log")"
  [ $rc -le 1 ] || exit $rc
done
