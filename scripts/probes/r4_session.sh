# Round 4 GPU visit: the GPU tier, then the 1-GPU bench four times alternating
# RCCL's private INFO log on (default) and off (P2P_RCCL_LOG=0) -- the A/B of
# the log's cost to the headline -- then the bench under
# rocprofv3 --kernel-trace --stats (the post-timing verify's launch counts).
# A crash, abort or time limit ends the script (exit statuses 0-3 are results).
O=${1:-gpurun_out/r4_session}
mkdir -p "$O"
ok() { [ "$1" -le 3 ] || { echo "stopping: rc=$1"; exit "$1"; }; }
bash scripts/gpu_tier.sh "$O/tier"; ok $?
for i in 1 2; do
  timeout -k 10 300 python bench.py > "$O/bench_default_$i.json" 2> "$O/bench_default_$i.err"; ok $?
  P2P_RCCL_LOG=0 timeout -k 10 300 python bench.py > "$O/bench_log0_$i.json" 2> "$O/bench_log0_$i.err"; ok $?
done
# The post-timing verification one buffer at a time (round 3's way), for
# verify_detail.seconds against the batched default above.
P2P_VERIFY_BATCH=0 timeout -k 10 300 python bench.py > "$O/bench_verify_unbatched.json" 2> "$O/bench_verify_unbatched.err"; ok $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench -- \
  python3 bench.py --steps 20 --warmup 5 > "$O/prof_bench.json" 2> "$O/prof_bench.err"; ok $?
echo "session done"
