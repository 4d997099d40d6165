#!/bin/bash
# A/B of the timing-mark event flags (csrc/hip_check.hpp timing_event_flags):
# the 1-GPU bench through RCCL and through the IPC pull engine, with marks
# that skip the system-scope fence (default) and with default events
# (P2P_MARK_FENCE=system), interleaved; plus a kernel trace of each IPC run.
set -o pipefail
out=gpurun_out/mark_fence
mkdir -p $out
for rep in 1 2; do
  for fence in none system; do
    for tr in rccl ipc; do
      env_fence=""; [ $fence = system ] && env_fence=system
      P2P_MARK_FENCE=$env_fence timeout -k 10 200 python bench.py --transport $tr --ipc-extra 0 --steps 20 --warmup 5 \
        > $out/${tr}_${fence}_$rep.json 2> $out/${tr}_${fence}_$rep.err || exit $?
      python -c "import json; r=json.load(open('$out/${tr}_${fence}_$rep.json')); print('$tr fence=$fence rep $rep: value %.1f device %.1f ms/step %.4f verify %s' % (r['value'], r['matrix_gbs_mean'], r['ms_per_step'], r['verify_mismatches']))"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for fence in none system; do
  env_fence=""; [ $fence = system ] && env_fence=system
  P2P_MARK_FENCE=$env_fence timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace_$fence -o run -- \
    python3 bench.py --transport ipc --ipc-extra 0 --steps 20 --warmup 5 > /dev/null 2> $out/trace_$fence.err || exit $?
done
