#!/bin/bash
# N back-to-back 1-GPU bench runs (default 8) plus one rocprofv3 kernel-stats
# run of the bench, on a GPU box from the repo root.  Output: gpurun_out/soak/.
set -o pipefail
mkdir -p gpurun_out/soak
for i in $(seq 1 "${1:-8}"); do
  timeout -k 10 200 python bench.py > gpurun_out/soak/bench_$i.json 2> gpurun_out/soak/bench_$i.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/soak/prof -o run -- \
  python3 bench.py --steps 20 --warmup 6 > gpurun_out/soak/bench_prof.json 2> gpurun_out/soak/bench_prof.err
