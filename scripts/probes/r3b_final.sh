# GPU tier, smoke and bench (scripts/gpu_check.sh), then four driver-shaped bench runs (run on the MI355X box).
set -o pipefail
mkdir -p gpurun_out/r3b_final/repeat
bash scripts/gpu_check.sh && cp gpurun_out/s2/* gpurun_out/r3b_final/ || exit $?
for i in 1 2 3 4; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_final/repeat/bench_$i.json 2> gpurun_out/r3b_final/repeat/bench_$i.err || exit $?
done
