# Closing GPU evidence of round 3 on the MI355X box: the GPU tier, smoke and bench (scripts/gpu_check.sh),
# then rocprofv3 kernel stats and counters (scripts/profile.sh, its own passes). Output: gpurun_out/r3b_close/.
set -o pipefail
mkdir -p gpurun_out/r3b_close
bash scripts/gpu_check.sh && cp gpurun_out/s2/* gpurun_out/r3b_close/ && \
bash scripts/profile.sh gpurun_out/r3b_close/prof > gpurun_out/r3b_close/profile.log 2>&1
