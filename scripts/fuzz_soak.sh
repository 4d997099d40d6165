# Data-integrity soak on one MI355X: long --fuzz runs (random verified message groups) through every engine that
# runs on one GPU. Each run is time-limited; the first failure ends the script. Logs in gpurun_out/fuzz_soak/.
set -o pipefail
mkdir -p gpurun_out/fuzz_soak
N=${1:-2000}
export P2P_IPC_POOL=1G
run() {
  name=$1; shift
  echo "== $name" >> gpurun_out/fuzz_soak/summary.txt
  timeout -k 10 300 "$@" > gpurun_out/fuzz_soak/$name.txt 2>&1 || { echo "FAILED rc=$?" >> gpurun_out/fuzz_soak/summary.txt; exit 1; }
  grep -E "groups of random|verified|mismatch" gpurun_out/fuzz_soak/$name.txt | tail -2 >> gpurun_out/fuzz_soak/summary.txt
}
run rccl_k1 ./build/p2p_matrix --mode self --size 64M -n 2 --fuzz $N --no-compat &&
run rccl_k4 ./build/p2p_matrix --mode self --size 64M -n 2 --comms 4 --fuzz $N --no-compat &&
run ipc_kernel_4 /opt/conda/bin/mpirun -n 4 ./build/p2p_matrix --transport ipc --device 0 --size 16M -n 2 --fuzz $N --no-compat &&
run ipc_push_4 /opt/conda/bin/mpirun -n 4 ./build/p2p_matrix --transport ipc --ipc-engine push --device 0 --size 16M -n 2 --fuzz $N --no-compat &&
run ipc_relay_4 /opt/conda/bin/mpirun -n 4 ./build/p2p_matrix --transport ipc --ipc-engine relay --device 0 --size 16M -n 2 --fuzz $N --no-compat &&
run ipc_relay_8 /opt/conda/bin/mpirun -n 8 ./build/p2p_matrix --transport ipc --ipc-engine relay --device 0 --size 16M -n 2 --fuzz $((N / 4)) --no-compat
