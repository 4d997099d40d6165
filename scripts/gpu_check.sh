# GPU tier, smoke, then the 1-GPU bench (run on the MI355X box). Extra args go to pytest.
set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 900 python -u -m pytest tests -m gpu "$@" -x -v --timeout 300 --timeout-method thread --durations=25 > gpurun_out/s2/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err
