# GPU parity + smoke + bench, each step under its own time limit, stop at the first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
if [ -n "$RUN_BENCH" ]; then timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1; fi
