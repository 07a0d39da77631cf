# bulk-message GPU tests (device programs, then the drop-in extension), then a regression slice of
# the engine tests; each step time-limited, stop at the first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bulk.py -x -v --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/bulk_tests.log 2>&1 && \
if [ -z "$BULK_ONLY" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 150 --timeout-method thread -k "bulk or stream or parents" > gpurun_out/dropin_bulk_tests.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/engine_tests.log 2>&1
fi
