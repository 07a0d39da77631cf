#!/bin/bash
# Quick GPU loop for kernel changes: device-program parity tests, then the storm / latency / decisions
# bench legs, then the fresh-world logged-storm stress.  bash tools/gpu_quick.sh [tag]
set -e -o pipefail
T=${1:-q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_sharded.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 200 python bench.py --no-pmc --no-api --no-bulk --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 240 python -u tools/stress_storm_logged.py --fresh --reps 40 > gpurun_out/${T}_ss.log 2>&1
