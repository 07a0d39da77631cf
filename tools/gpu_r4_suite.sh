# round-4 evidence, call 1: the whole -m gpu suite (one process), then the default bench line
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r4/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r4/gpu_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 560 python3 -u bench.py > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err || { tail -20 gpurun_out/r4/bench.err; exit 1; }
tail -3 gpurun_out/r4/bench.err
