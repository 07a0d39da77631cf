# round-3 checkpoint: the whole -m gpu suite (one process), then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_gpu_tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
rc=$?; tail -3 gpurun_out/r3_bench.err; exit $rc
