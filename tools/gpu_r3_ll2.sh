set -o pipefail
mkdir -p gpurun_out
echo "== doorbell pass v2"; timeout -k 10 120 python3 tools/lat_quick.py 4 8 64 256 2>&1 | tee gpurun_out/r3_lat_ll2.txt || exit 1
echo "== bulk"; timeout -k 10 120 python3 tools/bulk_quick.py 2>&1 | tee gpurun_out/r3_bulk_quick.txt || exit 1
echo "== drop-in api"; timeout -k 10 300 python3 tools/api_quick.py 2>&1 | tee gpurun_out/r3_api_quick.txt || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_gpu_tests2.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_gpu_tests2.log | tail -25
exit $rc
