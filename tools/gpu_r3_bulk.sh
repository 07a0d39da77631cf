# bulk path: parity first (bulk + C5 tests, the drop-in bulk stream), then the mover sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bulk.py tests/test_gpu_dropin.py -k "bulk or c5 or Bulk" -x -v --timeout 150 --timeout-method thread > gpurun_out/r3_bulk_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_bulk_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 tools/bulk_probe.py 128,0 1,4,16,64 2>&1 | tee gpurun_out/r3_bulk_probe3.txt
