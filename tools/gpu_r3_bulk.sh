# bulk path parity: one part (direct plan), two parts / processes, the chunked (multi-GPU) plan rehearsed on
# one GPU, the drop-in bulk stream, the storm engine tests; then the bulk probe and the ring-depth probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bulk.py tests/test_gpu_engine.py tests/test_gpu_dropin.py -k "bulk or c5 or storm or pulled" -x -v --timeout 150 --timeout-method thread > gpurun_out/r3_bulk_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_bulk_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 tools/bulk_probe.py 0 16k,1,4,16,64 2,8 2>&1 | tee gpurun_out/r3_bulk_probe13.txt || exit 1
