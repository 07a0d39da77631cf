# host-service doorbell pass: drop-in + host-mode parity first, then the drop-in API bench and the device latency probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_dropin.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r3_host_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_host_tests.log | tail -15; [ $rc -eq 0 ] || exit $rc
echo "== drop-in api"; timeout -k 10 300 python3 tools/api_quick.py 2>&1 | tee gpurun_out/r3_api_host_ll.txt || exit 1
echo "== device latency"; timeout -k 10 120 python3 tools/lat_quick.py 4 8 256 2>&1 | tee gpurun_out/r3_lat_host_ll.txt
echo "== host-service latency anatomy"; for n in 4 8; do timeout -k 10 120 python3 tools/host_latency.py --n $n --rounds 400 || exit 1; done 2>&1 | tee gpurun_out/r3_host_latency.txt
