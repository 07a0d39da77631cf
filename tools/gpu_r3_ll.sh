set -o pipefail
mkdir -p gpurun_out
echo "== doorbells on"; timeout -k 10 120 python3 tools/lat_quick.py 4 8 64 256 2>&1 | tee gpurun_out/r3_lat_ll.txt || exit 1
echo "== doorbells off (diag lib)"; RLO_DIAG_LIB=1 RLO_NO_LL=1 timeout -k 10 120 python3 tools/lat_quick.py 4 8 64 256 2>&1 | tee gpurun_out/r3_lat_noll.txt || exit 1
echo "== storm A/B"; timeout -k 10 200 python3 tools/storm_ab.py 2>&1 | tee gpurun_out/r3_storm_ab.txt || exit 1
RLO_LIB_DIR=lib_ab timeout -k 10 200 python3 tools/storm_ab.py 2>&1 | tee -a gpurun_out/r3_storm_ab.txt || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_gpu_tests.log | tail -25
exit $rc
