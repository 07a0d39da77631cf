# lone-message fast path: device parity suites, then latency / decisions with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_sharded.py tests/test_gpu_host.py tests/test_gpu_bulk.py -x -q --timeout 150 --timeout-method thread > gpurun_out/fast_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/fast_tests.log; exit 1; }
tail -1 gpurun_out/fast_tests.log
for n in 4 8 64 256; do timeout -k 5 60 python3 tools/lat_anatomy.py --n $n --rounds 400 2>/dev/null | head -1 || exit 1; done
RLO_NO_FAST=1 timeout -k 5 60 python3 tools/lat_anatomy.py --n 8 --rounds 400 2>/dev/null | head -1
timeout -k 10 120 python3 -c "
import sys, json, ctypes
sys.argv=['bench']
import bench
sys.path.insert(0, bench.PKG)
import rlo
lib = rlo.abi.load(); st = ctypes.c_void_p(); lib.rlo_stream_create(0, ctypes.byref(st))
print(json.dumps(bench.small_n_legs(rlo, 0, st)))
" 2>/dev/null
