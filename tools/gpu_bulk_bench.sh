# bench legs of the bulk path only (C3 latency rounds, C5 mixed storm) + the bulk parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bulk.py -x -q --timeout 150 --timeout-method thread > gpurun_out/bulk_tests.log 2>&1 || { echo "bulk tests rc=$?"; tail -20 gpurun_out/bulk_tests.log; exit 1; }
tail -2 gpurun_out/bulk_tests.log
timeout -k 10 300 python3 -u -c "
import sys, json, ctypes, os
sys.argv=['bench']
import bench
sys.path.insert(0, bench.PKG)
import rlo
lib = rlo.abi.load(); st = ctypes.c_void_p(); lib.rlo_stream_create(0, ctypes.byref(st))
red = lambda x, op: x
print(json.dumps(bench.bulk_leg(rlo, None, 1, 0, 0, st, red)))
print(json.dumps(bench.c5_leg(rlo, None, 1, 0, 0, st, red)))
" > gpurun_out/bulk_bench.json 2> gpurun_out/bulk_bench.err || { echo "bench rc=$?"; tail gpurun_out/bulk_bench.err; exit 1; }
cat gpurun_out/bulk_bench.json
