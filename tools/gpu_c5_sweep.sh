# C5 mixed-size storm: heap slots per origin x mover count (what bounds it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -c "
import sys, json, ctypes
sys.argv=['bench']
import bench
sys.path.insert(0, bench.PKG)
import rlo
lib = rlo.abi.load(); st = ctypes.c_void_p(); lib.rlo_stream_create(0, ctypes.byref(st))
red = lambda x, op: x
for slots, movers in ((2, 192), (4, 192), (2, 64), (2, 32)):
    r = bench.c5_leg(rlo, None, 1, 0, 0, st, red, bulk_slots=slots, movers=movers, steps=2)
    print(json.dumps({k: r[k] for k in ('bulk_slots', 'movers_per_part', 'kernel_ms', 'bcast_per_s', 'delivered_GBps', 'frac', 'verified')}), flush=True)
" > gpurun_out/c5_sweep.jsonl 2> gpurun_out/c5_sweep.err || { echo "rc=$?"; tail gpurun_out/c5_sweep.err; exit 1; }
cat gpurun_out/c5_sweep.jsonl
