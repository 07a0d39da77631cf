"""Diagnostic: device-only decisions (approve-all, 8 ranks on the GPU, no host in the loop) launched
repeatedly -- if these times swing like the drop-in's, the GPU (scheduling) is the cause, else the
host side is.  Usage: python tools/probe_erratic.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n, p = 8, 2000
with rlo.World(n, max_payload=64, device=0) as w:
    w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(p) for r in range(n)])
    for i in range(reps):
        t = time.perf_counter()
        ms = w.run()
        dt = time.perf_counter() - t
        st = w.stats()
        print("device iar n=%d p=%d: %.3f s wall, kernel %.3f ms, decided %d" % (n, p, dt, ms, int(st["own_decided"].sum())),
              flush=True)
