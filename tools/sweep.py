#!/usr/bin/env python3
"""Sweep storm throughput over ring capacity and origination window (diagnostic)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo

n, k = 256, 1 << 18
lens = tuple(int(x) for x in sys.argv[1:]) or (64, 4096)
for ln in lens:
    for slots in (256, 512, 1024, 2048, 4096):
        if ln >= 4096 and slots > 1024:
            continue
        try:
            w = rlo.World(n, max_payload=ln, ring_slots=slots)
        except Exception as e:
            print(ln, slots, e); continue
        for win in ((32, 64) if ln > 64 else (8, 16, 32, 64)):
            kk = k if ln <= 1024 else k // 8
            w.program_storm(kk, ln, window=win)
            ms = min(w.run() for _ in range(2))
            print("len %5d slots %5d win %3d: %8.0f bcast/s  %.2f ms" % (ln, slots, win, kk / ms * 1e3, ms), flush=True)
        w.close()
