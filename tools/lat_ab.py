"""A/B of the latency program and one-proposal decisions between this tree's library and an older build kept
under tools/ab_libs/<name>/ (its rlo package + lib/): python tools/lat_ab.py <name> [n ...].  Alternates the
two builds in one process per leg so box noise hits both."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import rlo
n = int(sys.argv[2])
with rlo.World(n, max_payload=64) as w:
    w.program_latency(2000, 64, seed=21)
    w.run()
    lat = w.latencies_ticks().astype(np.float64) * 0.01
    w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(64) for r in range(n)])
    w.run()
    ms = w.run()
    print("%.2f %.2f %.0f" % (np.percentile(lat, 50), np.percentile(lat, 99), n * 64 / (ms * 1e-3)))
'''
name = sys.argv[1]
builds = {"head": os.path.join(REPO, "rootless-coll-mpi-ops_amd"), name: os.path.join(REPO, "tools", "ab_libs", name)}
for n in [int(x) for x in (sys.argv[2:] or ["4", "8", "256"])]:
    for rep in range(2):
        for tag, path in builds.items():
            out = subprocess.run([sys.executable, "-c", CHILD, path, str(n)], capture_output=True, text=True, timeout=120)
            print("n %4d %-8s rep %d: p50 / p99 us, decisions/s = %s %s" % (n, tag, rep, out.stdout.strip(), out.stderr.strip()[-200:]),
                  flush=True)
