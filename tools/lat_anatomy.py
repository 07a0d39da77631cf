"""Per-phase shader cycles of BUSY iterations in the latency program (one bcast at a time):
what one hop costs besides memory round trips.  python tools/lat_anatomy.py [--n 256]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

PH = ["poll", "votes+stage", "classify", "admit", "effects", "copy", "consume", "select(C)+bar"]
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--rounds", type=int, default=200)
a = ap.parse_args()
with rlo.World(a.n, max_payload=64) as w:
    w.program_latency(a.rounds, 64)
    w.run()
    lat = w.latencies_ticks() * 0.01
    w.program_latency(a.rounds, 64, prof=True)
    ms = w.run()
    latp = w.latencies_ticks() * 0.01
    st = w.stats()
it = st["iterations"].astype(np.float64).sum()
busy = st["busy_iterations"].astype(np.float64).sum()
prof = st["prof"].astype(np.float64).sum(axis=0)
print("n %d: latency p50 %.1f us (prof build %.1f us); iterations %.0f, busy %.0f; kernel %.1f ms" %
      (a.n, np.percentile(lat, 50), np.percentile(latp, 50), it, busy, ms))
print("cycles per iteration (all): " + "  ".join("%s %.0f" % (p, c / it) for p, c in zip(PH, prof[:8])))
print("cycles per BUSY iteration (phases 1-5 only run when busy): " +
      "  ".join("%s %.0f" % (p, prof[i] / busy) for i, p in enumerate(PH[:6]) if i >= 1))
print("us per iteration (wall) %.3f" % (ms * 1e3 / (it / a.n)))
