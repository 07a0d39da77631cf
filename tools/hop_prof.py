"""Where a doorbell hop's instructions go (diagnostics build, RLO_HOP_PROF): shader clocks (s_memtime) at points
of every doorbell pass that took exactly one ring message, summed per segment over the latency program's hops.
    python tools/hop_prof.py [n ...]   (RLO_DIAG_LIB=1 and RLO_HOP_PROF=1 are set here)"""
import os
import sys

import numpy as np

os.environ["RLO_DIAG_LIB"] = "1"
os.environ["RLO_HOP_PROF"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

SEG = ["pass entry -> bells checked", "-> votes / commands done", "-> ring loop at the message", "-> lone(): checks",
       "-> effects", "-> forwards (fwd_small)", "-> pass drained", "-> counters published"]
for n in [int(x) for x in (sys.argv[1:] or ["8", "256"])]:
    with rlo.World(n, max_payload=64) as w:
        w.program_latency(2000, 64, seed=21)
        ms = w.run()
        st = w.stats()
        lat = w.latencies_ticks().astype(np.float64) * 0.01
    hops = float(st["dbg"][:, 0].astype(np.float64).sum())
    prof = st["prof"].astype(np.float64).sum(axis=0)
    print("n %d: p50 %.2f us (profiled build), %d hops profiled, kernel %.1f ms" % (n, np.percentile(lat, 50), hops, ms))
    tot = 0.0
    for k, name in enumerate(SEG):
        c = prof[k] / max(hops, 1.0)
        tot += c
        print("   %-32s %7.0f cycles" % (name, c))
    print("   %-32s %7.0f cycles" % ("total", tot), flush=True)
