"""Where a doorbell hop's instructions go (diagnostics build, RLO_HOP_PROF): shader clocks (s_memtime) at points
of every doorbell pass that took exactly one ring message, summed per segment over the latency program's hops.
    python tools/hop_prof.py [n ...] [--host]   (RLO_DIAG_LIB=1 and RLO_HOP_PROF=1 are set here; --host: the drop-in's
    host service, one bcast at a time).  The host kernels carried the stamps during round 5's analysis (DESIGN.md
    section 4.1.1); with the scalar doorbell poll they no longer fit the host kernel's registers, so --host now reports
    no profiled hops unless the kPmHost condition is put back into the kernel's HP macro (diagnostics build)."""
import os
import sys

import numpy as np

os.environ["RLO_DIAG_LIB"] = "1"
os.environ["RLO_HOP_PROF"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

SEG = ["pass entry -> bells checked", "-> votes / commands done", "-> ring loop at the message", "-> lone(): checks",
       "-> forwards (fwd_small)", "-> effects", "-> pass drained", "-> counters published"]
HOST = "--host" in sys.argv  # the drop-in's host service instead: its world shape, one bcast at a time, polled here


def host_run(n, rounds=500):
    """one bcast at a time through the host service (the drop-in's world: 32 KiB slots, 128-slot rings, bulk
    messages on), every rank's events polled here; device origination -> pickup record from the events"""
    lat = []
    with rlo.HostWorld(n, max_payload=32768, ring_slots=128, bulk_max=64 << 20, movers=4) as hw:
        for i in range(rounds):
            hw.bcast(i % n, b"x" * 64, seq=i)
            got, dmax = 0, 0
            while got < n - 1:
                for r in range(n):
                    for ev in hw.poll(r):
                        got += 1
                        dmax = max(dmax, ev["aux"])
            lat.append(dmax * 0.01)
    return hw.final_stats, np.asarray(lat), 0.0


for n in [int(x) for x in (a for a in sys.argv[1:] if not a.startswith("--"))] or [8, 256]:
    if HOST:
        st, lat, ms = host_run(n)
    else:
        with rlo.World(n, max_payload=64) as w:
            w.program_latency(2000, 64, seed=21)
            ms = w.run()
            st = w.stats()
            lat = w.latencies_ticks().astype(np.float64) * 0.01
    hops = float(st["dbg"][:, 0].astype(np.float64).sum())
    prof = st["prof"].astype(np.float64).sum(axis=0)
    print("n %d%s: p50 %.2f us (profiled build), %d hops profiled, kernel %.1f ms" % (n, " host service" if HOST else "",
                                                                                    np.percentile(lat, 50), hops, ms))
    tot = 0.0
    for k, name in enumerate(SEG):
        c = prof[k] / max(hops, 1.0)
        tot += c
        print("   %-32s %7.0f cycles" % (name, c))
    print("   %-32s %7.0f cycles" % ("total", tot), flush=True)
