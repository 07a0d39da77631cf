"""Where the hop kernel's rounds go (rlo_hop.hip kHopProf, diagnostics build): per rank, shader clocks per section of a
round -- poll + re-polls, bells, publish, slot loads, votes, loaded messages, originations, bookkeeping -- and the
event counts (rounds, re-polls, bell takes, slot takes, votes merged, refusals, originations, busy rounds), for the
latency program and one-proposal decisions (C4).
    python tools/hop_anatomy.py [n ...]"""
import os
import sys
import time

import numpy as np

os.environ.setdefault("RLO_DIAG_LIB", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

SEC = ["poll", "bells", "publish", "loads", "votes", "slots", "own", "books"]
CNT = ["rounds", "repolls", "bell_takes", "slot_takes", "votes", "refused", "originated", "busy"]


def show(tag, st, units, unit_name):
    prof = st["prof"].astype(np.float64)
    cnt = st["dbg"].astype(np.float64)
    tot = prof.sum(axis=1)
    print("  %s: kernel cycles per rank (median) %.0f; per %s:" % (tag, np.median(tot), unit_name), flush=True)
    print("    sections  " + " ".join("%9s" % s for s in SEC))
    print("    median    " + " ".join("%9.0f" % v for v in np.median(prof, axis=0) / units))
    print("    max rank  " + " ".join("%9.0f" % v for v in prof[np.argmax(tot)] / units))
    print("    counts    " + " ".join("%9s" % s for s in CNT))
    print("    median    " + " ".join("%9.2f" % v for v in np.median(cnt, axis=0) / units), flush=True)
    tk = st["hist"][:, -4:].astype(np.float64)  # a take's clocks: checks, forward, effects; takes
    ntk = np.maximum(tk[:, 3], 1)
    pre = st["hist"][:, -5].astype(np.float64)  # of the checks: entry -> the child set's computation
    print("    per take (median over ranks): checks %.0f (header / pending / judge %.0f) forward %.0f effects %.0f cycles"
          " (%.1f takes per %s)" % (np.median(tk[:, 0] / ntk), np.median(pre / ntk), np.median(tk[:, 1] / ntk),
                                    np.median(tk[:, 2] / ntk), np.median(tk[:, 3]) / units, unit_name), flush=True)


for n in [int(x) for x in (sys.argv[1:] or ["8"])]:
    with rlo.World(n, max_payload=64) as w:
        rounds = 2000
        w.program_latency(rounds, 64, seed=21)
        w.run()
        st = w.stats()
        lat = w.latencies_ticks().astype(np.float64) * 0.01
        assert (st["error"] == 0).all(), st["error"]
        print("n %d latency: p50 %.2f p99 %.2f us, last kernel %d" % (n, np.percentile(lat, 50), np.percentile(lat, 99),
                                                                        w.info_now()["last_kernel"]), flush=True)
        show("latency", st, rounds, "round")
        p = 64
        w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(p) for r in range(n)])
        w.run()
        ms = w.run()
        st = w.stats()
        assert (st["error"] == 0).all(), st["error"]
        print("n %d iar: %.0f decisions/s (%.2f us per decision of one rank), last kernel %d" % (
            n, n * p / (ms * 1e-3), ms * 1e3 / p, w.info_now()["last_kernel"]), flush=True)
        show("iar", st, p, "decision of one rank")
