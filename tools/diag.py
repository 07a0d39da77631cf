#!/usr/bin/env python3
"""Diagnostic: per-phase cycle split of the progress kernel (MODE_PROF build path) + batch sizes."""
import argparse, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import numpy as np
import rlo

# prof[] slots in the kernel's stamp order: 0 poll (+drain), 1 stage (LDS-DMA + vote loads), 2 classify,
# 3 admit, 4 effects, 5 copy, 6 consume (bookkeeping + eager publish), 7 select
PH = ["poll", "stage", "classify", "admit", "effects", "copy", "consume", "select"]


def report(name, w, ms, deliveries):
    st = w.stats()
    it = st["iterations"].astype(np.float64)
    busy = st["busy_iterations"].astype(np.float64)
    prof = st["prof"].astype(np.float64)
    cyc_per_it = prof.sum(axis=0)[:8] / it.sum()
    print("%-28s kernel %.3f ms | iters/rank %.0f busy %.0f | deliveries/busy-iter %.1f | stalls/rank %.0f | err %d"
          % (name, ms, it.mean(), busy.mean(), deliveries / max(busy.sum(), 1), st["stalls"].mean(), st["error"].max()))
    print("   cycles/iter: " + "  ".join("%s %.0f" % (p, c) for p, c in zip(PH, cyc_per_it)) + "  | total %.0f" % cyc_per_it.sum())
    dur = (st["t_end"].astype(np.float64) - st["t_start"].min()) * 0.01
    print("   per-rank end us p0/p50/p100 %.0f/%.0f/%.0f | busy p0/p50/p100 %d/%d/%d | stalls max %d at rank %d"
          % (dur.min(), np.median(dur), dur.max(), busy.min(), np.median(busy), busy.max(), st["stalls"].max(),
             int(np.argmax(st["stalls"]))))
    dbg = st["dbg"].astype(np.float64)
    for r in sorted(set([0, 1, 2, 128, 255, int(np.argmax(st["stalls"]))])):
        d = dbg[r]
        print("   rank %3d: iters %d busy %d | ring cands %.0f admitted %.0f | storm-allowed iters %.0f | "
              "large rounds: drain cycles %.0f, rounds (push) / relay-full pushes (pull) %.0f (%.0f cycles/round) | "
              "backlog %.0f | child copies %.0f | max out fill %.0f"
              % (r, st["iterations"][r], st["busy_iterations"][r], d[0], d[1], d[2], d[3], d[4], d[3] / max(d[4], 1),
                 d[5], d[6], d[7]))
        h = st["hist"][r].astype(np.float64)
        it_r = max(1, st["iterations"][r])
        print("            per out-ring (oi: misfits/iter, admitted/iter, free@start/iter): " + " ".join(
            "%d:%.1f/%.1f/%.0f" % (o, h[o] / it_r, h[32 + o] / it_r, 16 * h[64 + o] / it_r) for o in range(32) if h[32 + o] or h[o]))
        pr = st["prof"][r].astype(np.float64) / max(1, st["iterations"][r])
        print("            cycles/iter: " + "  ".join("%s %.0f" % (p, c) for p, c in zip(PH, pr)))
    sys.stdout.flush()


ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--k", type=int, default=1 << 18)
ap.add_argument("--lens", default="64,4096", help="storm payload sizes")
ap.add_argument("--storm-only", action="store_true")
args = ap.parse_args()
for ln in [int(x) for x in args.lens.split(",")]:
    win = 64 if ln <= 1024 else 32
    w = rlo.World(args.n, max_payload=max(64, ln))
    k = args.k if ln <= 1024 else args.k // 8
    w.program_storm(k, ln, window=win)
    ms0 = w.run()
    w.program_storm(k, ln, window=win, prof=True)
    ms = w.run()
    report("storm len=%d win=%d (%.0f/s)" % (ln, win, k / ms0 * 1e3), w, ms, k * (args.n - 1))
    w.close()
if args.storm_only:
    sys.exit(0)
w = rlo.World(args.n)
p = 32
props = [(r, it * args.n + r, b"0123456789abcdef") for it in range(p) for r in range(args.n)]
w.program_iar(props, prof=True)
ms = w.run()
report("iar p=%d (%.0f dec/s)" % (p, args.n * p / ms * 1e3), w, ms, args.n * p * (args.n - 1) * 2)
w.program_latency(200, 64)
ms = w.run()
lat = w.latencies_ticks() * 0.01
print("latency p50 %.1f us p99 %.1f us" % (np.percentile(lat, 50), np.percentile(lat, 99)))
