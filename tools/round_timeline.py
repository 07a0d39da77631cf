"""Where a latency round's time goes (RLO_FLAG_TIMELINE): per round the device clock of the origination, the
scatter job's post / claim / completion-count adds (bulk), every rank's arrival (message or bulk announcement)
and bulk completion, the round's last pickup, and the start of the next round; medians over rounds, in us
after the origination.  One GPU, one part.
    python tools/round_timeline.py [--n 8] [--sizes 64,16384,1048576] [--rounds 64]"""
import argparse
import os
import sys

import numpy as np

os.environ.setdefault("RLO_DIAG_LIB", "1")  # RLO_FLAG_TIMELINE: the diagnostics build (make DIAG=1 -> lib_diag/)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--sizes", default="64,16384,1048576")
ap.add_argument("--rounds", type=int, default=64)
ap.add_argument("--bulk-max", type=int, default=64 << 20)
ap.add_argument("--dump", type=int, default=0, help="print this many rounds' per-rank clocks")
a = ap.parse_args()


def rel(t, t0):
    """clock difference in us (32-bit wrap), NaN where the event was not seen"""
    d = ((t.astype(np.int64) - t0.astype(np.int64)) + (1 << 31)) % (1 << 32) - (1 << 31)
    return np.where(t == 0, np.nan, d * 0.01)


sizes = [int(x) for x in a.sizes.split(",")]
nl = a.n
for ln in sizes:
    # ring-slot sizes in a world without bulk messages (the latency bench's), larger ones as bulk messages
    with (rlo.World(a.n, max_payload=max(64, ln)) if ln <= 112 else
          rlo.World(a.n, max_payload=64, bulk_max=a.bulk_max)) as w:
        w.program_latency(a.rounds, ln, seed=0x7100 + ln, timeline=True)
        kms = w.run()
        st = w.stats()
        assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
        tl = w.timeline()
        t0 = tl[:, 0]
        g = {k: rel(tl[:, i], t0) for i, k in enumerate(["origin", "posted", "claimed", "moved", "round", "verified", "gen", "drained"])}
        arr = rel(tl[:, 8:8 + nl], t0[:, None])
        comp = rel(tl[:, 8 + nl:8 + 2 * nl], t0[:, None])
        par = tl[:, 8 + 2 * nl:8 + 3 * nl].astype(np.int64) - 1
        iss = rel(tl[:, 8 + 3 * nl:8 + 4 * nl], t0[:, None])
        pas = rel(tl[:, 8 + 4 * nl:8 + 5 * nl], t0[:, None])
        fwdb = rel(tl[:, 8 + 5 * nl:8 + 6 * nl], t0[:, None])
        nxts = rel(tl[:, 8 + 6 * nl:8 + 7 * nl], t0[:, None])
        p1 = rel(tl[:, 8 + 7 * nl:8 + 8 * nl], t0[:, None])
        p2 = rel(tl[:, 8 + 8 * nl:8 + 9 * nl], t0[:, None])
        nxt = np.append(rel(tl[1:, 0], tl[:-1, 4]), np.nan)  # this round's last pickup -> next origination
        per = np.append(rel(tl[1:, 0], tl[:-1, 0]), np.nan)
        sl = slice(2, None)  # the first rounds warm the caches
        md = lambda x: float(np.nanmedian(x[sl])) if np.isfinite(x[sl]).any() else float("nan")  # noqa: E731
        line = "n %d len %8d: round %6.2f us | posted %5.2f claimed %5.2f gen %5.2f drained %5.2f moved %5.2f | arrival med %5.2f max %5.2f" % (
            a.n, ln, md(per), md(g["posted"]), md(g["claimed"]), md(g["gen"]), md(g["drained"]), md(g["moved"]), md(np.nanmedian(arr, axis=1)),
            md(np.nanmax(arr, axis=1)))
        if ln > 112 and np.isfinite(comp).any():
            line += " | completion med %5.2f max %5.2f" % (md(np.nanmedian(comp, axis=1)), md(np.nanmax(comp, axis=1)))
            # per receiver: the last poll that found its copy incomplete, the one that found it complete
            line += " [complete poll issued med %5.2f, its loads back med %5.2f]" % (
                md(np.nanmedian(iss, axis=1)), md(np.nanmedian(pas, axis=1)))
        elif np.isfinite(comp).any():
            # per hop: parent's forwards issued (the origin: its origination) -> child's doorbell pass took it;
            # per rank: took it -> its own forwards issued
            hop, proc, wait, rtt, pre, pa, pb, l1, l2, l3 = [], [], [], [], [], [], [], [], [], []
            for r in range(2, len(tl)):
                for c in range(nl):
                    p = par[r, c]
                    if p < 0 or not np.isfinite(arr[r, c]):
                        continue
                    sent = 0.0 if np.isnan(arr[r, p]) else comp[r, p]  # (the origin takes nothing: its origination)
                    if np.isfinite(sent):
                        hop.append(arr[r, c] - sent)
                        if np.isfinite(iss[r, c]) and 0 <= pas[r, c] - iss[r, c] < 20:  # (taken by the doorbell pass)
                            wait.append(iss[r, c] - sent)
                            rtt.append(pas[r, c] - iss[r, c])
                            pre.append(arr[r, c] - pas[r, c])
                            pa.append(fwdb[r, c] - pas[r, c])
                            pb.append(nxts[r, c] - fwdb[r, c])
                    if np.isfinite(comp[r, c]):
                        proc.append(comp[r, c] - arr[r, c])
                        l1.append(p1[r, c] - arr[r, c])
                        l2.append(p2[r, c] - p1[r, c])
                        l3.append(comp[r, c] - p2[r, c])
            if hop:
                line += " | hop med %5.2f p90 %5.2f, take->forwarded med %5.2f (%d hops)" % (
                    np.median(hop), np.percentile(hop, 90), np.median(proc) if proc else np.nan, len(hop))
            if l1:
                line += " [take: checks %5.2f, effects %5.2f, forwards %5.2f]" % (np.median(l1), np.median(l2), np.median(l3))
            if wait:
                line += " [sent -> poll issued %5.2f, poll -> pass %5.2f, pass -> taken %5.2f (preamble %5.2f, to the ring loop %5.2f); %d]" % (
                    np.median(wait), np.median(rtt), np.median(pre), np.median(pa), np.median(pb), len(wait))
        line += " | last pickup %5.2f -> next origin +%5.2f | verified %5.2f" % (md(g["round"]), md(nxt), md(g["verified"]))
        line += " | kernel %.2f us per round" % (kms * 1e3 / a.rounds)
        print(line, flush=True)
        for r in range(2, 2 + a.dump):
            print("    round %d: origin %d, posted %.2f claimed %.2f moved %.2f round %.2f" % (
                r, int(np.argmax(np.isnan(arr[r]))), g["posted"][r], g["claimed"][r], g["moved"][r], g["round"][r]))
            for c in range(nl):
                print("      rank %3d parent %3d: arrival %6.2f  poll %6.2f  pass/complete-poll %6.2f  done %6.2f"
                      "  fwd %6.2f  next-spin %6.2f" % (
                          c, par[r, c], arr[r, c], iss[r, c], pas[r, c], comp[r, c],
                          fwdb[r, c], nxts[r, c]))
        why = st["dbg"][:, :7].astype(np.int64)  # wave 0's spin exits (rlo_kernel.hip SPIN_WHY)
        print("    spin exits over ranks: not-idle %d bound %d need-full %d 64-passes %d posts %d bulk-done %d moved %d;"
              " iterations %d (%.1f per round per rank)" % (*why.sum(axis=0), int(st["iterations"].sum()),
                                                            st["iterations"].sum() / a.rounds / nl), flush=True)
