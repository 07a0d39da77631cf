"""C3 probe (one GPU, 8 ranks): bulk round time vs mover count, to tell a bandwidth limit (scales with
movers) from a serial hand-off chain (does not).  Median round on world rank 0's clock."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

rounds = 8
movers = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16,64,128,0").split(",")]
# sizes in MiB, or KiB with a k suffix
sizes = [(int(x[:-1]) << 10) if x.endswith("k") else (int(x) << 20) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,64").split(",")]
ranks = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "8").split(",")]
for G, mv in [(g, m) for g in ranks for m in movers]:
    with rlo.World(G, max_payload=64, bulk_max=max(sizes), movers=mv) as w:
        for nb in sizes:
            mib = nb / float(1 << 20)
            w.program_latency(rounds, nb, seed=0xB0 + (nb >> 10))
            w.run()
            st = w.stats()
            assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
            obs = w.round_ticks().astype(np.float64)
            d = np.diff(obs[obs > 0])
            rt = float(np.median(d)) * 1e-8 if len(d) else float("nan")
            lat = w.latencies_ticks().astype(np.float64) * 0.01  # origination -> last receiver holds it (us)
            print("N %3d movers %3d (%3d) %8.3f MiB: round %8.1f us  latency p50 %7.1f us  kernel %7.3f ms  hbm %7.1f GB/s (frac %.3f)" %
                  (G, mv, w.info["movers"], mib, rt * 1e6, float(np.median(lat)) if len(lat) else -1.0, w.kernel_ms(), 2 * G * nb / rt / 1e9,
                   2 * G * nb / rt / 8e12), flush=True)
