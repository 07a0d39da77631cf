"""C3 probe (one GPU, 8 ranks): bulk round time vs mover count, to tell a bandwidth limit (scales with
movers) from a serial hand-off chain (does not).  Median round on world rank 0's clock."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

G, rounds = 8, 8
movers = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16,64,128,0").split(",")]
sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,64").split(",")]
for mv in movers:
    with rlo.World(G, max_payload=64, bulk_max=max(sizes) << 20, movers=mv) as w:
        for mib in sizes:
            nb = mib << 20
            w.program_latency(rounds, nb, seed=0xB0 + mib)
            w.run()
            st = w.stats()
            assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
            obs = w.round_ticks().astype(np.float64)
            d = np.diff(obs[obs > 0])
            rt = float(np.median(d)) * 1e-8 if len(d) else float("nan")
            print("movers %3d (%3d) %2d MiB: round %8.1f us  kernel %7.3f ms  hbm %7.1f GB/s (frac %.3f)" %
                  (mv, w.info["movers"], mib, rt * 1e6, w.kernel_ms(), 2 * G * nb / rt / 1e9,
                   2 * G * nb / rt / 8e12), flush=True)
