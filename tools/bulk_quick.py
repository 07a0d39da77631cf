"""Quick C3 probe (one GPU, 8 ranks): round time of the rootless bulk bcast at 1 / 4 / 16 / 64 MiB (the
latency program, median round on world rank 0's clock), HBM GB/s by the (2G+1)S byte model."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

G, rounds = 8, 8
with rlo.World(G, max_payload=64, bulk_max=64 << 20) as w:
    for mib in (1, 4, 16, 64):
        nb = mib << 20
        w.program_latency(rounds, nb, seed=0xB0 + mib)
        sums = []
        for _ in range(2):
            w.run()
            st = w.stats()
            assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
            sums.append(st["bcast_sum"].copy())
        obs = w.round_ticks().astype(np.float64)
        d = np.diff(obs[obs > 0])
        if not len(d):
            print("bulk %2d MiB: no rounds observed (%s)" % (mib, obs), flush=True)
            continue
        rt = float(np.median(d)) * 1e-8
        print("bulk %2d MiB: round %8.1f us  algbw %7.1f GB/s  hbm %7.1f GB/s (frac %.3f)  same %s" %
              (mib, rt * 1e6, nb / rt / 1e9, (2 * G + 1) * nb / rt / 1e9, (2 * G + 1) * nb / rt / 8e12,
               np.array_equal(sums[0], sums[1])), flush=True)
