"""Storm A/B probe (one GPU): kernel ms of the 256-rank storm at 64 B (2^18 bcasts) and 256 B / 1 KiB /
4 KiB (2^16), median of 5 launches, every launch's checksums equal.  Run once per library
(RLO_LIB_DIR=lib_<name> picks an A/B build)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

tag = os.environ.get("RLO_LIB_DIR", "lib")
for ln, k in [(64, 1 << 18), (256, 1 << 16), (1024, 1 << 16), (4096, 1 << 16)]:
    with rlo.World(256, max_payload=ln) as w:
        w.program_storm(k, ln, seed=0x5EED)
        ms, sums = [], []
        for i in range(6):
            ms.append(w.run())
            st = w.stats()
            sums.append(st["bcast_sum"].copy())
            assert (st["error"] == 0).all()
        ok = all(np.array_equal(sums[0], x) for x in sums)
        m = float(np.median(ms[1:]))
        alg = k * 2.0 * 255 * (ln + 16) / (m * 1e-3) / 1e9
        print("%-8s len %5d waves %d kernel_ms med %8.3f min %8.3f  bcast/s %6.2fM frac %.4f same_bytes %s" %
              (tag, ln, w.info["waves"], m, min(ms[1:]), k / (m * 1e-3) / 1e6, alg / 8000, ok), flush=True)
