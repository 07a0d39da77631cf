"""Ring-depth probe of the payload-size storms (one GPU, 256 ranks, 65,536 bcasts): kernel ms per ring
capacity, every launch's checksums equal to the first's."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

k = 1 << 16
for ln in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "256,1024").split(",")]:
    for slots in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "512,1024,2048").split(",")]:
        with rlo.World(256, max_payload=ln, ring_slots=slots) as w:
            w.program_storm(k, ln, seed=0x5EED)
            ms, sums = [], []
            for i in range(4):
                ms.append(w.run())
                st = w.stats()
                assert (st["error"] == 0).all()
                sums.append(st["bcast_sum"].copy())
            m = float(np.median(ms[1:]))
            alg = k * 2.0 * 255 * (ln + 16) / (m * 1e-3) / 1e9
            print("len %5d slots %5d waves %d pull %d kernel_ms %8.3f bcast/s %6.2fM frac %.4f same %s" %
                  (ln, slots, w.info["waves"], w.info.get("pull", 0), m, k / (m * 1e-3) / 1e6, alg / 8000,
                   all(np.array_equal(sums[0], x) for x in sums)), flush=True)
