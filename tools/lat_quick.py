"""Quick latency / decisions probe of the device programs (one GPU): p50 / p99 one-way latency of the
latency program and decisions/s with one outstanding proposal per rank, at a few world sizes.
RLO_DIAG_LIB=1 RLO_NO_LL=1 runs the diagnostics library without doorbells (A/B)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

for n in [int(x) for x in (sys.argv[1:] or ["4", "8", "64", "256"])]:
    with rlo.World(n, max_payload=64) as w:
        w.program_latency(2000, 64, seed=21)
        w.run()
        st = w.stats()
        lat = w.latencies_ticks().astype(np.float64) * 0.01
        obs = w.round_ticks().astype(np.float64)
        rd = np.diff(obs[obs > 0]) * 0.01  # successive round completions seen by world rank 0 (us)
        ok_l = bool((st["error"] == 0).all())
        p = 256 if n <= 64 else 32
        w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(p) for r in range(n)])
        w.run()
        t = time.perf_counter()
        ms = w.run()
        dt = time.perf_counter() - t
        st2 = w.stats()
        ok_i = bool((st2["error"] == 0).all()) and int(st2["own_decided"].sum()) == n * p
        print("n %4d  lat p50 %6.2f us p99 %6.2f us round p50 %6.2f p99 %7.2f | decisions/s %9.0f (kernel %9.0f) decision_us %6.1f  ok %s %s" %
              (n, np.percentile(lat, 50), np.percentile(lat, 99), np.percentile(rd, 50), np.percentile(rd, 99), n * p / dt, n * p / (ms * 1e-3), ms * 1e3 / p, ok_l, ok_i),
              flush=True)
