"""The latency program at a world size, product library: the workload for a rocprof pass over the hop kernel.
    python tools/lat_run.py [n] [rounds] [runs] [one_xcd]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
one_xcd = len(sys.argv) > 4 and sys.argv[4] == "one_xcd"  # RLO_PART_ONE_XCD
with rlo.World(n, max_payload=64, one_xcd=one_xcd) as w:
    w.program_latency(rounds, 64, seed=21)
    for _ in range(runs):
        ms = w.run()
        st = w.stats()
        assert (st["error"] == 0).all(), st["error"]
        lat = w.latencies_ticks().astype(np.float64) * 0.01
        print("n %d: p50 %.2f p99 %.2f us, kernel %.3f ms (%d rounds), last kernel %d" % (
            n, np.percentile(lat, 50), np.percentile(lat, 99), ms, rounds, w.info_now()["last_kernel"]), flush=True)
