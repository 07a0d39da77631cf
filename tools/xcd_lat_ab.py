"""The latency program in default worlds vs RLO_PART_ONE_XCD worlds (every rank-wave on one XCD), at
the world sizes one XCD can hold, interleaved; per run the deliveries and checksums of the two must agree.
    python tools/xcd_lat_ab.py [sizes, comma-separated] [rounds] [reps]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,32,64,128,256").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2


def run(n, one_xcd):
    with rlo.World(n, max_payload=64, one_xcd=one_xcd) as w:
        w.program_latency(rounds, 64, seed=21)
        ms = w.run()
        st = w.stats()
        assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
        lat = w.latencies_ticks().astype(np.float64) * 0.01
        return np.percentile(lat, 50), np.percentile(lat, 99), ms, st["bcast_delivered"].copy(), st["bcast_sum"].copy()


for n in sizes:
    for rep in range(reps):
        res = {}
        for ox in (False, True):
            try:
                res[ox] = run(n, ox)
            except Exception as e:  # (a world one XCD cannot hold is refused at launch)
                res[ox] = None
                print("n %d %s: %s" % (n, "one_xcd" if ox else "default", e), flush=True)
        for ox, r in res.items():
            if r is not None:
                print("n %3d rep %d %-8s p50 %6.2f p99 %6.2f us, kernel %.2f ms" % (n, rep, "one_xcd" if ox else "default",
                                                                                  r[0], r[1], r[2]), flush=True)
        if res[False] is not None and res[True] is not None:
            same = np.array_equal(res[False][3], res[True][3]) and np.array_equal(res[False][4], res[True][4])
            print("n %3d rep %d deliveries and checksums equal: %s" % (n, rep, same), flush=True)
            assert same
