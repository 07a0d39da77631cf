"""Latency anatomy of the host-service path (one bcast at a time, all ranks in this process):
host wall time from rlo_host_post to the last rank's pickup event vs the device's own
origination -> pickup-record time (LogRec.aux of a delivery, 10 ns ticks).

  python tools/host_latency.py [--n 4 --rounds 300]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=300)
    a = ap.parse_args()
    import rlo

    n = a.n
    host_us, dev_us, first_us = [], [], []
    with rlo.HostWorld(n, max_payload=64) as hw:
        for i in range(a.rounds):
            o = i % n
            got, dmax, tfirst = 0, 0, None
            t0 = time.perf_counter()
            hw.bcast(o, b"x" * 64, seq=i)
            while got < n - 1:
                for r in range(n):
                    for ev in hw.poll(r):
                        got += 1
                        dmax = max(dmax, ev["aux"])
                        if tfirst is None:
                            tfirst = time.perf_counter()
            t1 = time.perf_counter()
            host_us.append((t1 - t0) * 1e6)
            first_us.append((tfirst - t0) * 1e6)
            dev_us.append(dmax * 0.01)
    pct = lambda x, q: round(float(np.percentile(x, q)), 2)
    print({"n": n, "rounds": a.rounds, "host_p50_us": pct(host_us, 50), "host_p99_us": pct(host_us, 99),
           "first_pickup_p50_us": pct(first_us, 50), "device_origin_to_last_pickup_p50_us": pct(dev_us, 50),
           "device_p99_us": pct(dev_us, 99)})


if __name__ == "__main__":
    main()
