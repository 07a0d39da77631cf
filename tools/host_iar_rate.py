"""Decisions/s of the host-service path with every rank in this process (no MPI, no pump):
each rank keeps one proposal outstanding, approve-all host judge.  Separates the engine's
IAR round trips from the MPI drop-in library's.

  python tools/host_iar_rate.py [--n 8 --p 200]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--p", type=int, default=200)
    a = ap.parse_args()
    import rlo
    from rlo import abi

    n, P = a.n, a.p
    done = [0] * n
    with rlo.HostWorld(n, max_payload=256) as hw:
        for r in range(n):
            hw.propose(r, r, b"0123456789abcdef")
        t0 = time.perf_counter()
        while min(done) < P:
            hw.flush()
            for r in range(n):
                for ev in hw.poll(r):
                    k = ev["kind"]
                    if k == abi.RLO_EV_JUDGE:
                        hw.judge(r, ev, 1)
                    elif k == abi.RLO_EV_OWN_JUDGE:
                        hw.own_judge(r, ev, 1)
                    elif k == abi.RLO_EV_RESULT:
                        done[r] += 1
                        if done[r] < P:
                            hw.propose(r, done[r] * n + r, b"0123456789abcdef")
            if time.perf_counter() - t0 > 60:
                print("stalled", done)
                break
        dt = time.perf_counter() - t0
    print({"n": n, "P": P, "seconds": round(dt, 3), "decisions_per_s": round(sum(done) / dt, 1)})


if __name__ == "__main__":
    main()
