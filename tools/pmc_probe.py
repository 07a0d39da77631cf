"""One storm launch of the bench workload (for rocprofv3 --pmc passes; bench.py spawns it).

  python tools/pmc_probe.py [--ranks 256 --len 64 --k 262144 --launches 2]
  python tools/pmc_probe.py --iar 8 [--pend-hbm]    (the C4 leg instead: every rank keeps one proposal in flight,
                                                    8 in turn; --pend-hbm forces the pending tables into HBM)

Every launch is the same storm bench.py times; rocprofv3 attributes counters per dispatch,
the caller keeps the last launch's values.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=256)
    ap.add_argument("--len", type=int, default=64)
    ap.add_argument("--k", type=int, default=1 << 18)
    ap.add_argument("--launches", type=int, default=2)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--iar", type=int, default=0)
    ap.add_argument("--pend-hbm", action="store_true")
    a = ap.parse_args()
    import rlo

    with rlo.World(a.ranks, max_payload=max(64, a.len), device=a.device, pend_hbm=a.pend_hbm) as w:
        if a.iar:
            w.program_iar([(r, it * a.ranks + r, b"0123456789abcdef") for it in range(a.iar) for r in range(a.ranks)])
        else:
            w.program_storm(a.k, a.len, seed=0x5EED)
        for _ in range(a.launches):
            w.run()
        st = w.stats()
        assert (st["error"] == 0).all(), st["error"]
    print("pmc_probe ok", flush=True)


if __name__ == "__main__":
    main()
