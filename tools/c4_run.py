"""One-proposal decisions (C4) at a small world, product library: the workload for a PMC pass over the hop kernel.
    python tools/c4_run.py [n] [proposals per rank] [runs] [one_xcd]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
import rlo  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
p = int(sys.argv[2]) if len(sys.argv) > 2 else 256
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
one_xcd = len(sys.argv) > 4 and sys.argv[4] == "one_xcd"  # RLO_PART_ONE_XCD
with rlo.World(n, max_payload=64, one_xcd=one_xcd) as w:
    w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(p) for r in range(n)])
    for _ in range(runs):
        ms = w.run()
        st = w.stats()
        assert (st["error"] == 0).all(), st["error"]
        print("n %d: %.0f decisions/s, kernel %d, iterations per rank %.0f" % (n, n * p / (ms * 1e-3), w.info_now()["last_kernel"],
                                                                               st["iterations"].mean()), flush=True)
