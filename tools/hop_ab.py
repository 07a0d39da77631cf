"""A/B of the hop kernel (rlo_hop.hip) against the progress kernel's doorbell pass on the programs it serves: the latency
program (one-way p50 / p99) and the iar program (decisions/s with one and with 16 own proposals in flight per rank),
at several world sizes.  Arms: the product library (the hop kernel wherever it is eligible) and the diagnostics library
with RLO_NO_HOP=1 (the progress kernel), alternated per leg so box noise hits both.  Every run's kernel
(rlo_world_info_t.last_kernel) and its error words are printed beside the numbers.
  python tools/hop_ab.py [n ...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rootless-coll-mpi-ops_amd")
CHILD = r'''
import sys, time, numpy as np
sys.path.insert(0, sys.argv[1])
import rlo
n = int(sys.argv[2])
out = []
with rlo.World(n, max_payload=64) as w:
    w.program_latency(2000, 64, seed=21)
    w.run()
    k1 = w.info_now()["last_kernel"]
    st = w.stats()
    lat = w.latencies_ticks().astype(np.float64) * 0.01
    out += ["p50 %.2f p99 %.2f" % (np.percentile(lat, 50), np.percentile(lat, 99))]
    p = 64 if n <= 64 else 32
    w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(p) for r in range(n)])
    w.run()
    t = time.perf_counter(); ms = w.run(); dt = time.perf_counter() - t
    st2 = w.stats()
    ok = int(st2["own_decided"].sum()) == n * p and (st2["error"] == 0).all() and (st["error"] == 0).all()
    out += ["dec/s %.0f (kernel %.0f)" % (n * p / dt, n * p / (ms * 1e-3)), "kern %d/%d" % (k1, w.info_now()["last_kernel"]), "ok %d" % ok]
with rlo.World(n, max_payload=32, proposal_pool=16) as w:
    pp = 128 if n <= 64 else 128
    w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(pp) for r in range(n)], pool=16)
    w.run()
    t = time.perf_counter(); ms = w.run(); dt = time.perf_counter() - t
    st = w.stats()
    ok = int(st["own_decided"].sum()) == n * pp and (st["error"] == 0).all()
    out += ["pool16 %.0f kern %d ok %d" % (n * pp / dt, w.info_now()["last_kernel"], ok)]
print(" | ".join(out))
'''
ns = [int(x) for x in (sys.argv[1:] or ["4", "8", "64", "256"])]
arms = [("hop", dict(os.environ)), ("full", dict(os.environ, RLO_DIAG_LIB="1", RLO_NO_HOP="1"))]
for n in ns:
    for rep in range(2):
        for tag, env in arms:
            r = subprocess.run([sys.executable, "-c", CHILD, PKG, str(n)], capture_output=True, text=True, timeout=150, env=env)
            print("n %4d %-4s rep %d: %s %s" % (n, tag, rep, r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else ""),
                  flush=True)
