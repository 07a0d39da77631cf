# A/B of pulled payloads (RLO_PULL) on the payload-size legs: 256 ranks, 65,536 bcasts, bench.py's storm
set -o pipefail
for pull in 0 1; do
  for L in 256 1024 4096; do
    RLO_PULL=$pull timeout -k 10 120 python3 - $L <<'PY' || exit 1
import sys, time
sys.path.insert(0, "rootless-coll-mpi-ops_amd"); sys.path.insert(0, "oracle")
import rlo, pyoracle as orc, numpy as np, os
L = int(sys.argv[1]); n, k = 256, 1 << 16
with rlo.World(n, max_payload=max(64, L)) as w:
    w.program_storm(k, L, seed=0x5EED)
    w.run(); w.run()
    ms = w.kernel_ms(); st = w.stats()
exp = orc.storm_expected(n, 0x5EED, k, L)
ok = bool((st["error"] == 0).all() and np.array_equal(st["bcast_sum"], exp["sum"]))
alg = 2 * (n - 1) * (L + 16) * k / (ms * 1e-3) / 1e9
print("pull=%s len=%d kernel_ms=%.3f bcast/s=%.0f alg_GBps=%.1f frac=%.4f ok=%s" % (os.environ.get("RLO_PULL"), L, ms, k / (ms * 1e-3), alg, alg / 8000, ok), flush=True)
PY
  done
done
