# A/B of kernel builds (tools/ab_libs/<commit>/librlo_hip.so vs HEAD's) on the 64 B headline storm
set -o pipefail
one() {  # lib
  RLO_LIB_AB=$1 timeout -k 10 120 python3 - <<'PY' || exit 1
import sys, os
sys.path.insert(0, "rootless-coll-mpi-ops_amd")
import rlo, numpy as np
n, k, L = 256, 1 << 18, 64
with rlo.World(n, max_payload=64) as w:
    w.program_storm(k, L, seed=0x5EED, window=64)
    ms = [w.run() for _ in range(4)][1:]
    st = w.stats()
print("%-60s kernel_ms min %.3f med %.3f  bcast/s %.2fM  waves %d err %d" % (os.environ.get("RLO_LIB_AB") or "HEAD", min(ms), sorted(ms)[1], k / min(ms) * 1e-3 / 1e3, w.info["waves"], int(st["error"].max())), flush=True)
PY
}
for rep in 1 2; do
  for lib in "" tools/ab_libs/*/librlo_hip.so; do one "$lib" || exit 1; done
done
