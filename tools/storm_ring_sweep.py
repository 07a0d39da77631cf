import os, sys
sys.path.insert(0, "rootless-coll-mpi-ops_amd")
import rlo
n, k = 256, 1 << 18
for ln, slots_l, wins in ((64, (2048, 4096, 8192), (32, 64, 128)), (256, (2048, 4096), (64, 128))):
    for slots in slots_l:
        w = rlo.World(n, max_payload=ln, ring_slots=slots)
        for win in wins:
            kk = k if ln <= 64 else k // 4
            w.program_storm(kk, ln, window=win)
            ms = sorted(w.run() for _ in range(3))[1]
            print("len %5d slots %5d win %3d: %6.2f M bcast/s  %.3f ms" % (ln, slots, win, kk / ms * 1e-3, ms), flush=True)
        w.close()
