"""Graded diagnostic of the bulk-message path (one step per process; the shell chain stops at the
first failure).  Steps: 1 bulk kernel, 64 B storm, no bulk traffic; 2 mixed ring sizes 64 B..4 KiB;
3 fixed 64 KiB bulk bcasts, 4 ranks; 4 the C5 mixed storm (16 ranks, 64 B .. 1 MiB, slots order);
5 the same with the delivery log."""
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rootless-coll-mpi-ops_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np  # noqa: E402

import pyoracle as orc  # noqa: E402
import rlo  # noqa: E402

step = int(sys.argv[1])
cfgs = {1: (16, 64, 64, 0, 4096, 1 << 20, 256), 2: (16, 64, 4096, 1, 4096, 1 << 20, 256),
        3: (4, 65536, 65536, 0, 64, 1 << 20, 16), 4: (16, 64, 1 << 20, 1, 4096, 1 << 20, 96),
        5: (16, 64, 1 << 20, 1, 4096, 1 << 20, 96), 6: (16, 64, 1 << 20, 1, 4096, 1 << 20, 96)}
n, lo, hi, order, cap, bmax, k = cfgs[step]
# step 6: exactly tests/test_gpu_bulk.py::test_c5_mixed_storm_one_part[16-96-1-5] (auto movers), repeated
reps = int(os.environ.get("REPS", "1"))
movers = 0 if step == 6 else 8
for rep in range(reps):
  with rlo.World(n, max_payload=cap, bulk_max=bmax, movers=movers) as w:
      print("info", {x: w.info[x] for x in ("waves", "movers", "bulk_slots", "heap_bytes", "blocks_per_cu")}, flush=True)
      w.program_storm(k, lo, seed=5, len_max=hi if hi > lo else 0, order=order, log=step in (5, 6), log_cap=k + 8)
      w.launch()
      rc = w.wait(raise_on_device_error=False)
      st = w.stats()
      code, aux = w.device_error()
      print("step", step, "rc", rc, "device error", code, hex(aux), "rank errors", st["error"].tolist(), flush=True)
      exp = orc.storm_expected(n, 5, k, lo, len_max=hi if hi > lo else 0, order=order)
      ok = rc == 0 and np.array_equal(st["bcast_sum"], exp["sum"]) and np.array_equal(
          st["bcast_delivered"].astype(np.int64), exp["count"])
      print("delivered", st["bcast_delivered"].tolist(), "expected", exp["count"].tolist(), flush=True)
      import ctypes
      dbg = (ctypes.c_uint64 * 48)()
      w.lib.rlo_bulk_debug(w.h, dbg, 48)
      d = list(dbg)
      print("jobs A posted %d head %d | B posted %d head %d | exited %d | tiles A %d B %d | gather waits %d passed %d "
            "last wait %x" % (d[0], d[8], d[16], d[24], d[32], d[36], d[37], d[38], d[39], d[46]), flush=True)
      print("posts scatter %d gather %d verify %d | releases %d | slot waits %d" % (d[41], d[42], d[43], d[44], d[45]),
            flush=True)
      g = d[47]
      if g:
          print("jctl47 %x" % g, flush=True)
          if g >> 56 == 0xDD:
              print("LDS-CORRUPT rank %d e %d fields %s shadow bid %d lds bid %d" % ((g >> 48) & 0xff, (g >> 40) & 0xff,
                    bin((g >> 32) & 0x7f), (g >> 16) & 0xffff, g & 0xffff), flush=True)
          if g >> 56 == 0xCC:
              print("WRONG-ORIGIN at rank %d from %d: header origin %d tag %d id %d" % ((g >> 48) & 0xff, (g >> 40) & 0xff,
                    (g >> 32) & 0xff, (g >> 24) & 0xff, g & 0xffffff), flush=True)
          if g >> 56 == 0xEE:
              print("EARLY-RELEASE rank %d o %d s %d bid %d tflag %d want %d" % ((g >> 48) & 0xff, (g >> 40) & 0xff,
                    (g >> 36) & 0xf, (g >> 24) & 0xfff, (g >> 12) & 0xfff, g & 0xfff), flush=True)
          print("LIVE-REGISTER rank %d e %d old bid %d new bid %d tflag %d old target %d" % (
              g >> 56, (g >> 48) & 0xff, (g >> 32) & 0xffff, (g >> 16) & 0xffff, (g >> 8) & 0xff, g & 0xff), flush=True)
      for r in range(n):
          g = [int(x) for x in st["dbg"][r]]
          print("rank %d bulk_q %d pending %d:" % (r, g[0] >> 32, g[0] & 0xffffffff),
                ["e=%d(o%d,s%d) target %d sflag %d tflag %d" % (g[1 + 2 * i] >> 32, (g[1 + 2 * i] >> 32) // 2,
                                                              (g[1 + 2 * i] >> 32) % 2, g[1 + 2 * i] & 0xffffffff,
                                                              g[2 + 2 * i] >> 32, g[2 + 2 * i] & 0xffffffff)
                 for i in range(min(3, g[0] & 0xffffffff))], "sdone", g[7] & 0xffffffff, g[7] >> 32, flush=True)
      print("STEP", step, "rep", rep, "OK" if ok else "MISMATCH", flush=True)
      if not ok:
          sys.exit(1)
