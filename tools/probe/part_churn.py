"""Probe (round 5): the 8-part rehearsal's stale heap mapping, outside bench.py.  P part processes (spawned, one
GPU) run the bench's leg sequence on sharded worlds -- a bulk world (one rank per part, 64 MiB slots: the C3 leg),
then a C5-like world (16 ranks per part, 4 KiB ring slots, 1 MiB bulk slots: ~4 GiB of heap per part) -- and
report every rlo_part_connect that fails (RLO_E_STALE prints which region).  Knobs (argv):
    python tools/probe/part_churn.py [parts=8] [repeats=2] [mode=plain|sync|split]
  sync : hipDeviceSynchronize (torch.cuda.synchronize) in every part before it closes a world
  split: close in two phases -- every part closes its imports, barrier, then frees its own regions
  nobar / split-nobar: the same without the barrier after the close (the bench's legs: a part may create and export
         its next world while its peers still hold imports of its previous one)"""
import multiprocessing as mp
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PARTS = int(sys.argv[1]) if len(sys.argv) > 1 else 8
REPEATS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
MODE = sys.argv[3] if len(sys.argv) > 3 else "plain"
TORCH = os.environ.get("PROBE_TORCH", "1") == "1"  # the bench's processes run torch on the GPU too
LEGS = [dict(per=32, max_payload=64, bulk_max=0, movers=0, prog=("storm", 16384, 64)),
        dict(per=1, max_payload=64, bulk_max=64 << 20, movers=16, prog=("lat", 8, 1 << 20)),
        dict(per=16, max_payload=4096, bulk_max=1 << 20, movers=4, prog=("storm", 2048, 64))]


def worker(part, blob_q, blobs_q, bar, out_q):
    sys.path.insert(0, os.path.join(REPO, "rootless-coll-mpi-ops_amd"))
    if TORCH:
        import torch
        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    import rlo
    res = []
    try:
        for rep in range(REPEATS):
            for li, leg in enumerate(LEGS):
                n = leg["per"] * PARTS
                w = rlo.World.part(n, PARTS, part, max_payload=leg["max_payload"], uncached=True, bulk_max=leg["bulk_max"],
                                   movers=leg["movers"])
                blob_q.put((part, w.export()))
                blobs = blobs_q.get(timeout=120)
                err = None
                try:
                    if MODE.startswith("staged"):
                        w.staged_connect(blobs, lambda: bar.wait(timeout=120))
                    else:
                        w.connect(blobs)
                except Exception as e:  # noqa: BLE001
                    err = repr(e)
                bar.wait(timeout=120)
                ok = err is None
                if ok:
                    kind, a, b = leg["prog"]
                    if kind == "lat":
                        w.program_latency(a, b, seed=0xB0)
                    elif leg["bulk_max"]:
                        w.program_storm(a, b, seed=0xC5, len_max=leg["bulk_max"], order=1)
                    else:
                        w.program_storm(a, b, seed=0x5EED)
                    w.reset()
                bar.wait(timeout=120)
                rc = None
                if ok:
                    w.launch(no_reset=True)
                    rc = w.wait(raise_on_device_error=False)
                bar.wait(timeout=120)
                if MODE == "sync":
                    import ctypes
                    ctypes.CDLL("libamdhip64.so").hipDeviceSynchronize()
                if MODE.startswith("split"):
                    w.close_imports()
                    bar.wait(timeout=120)
                w.close()
                res.append((rep, li, err, rc))
                if not MODE.endswith("nobar"):
                    bar.wait(timeout=120)
        out_q.put((part, res))
    except Exception as e:  # noqa: BLE001
        out_q.put((part, repr(e)))


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    blob_q, out_q = ctx.Queue(), ctx.Queue()
    blobs_qs = [ctx.Queue() for _ in range(PARTS)]
    bar = ctx.Barrier(PARTS)
    procs = [ctx.Process(target=worker, args=(p, blob_q, blobs_qs[p], bar, out_q)) for p in range(PARTS)]
    for p in procs:
        p.start()
    for _ in range(REPEATS * len(LEGS)):
        got = dict(blob_q.get(timeout=300) for _ in range(PARTS))
        for q in blobs_qs:
            q.put([got[p] for p in range(PARTS)])
    outs = dict(out_q.get(timeout=600) for _ in range(PARTS))
    for p in procs:
        p.join(timeout=60)
    bad = 0
    for part in range(PARTS):
        r = outs[part]
        if isinstance(r, str):
            print("part %d: %s" % (part, r))
            bad += 1
            continue
        for rep, li, err, rc in r:
            if err or rc:
                bad += 1
                print("part %d repeat %d leg %d: connect %s rc %s" % (part, rep, li, err, rc))
    print("PART_CHURN parts %d repeats %d mode %s: %d failures" % (PARTS, REPEATS, MODE, bad), flush=True)
