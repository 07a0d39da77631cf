"""Sharded worlds: the ranks of one world split into parts, each part its own kernel and
its own rings, producers storing into peer parts' rings.

run_inprocess(): every part in this process, one HIP stream each (same GPU or several).
run_processes(): one spawned process per part; blobs are exchanged through a queue, the
                 regions are mapped with hipIpc (dmabuf), launches start after a barrier
                 that follows every part's reset.
A program spec is a dict: {"kind": "storm", "k", "len", "seed", "window", "log", "len_max", "order"} or
{"kind": "iar", "props": [(origin, pid, bytes)], "judge", "mask", "isp", "seed", "ppm", "log", "pool"} or
{"kind": "lat", "rounds", "len", "seed"} (the round word lives in part 0; st["round_ticks"] is world
rank 0's clock at each round's completion).
"""
import ctypes
import multiprocessing as mp
import os

import numpy as np


def even_bounds(n, parts):
    return [n * p // parts for p in range(parts + 1)]


def _program(w, spec):
    if spec["kind"] == "storm":
        w.program_storm(spec["k"], spec["len"], seed=spec.get("seed", 0x5EED), window=spec.get("window", 64),
                        log=spec.get("log", False), log_cap=spec.get("log_cap", 0), hist=spec.get("hist", False),
                        len_max=spec.get("len_max", 0), order=spec.get("order", 0))
    elif spec["kind"] == "iar":
        from . import _lib as L
        w.program_iar(spec["props"], judge=spec.get("judge", L.RLO_JUDGE_APPROVE), mask=spec.get("mask"),
                      isp=spec.get("isp"), seed=spec.get("seed", 0), ppm=spec.get("ppm", 0),
                      log=spec.get("log", False), log_cap=spec.get("log_cap", 0), pool=spec.get("pool", 1))
    elif spec["kind"] == "lat":
        w.program_latency(spec["rounds"], spec["len"], seed=spec.get("seed", 0x5EED))
    else:
        raise ValueError(spec["kind"])


def _collect(w, spec):
    st = w.stats()
    out = {"rank_begin": w.rank_begin, "stats": st, "ms": w.kernel_ms(), "info": dict(w.info)}
    if spec["kind"] == "lat" and w.rank_begin == 0:
        out["rounds"] = w.round_ticks()
    if spec.get("log"):
        cap = spec.get("log_cap", 0) or 1024
        out["logs"] = {r: w.log(r, cap=cap, payload=spec["kind"] == "storm") for r in range(w.rank_begin, w.rank_end)}
    return out


def merge(results):
    """Concatenate per-part stats (ordered by rank) into world-wide arrays."""
    results = sorted(results, key=lambda r: r["rank_begin"])
    st = {}
    for key in results[0]["stats"]:
        st[key] = np.concatenate([r["stats"][key] for r in results])
    # per world rank: its part's rlo_world_info_t.peers / sys_scope (where that part's peers are)
    for key in ("peers", "sys_scope"):
        st["part_" + key] = np.concatenate([np.full(len(r["stats"]["error"]), r["info"][key]) for r in results])
    logs = {}
    for r in results:
        logs.update(r.get("logs", {}))
        if "rounds" in r:
            st["round_ticks"] = r["rounds"]
    return st, logs, [r["ms"] for r in results]


def run_inprocess(n, bounds, spec, max_payload=4096, ring_slots=0, devices=None, uncached=False, blobs_for=None,
                  **world_kw):
    """world_kw: bulk_max / bulk_slots / movers / chunked (World.part).  blobs_for(p, blobs): the blobs part p
    connects with (tests: a forged PCI bus puts a peer "on another GPU", so the part runs system scope)"""
    from . import _lib as L
    from .world import World

    parts = len(bounds) - 1
    devices = devices or [0] * parts
    streams = []
    ws = [World.part(n, parts, p, part_begin=bounds, max_payload=max_payload, ring_slots=ring_slots,
                     device=devices[p], uncached=uncached, **world_kw) for p in range(parts)]
    try:
        blobs = [w.export() for w in ws]
        for p, w in enumerate(ws):
            w.connect(blobs_for(p, blobs) if blobs_for else blobs)
        for w in ws:
            _program(w, spec)
        for w in ws:
            w.reset()
        lib = L.load()
        for d in devices:
            s = ctypes.c_void_p()
            L.check(lib.rlo_stream_create(d, ctypes.byref(s)), "rlo_stream_create")
            streams.append(s)
        for w, s in zip(ws, streams):
            w.launch(stream=s, no_reset=True)
        rcs = [w.wait(raise_on_device_error=False) for w in ws]
        res = [_collect(w, spec) for w in ws]
        return merge(res), rcs
    finally:
        for w in ws:
            w.close()
        for s in streams:
            L.load().rlo_stream_destroy(s)


def _worker(n, bounds, part, device, spec, max_payload, ring_slots, uncached, blob_q, blobs_q, barrier, out_q,
            world_kw, repeat=1):
    try:
        from . import _lib as L
        from .world import World, pool_trim

        for it in range(repeat):
            w = World.part(n, len(bounds) - 1, part, part_begin=bounds, max_payload=max_payload, ring_slots=ring_slots,
                           device=device, uncached=uncached, **world_kw)
            blob_q.put((part, w.export()))
            blobs = blobs_q.get(timeout=120)

            def bcast(blob, k):  # part k's fresh blob, relayed by the parent
                if blob is not None:
                    blob_q.put((k, blob))
                return blobs_q.get(timeout=120)

            # one exporter at a time, its handles exported at its own stage (rlo_hip.h rlo_part_import)
            w.staged_connect(blobs, lambda: barrier.wait(timeout=120), bcast)
            _program(w, spec)
            w.reset()
            barrier.wait(timeout=120)  # every part is reset before any part launches
            w.launch(no_reset=True)
            rc = w.wait(raise_on_device_error=False)
            res = _collect(w, spec)
            barrier.wait(timeout=120)  # no peer still stores into this part's rings
            # every part drops its imports of its peers' regions before any part frees its own (a part that frees and
            # re-exports memory a peer still imports can hand that peer its OLD memory for the new handle)
            w.close_imports()
            barrier.wait(timeout=120)
            w.close()
            if os.environ.get("RLO_POOL_CAP_BYTES"):
                # a lowered pool cap (the test hook): the world-wide close, so exported regions beyond it are freed --
                # every part drops its idle imports, then every part frees its retired regions (rlo_hip.h rlo_pool_trim)
                pool_trim(L.RLO_TRIM_IMPORTS | L.RLO_TRIM_FREE)
                barrier.wait(timeout=120)
                res["pool_freed"] = pool_trim(L.RLO_TRIM_RETIRED)
                barrier.wait(timeout=120)
            out_q.put((part, rc, res, None))
    except Exception as e:  # report instead of hanging the parent
        out_q.put((part, -99, None, repr(e)))


def run_processes(n, bounds, spec, max_payload=4096, ring_slots=0, devices=None, uncached=False, timeout=300,
                  repeat=1, **world_kw):
    """repeat > 1: every part process creates, connects (hipIpc), runs and destroys the world `repeat` times
    in a row -- the per-leg churn of bench.py's N-part run; returns the list of per-repeat results"""
    parts = len(bounds) - 1
    devices = devices or [0] * parts
    ctx = mp.get_context("spawn")
    blob_q, out_q = ctx.Queue(), ctx.Queue()
    blobs_qs = [ctx.Queue() for _ in range(parts)]
    barrier = ctx.Barrier(parts)
    procs = [ctx.Process(target=_worker, args=(n, bounds, p, devices[p], spec, max_payload, ring_slots, uncached,
                                               blob_q, blobs_qs[p], barrier, out_q, world_kw, repeat))
             for p in range(parts)]
    for p in procs:
        p.start()
    runs = []
    try:
        for _ in range(repeat):
            got = dict(blob_q.get(timeout=timeout) for _ in range(parts))
            blobs = [got[p] for p in range(parts)]
            for q in blobs_qs:
                q.put(blobs)
            for k in range(parts):  # staged connect: part k's fresh blob to every part
                pk, bk = blob_q.get(timeout=timeout)
                assert pk == k, (pk, k)
                for q in blobs_qs:
                    q.put(bk)
            outs = [out_q.get(timeout=timeout) for _ in range(parts)]
            errs = [(p, e) for p, rc, r, e in outs if e]
            if errs:
                raise RuntimeError("part failed: %s" % errs)
            runs.append((merge([r for _, _, r, _ in outs]), [rc for _, rc, _, _ in sorted(outs, key=lambda x: x[0])]))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return runs[0] if repeat == 1 else runs
