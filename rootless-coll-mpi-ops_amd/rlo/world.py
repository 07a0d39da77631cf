"""Python host mirror of the device engine (librlo_hip.so).

World(n) hosts n virtual ranks on one MI355X (one persistent workgroup each).
Programs map the reference's application loops onto the device:

  storm()    -- K bcasts from random originators: RLO_msg_new_bc + RLO_bcast_gen at the
                originator, RLO_make_progress_all + RLO_user_pickup_next everywhere
                (rootless_ops.c:311, :1581, :538, :938; testcases.c:638-697)
  latency()  -- one bcast at a time (test_gen_bcast style, testcases.c:59-108)
  iar()      -- RLO_submit_proposal / vote / decision (rootless_ops.c:668-917)
"""
import ctypes

import numpy as np

from . import _lib as L
from ._lib import check


class World:
    """A world of n ranks.  World(n) hosts all of them on one GPU; World.part(...) creates one
    part of a sharded world (export() -> exchange blobs -> connect(blobs))."""

    def __init__(self, n, max_payload=4096, ring_slots=0, device=-1, _part=None, bulk_max=0, bulk_slots=0, movers=0,
                 proposal_pool=0, pend_hbm=False, one_xcd=False):
        """bulk_max > 0: messages longer than max_payload (up to bulk_max bytes) are bulk messages --
        announced through the rings, moved by `movers` mover workgroups (0 = auto) between per-rank
        heaps of bulk_slots slots per origin (rlo_hip.h).  proposal_pool: pending entries per origin
        = the most own proposals a rank can keep in flight (power of two <= 16; 0 = 2).  pend_hbm: the
        pending-proposal tables in HBM whatever N (the 8-GPU world's layout, rehearsed at a smaller N).
        one_xcd (no bulk, as many ranks as one XCD holds: <= 256): cached rings and every rank-wave of the hop kernel on one XCD, hand-offs
        through its L2 (RLO_PART_ONE_XCD); only the hop kernel's programs run in such a world."""
        self.lib = L.load()
        h = ctypes.c_void_p()
        if _part is None:
            cfg = L.WorldCfg(n, max_payload, ring_slots, device, bulk_max, bulk_slots, movers, proposal_pool,
                             (L.RLO_PART_PEND_HBM if pend_hbm else 0) | (L.RLO_PART_ONE_XCD if one_xcd else 0))
            check(self.lib.rlo_world_create(ctypes.byref(cfg), ctypes.byref(h)), "rlo_world_create")
        else:
            n_parts, part, begin, flags = _part
            self._pb = None
            pb = None
            if begin is not None:
                self._pb = (ctypes.c_int32 * (n_parts + 1))(*begin)
                pb = ctypes.cast(self._pb, ctypes.c_void_p)
            cfg = L.PartCfg(n, n_parts, part, pb, max_payload, ring_slots, device, flags, bulk_max, bulk_slots, movers,
                            proposal_pool)
            check(self.lib.rlo_part_create(ctypes.byref(cfg), ctypes.byref(h)), "rlo_part_create")
        self.h = h
        self.n = n
        self._query()
        self._lat_rounds = 0

    @classmethod
    def part(cls, n, n_parts, part, part_begin=None, max_payload=4096, ring_slots=0, device=-1, uncached=False,
             bulk_max=0, bulk_slots=0, movers=0, proposal_pool=0, chunked=False, pend_hbm=False):
        """pend_hbm: the pending-proposal tables in HBM whatever N (the layout of the 8-GPU world's parts,
        rehearsed at a smaller N)"""
        return cls(n, max_payload, ring_slots, device,
                   _part=(n_parts, part, part_begin, (L.RLO_PART_UNCACHED if uncached else 0) |
                          (L.RLO_PART_CHUNKED if chunked else 0) | (L.RLO_PART_PEND_HBM if pend_hbm else 0)),
                   bulk_max=bulk_max,
                   bulk_slots=bulk_slots, movers=movers, proposal_pool=proposal_pool)

    def _query(self):
        info = L.WorldInfo()
        check(self.lib.rlo_world_query(self.h, ctypes.byref(info)), "rlo_world_query")
        self.info = {f: getattr(info, f) for f, _ in L.WorldInfo._fields_}
        self.rank_begin, self.rank_end = self.info["rank_begin"], self.info["rank_end"]
        self.n_local = self.rank_end - self.rank_begin

    def info_now(self):
        """rlo_world_query now (self.info is the answer at creation / connection): e.g. last_kernel after a launch"""
        self._query()
        return self.info

    def export(self):
        buf = ctypes.create_string_buffer(L.RLO_PART_BLOB_BYTES)
        check(self.lib.rlo_part_export(self.h, buf, L.RLO_PART_BLOB_BYTES), "rlo_part_export")
        return buf.raw

    def connect(self, blobs):
        joined = b"".join(blobs)
        check(self.lib.rlo_part_connect(self.h, joined, len(blobs)), "rlo_part_connect")
        self._query()

    def reset(self, stream=None):
        check(self.lib.rlo_reset(self.h, stream), "rlo_reset")

    def import_part(self, blob, q):
        """rlo_part_import: map part q's regions now (connect() then skips q)"""
        check(self.lib.rlo_part_import(self.h, blob, q), "rlo_part_import")

    def staged_connect(self, blobs, barrier, bcast=None):
        """connect in n_parts stages: in stage k every other part imports part k's regions while part k imports
        nothing, then barrier() (rlo_hip.h rlo_part_import).  bcast(blob or None, k) -> part k's blob: part k
        exports its handles afresh at the start of its stage and every part imports those (a handle exported
        before its exporter imported anything).  An import error is raised after the last stage, so every part
        still joins every barrier"""
        err = None
        me = self.info["part"]
        for k, b in enumerate(blobs):
            if bcast is not None:
                b = bcast(self.export() if k == me else None, k)
            if k != me and err is None:
                try:
                    self.import_part(b, k)
                except Exception as e:  # noqa: BLE001 - re-raised below
                    err = e
            barrier()
        if err is not None:
            raise err
        self.connect(blobs)

    def close_imports(self):
        """rlo_part_close_imports: drop the hipIpc imports of the peers' regions (the part can no longer launch)"""
        if self.h:
            check(self.lib.rlo_part_close_imports(self.h), "rlo_part_close_imports")

    def close(self):
        if self.h:
            self.lib.rlo_world_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ programs
    def program_storm(self, k, length, seed=0x5EED, window=64, log=False, hist=False, log_cap=0, prof=False,
                      len_max=0, order=L.RLO_ORDER_RANDOM):
        """len_max > length: mixed sizes (piecewise log-uniform per bcast); order RLO_ORDER_SLOTS: bcast b
        originates at rank b % n (every rank originates in every slot of n bcasts)."""
        flags = (L.RLO_FLAG_LOG if log else 0) | (L.RLO_FLAG_HIST if hist else 0) | (L.RLO_FLAG_PROF if prof else 0)
        cfg = L.StormCfg(seed, k, length, window, flags, log_cap, len_max, order)
        check(self.lib.rlo_program_storm(self.h, ctypes.byref(cfg)), "rlo_program_storm")

    def program_latency(self, rounds, length, seed=0x5EED, hist=False, log=False, prof=False, timeline=False):
        flags = (L.RLO_FLAG_LOG if log else 0) | (L.RLO_FLAG_HIST if hist else 0) | (L.RLO_FLAG_PROF if prof else 0)
        flags |= L.RLO_FLAG_TIMELINE if timeline else 0
        check(self.lib.rlo_program_latency(self.h, rounds, length, seed, flags), "rlo_program_latency")
        self._lat_rounds = rounds

    def program_iar(self, proposals, judge=L.RLO_JUDGE_APPROVE, mask=None, isp=None, seed=0, ppm=0, log=False,
                    log_cap=0, prof=False, pool=1):
        """proposals: list of (origin, pid, data bytes) in per-origin submission order; every rank keeps
        up to `pool` of its own in flight (the proposal pool, <= the world's proposal_pool)."""
        origin = np.array([p[0] for p in proposals], dtype=np.int32)
        pid = np.array([p[1] for p in proposals], dtype=np.int32)
        blob = np.frombuffer(b"".join(p[2] for p in proposals) or b"\0", dtype=np.uint8).copy()
        dlen = np.array([len(p[2]) for p in proposals], dtype=np.uint32)
        doff = (np.cumsum(dlen) - dlen).astype(np.uint32)
        self._keep = [origin, pid, blob, dlen, doff]
        cfg = L.IarCfg()
        cfg.judge_kind = judge
        cfg.judge_ppm = ppm
        cfg.judge_seed = seed
        if mask is not None:
            m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8))
            self._keep.append(m)
            cfg.judge_mask = m.ctypes.data
        if isp is not None:
            cfg.judge_isp = b"".join(s.encode() + b"\0" for s in isp)
            self._keep.append(cfg.judge_isp)
        cfg.flags = (L.RLO_FLAG_LOG if log else 0) | (L.RLO_FLAG_PROF if prof else 0)
        cfg.log_cap = log_cap
        cfg.pool = pool
        self._keep.append(cfg)
        d = lambda a: a.ctypes.data
        check(self.lib.rlo_program_iar(self.h, ctypes.byref(cfg), len(proposals), d(origin), d(pid), d(blob), d(doff),
                                       d(dlen)), "rlo_program_iar")

    # ------------------------------------------------------------ run
    def launch(self, stream=None, no_reset=False):
        check(self.lib.rlo_launch_ex(self.h, stream, L.RLO_LAUNCH_NO_RESET if no_reset else 0), "rlo_launch")

    def wait(self, raise_on_device_error=True):
        rc = self.lib.rlo_wait(self.h)
        if rc == L.RLO_E_DEVICE and not raise_on_device_error:
            return rc
        if rc == L.RLO_E_DEVICE:
            errs = {(self.rank_begin + r, L.DERR.get(s.error, s.error), s.error_aux)
                    for r, s in enumerate(self.stats_raw()) if s.error}
            code, aux = self.device_error()
            raise L.RloError("device engine error: %s; part error word %s aux 0x%08x" %
                             (sorted(errs)[:8], L.DERR.get(code, code), aux))
        return check(rc, "rlo_wait")

    def device_error(self):
        """(code, aux) of this part's device error word (rlo_device_error)"""
        c, a = ctypes.c_uint32(), ctypes.c_uint32()
        check(self.lib.rlo_device_error(self.h, ctypes.byref(c), ctypes.byref(a)), "rlo_device_error")
        return c.value, a.value

    def run(self, stream=None):
        """launch + wait; returns the kernel time in ms (HIP events on the launch stream)."""
        ms = ctypes.c_float()
        rc = self.lib.rlo_run(self.h, stream, ctypes.byref(ms))
        if rc == L.RLO_E_DEVICE:
            self.wait()
        check(rc, "rlo_run")
        return ms.value

    def kernel_ms(self):
        ms = ctypes.c_float()
        check(self.lib.rlo_last_kernel_ms(self.h, ctypes.byref(ms)), "rlo_last_kernel_ms")
        return ms.value

    # ------------------------------------------------------------ results
    def stats_raw(self):
        arr = (L.RankStats * self.n_local)()
        check(self.lib.rlo_stats(self.h, arr, self.n_local), "rlo_stats")
        return list(arr)

    def stats(self):
        raw = self.stats_raw()
        out = {}
        for f, _ in L.RankStats._fields_:
            if f in ("hist", "prof", "dbg"):
                out[f] = np.array([list(getattr(s, f)) for s in raw], dtype=np.uint64)
            else:
                out[f] = np.array([getattr(s, f) for s in raw], dtype=np.uint64)
        return out

    def log(self, rank, cap=1 << 16, payload=False):
        recs = (L.LogRec * cap)()
        stride = self.info["slot_stride"] - 16
        buf = np.zeros(cap * stride, dtype=np.uint8) if payload else None
        n = check(self.lib.rlo_log(self.h, rank, recs, cap, buf.ctypes.data if payload else None, stride), "rlo_log")
        rows = [(r.kind & 0xff, (r.kind >> 8) & 0xff, r.origin, r.from_, r.id, r.len, r.vote, r.aux, r.payload_idx)
                for r in recs[:n]]
        if payload:
            return rows, buf.reshape(cap, stride)
        return rows

    def latencies_ticks(self):
        arr = (ctypes.c_uint64 * self._lat_rounds)()
        n = check(self.lib.rlo_latencies(self.h, arr, self._lat_rounds), "rlo_latencies")
        return np.array(arr[:n], dtype=np.uint64)

    def round_ticks(self):
        """Clock of world rank 0 (10 ns ticks) when it saw each round complete (the part holding rank 0)."""
        arr = (ctypes.c_uint64 * self._lat_rounds)()
        n = check(self.lib.rlo_round_ticks(self.h, arr, self._lat_rounds), "rlo_round_ticks")
        return np.array(arr[:n], dtype=np.uint64)


    def timeline(self):
        """RLO_FLAG_TIMELINE rows (rlo_hip.h rlo_timeline): uint32 array [rounds][8 global + 9 x local ranks]
        of 10-ns clock values (0 = not seen on this part); the third per-rank column is the tree parent + 1."""
        stride = ctypes.c_uint32()
        check(self.lib.rlo_timeline(self.h, (ctypes.c_uint32 * 1)(), 0, ctypes.byref(stride)), "rlo_timeline")
        cap = 64 * stride.value
        arr = (ctypes.c_uint32 * cap)()
        n = check(self.lib.rlo_timeline(self.h, arr, cap, ctypes.byref(stride)), "rlo_timeline")
        return np.array(arr[:n * stride.value], dtype=np.uint32).reshape(n, stride.value)


def pool_trim(what):
    """rlo_pool_trim: give pooled device regions / idle peer imports back (rlo_hip.h RLO_TRIM_*); returns bytes freed"""
    lib = L.load()
    freed = ctypes.c_uint64()
    check(lib.rlo_pool_trim(what, ctypes.byref(freed)), "rlo_pool_trim")
    return int(freed.value)


def pool_stats():
    """rlo_pool_stats: bytes live / free / free exported / retired, imports in use / idle"""
    lib = L.load()
    out = (ctypes.c_uint64 * 6)()
    check(lib.rlo_pool_stats(out, 6), "rlo_pool_stats")
    return dict(zip(("live", "free", "free_exported", "retired", "imports_used", "imports_idle"), [int(x) for x in out]))


def hist_percentile(hist, p):
    """Percentile (in 10 ns ticks) from the device log-bucket histogram (4 sub-bins per octave)."""
    hist = np.asarray(hist, dtype=np.float64)
    tot = hist.sum()
    if tot == 0:
        return 0.0
    c = np.cumsum(hist)
    b = int(np.searchsorted(c, p / 100.0 * tot))
    if b < 4:
        return float(b)
    o, sub = b // 4 + 1, b % 4
    lo = (4 + sub) << (o - 2)
    hi = (5 + sub) << (o - 2)
    return 0.5 * (lo + hi)


def bulk_plan(n, nbytes, cross=False):
    """rlo_bulk_plan: the chunk / stripe / tile plan every rank derives for a bulk message (host
    arithmetic, no GPU)"""
    out = L.BulkPlan()
    check(L.load().rlo_bulk_plan(n, nbytes, 1 if cross else 0, ctypes.byref(out)), "rlo_bulk_plan")
    return {"nchunks": out.nchunks, "stripe": out.stripe, "chunk": out.chunk, "tile": out.tile,
            "total_tiles": out.total_tiles, "direct": out.direct}


def layout_plan(n, n_parts=1, part=0, max_payload=4096, ring_slots=0, bulk_max=0, bulk_slots=0, movers=0,
                proposal_pool=0, pend_hbm=False, cus=256):
    """rlo_layout_plan: the LDS layout (waves, nsmall, stage2_bytes, ll_ok, pend_hbm, ...) a part of this world
    would get, from host arithmetic and the build's register guarantees (no GPU)"""
    cfg = L.PlanCfg(n, n_parts, part, max_payload, ring_slots, L.RLO_PART_PEND_HBM if pend_hbm else 0, bulk_max,
                    bulk_slots, movers, proposal_pool, cus)
    out = L.WorldInfo()
    check(L.load().rlo_layout_plan(ctypes.byref(cfg), ctypes.byref(out)), "rlo_layout_plan")
    return {f: getattr(out, f) for f, _ in L.WorldInfo._fields_}


def storm_lengths(seed, k, length, len_max=0):
    """rlo_storm_lengths: the payload length of each of the storm program's k bcasts (uint32 array)"""
    out = np.zeros(max(k, 1), dtype=np.uint32)
    check(L.load().rlo_storm_lengths(seed, k, length, len_max, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))),
          "rlo_storm_lengths")
    return out[:k]


def topology(n, rank):
    lib = L.load()
    v = [ctypes.c_int() for _ in range(4)]
    sl = (ctypes.c_int * 16)()
    check(lib.rlo_topology(n, rank, *[ctypes.byref(x) for x in v], sl), "rlo_topology")
    level, lw, scc, sll = (x.value for x in v)
    return {"level": level, "last_wall": lw, "send_channel_cnt": scc, "send_list_len": sll, "send_list": list(sl[:sll])}


def children(n, rank, origin, frm):
    out = (ctypes.c_int * 16)()
    k = check(L.load().rlo_children(n, rank, origin, frm, out), "rlo_children")
    return list(out[:k])
