"""ctypes view of liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / CPU baseline.  The product path never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

ORC_JUDGE_APPROVE, ORC_JUDGE_MASK, ORC_JUDGE_ISP, ORC_JUDGE_HASH = 0, 1, 2, 3
ORC_EV_JUDGE, ORC_EV_ACTION, ORC_EV_PICKUP, ORC_EV_RESULT, ORC_EV_ERROR = 1, 2, 3, 4, 5  # rlo_oracle.h
EV_JUDGE, EV_ACTION, EV_PICKUP, EV_RESULT, EV_ERROR = 1, 2, 3, 4, 5


class JudgeCfg(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("decline", ctypes.c_void_p), ("isp", ctypes.c_char_p),
                ("seed", ctypes.c_uint64), ("ppm", ctypes.c_uint32)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        ip = ctypes.POINTER(ctypes.c_int)
        L.orc_topology.argtypes = [ctypes.c_int, ctypes.c_int, ip, ip, ip, ip, ip]
        L.orc_children.argtypes = [ctypes.c_int] * 4 + [ip]
        L.orc_fwd_send_cnt.argtypes = [ctypes.c_int] * 4
        L.orc_check_passed_origin.argtypes = [ctypes.c_int] * 4
        L.orc_tree.argtypes = [ctypes.c_int, ctypes.c_int, i32p]
        L.orc_payload.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.orc_origin_of.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_origin_of.restype = ctypes.c_uint32
        L.orc_chunk_mix.argtypes = [ctypes.c_uint32] * 5
        L.orc_chunk_mix.restype = ctypes.c_uint32
        L.orc_msg_checksum.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
        L.orc_msg_checksum.restype = ctypes.c_uint64
        L.orc_region_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_region_hash.restype = ctypes.c_uint64
        L.orc_fnv1a.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_fnv1a.restype = ctypes.c_uint64
        L.orc_storm.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32, i32p, i64p, u64p]
        L.orc_storm.restype = ctypes.c_int64
        L.orc_storm_expected.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32, i64p, u64p]
        L.orc_storm_expected.restype = ctypes.c_int64
        u32 = ctypes.c_uint32
        L.orc_storm2.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, u32, u32, u32, i32p, i64p, u64p]
        L.orc_storm2.restype = ctypes.c_int64
        L.orc_storm_mt.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, u32, u32, u32, ctypes.c_int, i64p,
                                   u64p]
        L.orc_storm_mt.restype = ctypes.c_int64
        L.orc_iar_rounds.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, i32p, ctypes.c_int]
        L.orc_iar_rounds.restype = ctypes.c_int
        L.orc_storm_expected2.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, u32, u32, u32, i64p, u64p]
        L.orc_storm_expected2.restype = ctypes.c_int64
        L.orc_len_of.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u32, u32]
        L.orc_len_of.restype = u32
        L.orc_origin_of2.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u32, u32]
        L.orc_origin_of2.restype = u32
        L.orc_judge_hash.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32]
        L.orc_judge_hash.restype = ctypes.c_uint32
        L.orc_iar.argtypes = [ctypes.c_int, ctypes.c_int, i32p, i32p, ctypes.c_char_p, i32p, i32p, ctypes.POINTER(JudgeCfg),
                              i32p, ctypes.c_int]
        L.orc_iar_pool.argtypes = [ctypes.c_int, ctypes.c_int, i32p, i32p, ctypes.c_char_p, i32p, i32p,
                                   ctypes.POINTER(JudgeCfg), ctypes.c_int, i32p, ctypes.c_int]
        L.orc_iar_pool.restype = ctypes.c_int
        L.orc_iar_rounds_pool.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, i32p, ctypes.c_int]
        L.orc_iar_rounds_pool.restype = ctypes.c_int
        L.orc_iar_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(JudgeCfg), i64p, i64p, i64p]
        L.orc_iar_bench.restype = ctypes.c_int64
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t)) if a is not None else None


def topology(n, rank):
    L = lib()
    v = [ctypes.c_int() for _ in range(4)]
    sl = (ctypes.c_int * 32)()
    if L.orc_topology(n, rank, *[ctypes.byref(x) for x in v], sl) != 0:
        raise ValueError("bad topology args")
    level, lw, scc, sll = (x.value for x in v)
    return {"level": level, "last_wall": lw, "send_channel_cnt": scc, "send_list_len": sll, "send_list": list(sl[:sll])}


def children(n, rank, origin, frm):
    out = (ctypes.c_int * 32)()
    k = lib().orc_children(n, rank, origin, frm, out)
    return list(out[:k])


def tree(n, origin):
    parent = np.full(n, -1, dtype=np.int32)
    cnt = lib().orc_tree(n, origin, _p(parent, ctypes.c_int32))
    return parent, cnt


def payload(origin, bid, length):
    buf = ctypes.create_string_buffer(max(length, 1))
    lib().orc_payload(origin, bid, buf, length)
    return buf.raw[:length]


def origin_of(seed, bid, n, order=0):
    """origin of bcast bid: order 0 random (splitmix64(seed + bid) % n), 1 slots (bid % n)"""
    return lib().orc_origin_of2(seed, bid, n, order)


def len_of(seed, bid, lo, hi):
    """payload bytes of bcast bid in a mixed-size storm (rlo_testvec.h rlo_tv_len)"""
    return lib().orc_len_of(seed, bid, lo, hi)


def msg_checksum(origin, bid, tag, data):
    return lib().orc_msg_checksum(origin, bid, tag, data, len(data))


def region_hash(data):
    return lib().orc_region_hash(data, len(data))


def fnv1a(data):
    return lib().orc_fnv1a(data, len(data))


def storm(n, seed, k, length, want_parent=False, len_max=0, order=0):
    parent = np.full(k * n, -1, dtype=np.int32) if want_parent else None
    count = np.zeros(n, dtype=np.int64)
    ssum = np.zeros(n, dtype=np.uint64)
    d = lib().orc_storm2(n, seed, k, length, max(length, len_max), order, _p(parent, ctypes.c_int32),
                         _p(count, ctypes.c_int64), _p(ssum, ctypes.c_uint64))
    if d < 0:
        raise RuntimeError("oracle storm failed")
    return {"deliveries": d, "count": count, "sum": ssum, "parent": parent.reshape(k, n) if want_parent else None}


def storm_mt(n, seed, k, length, threads, len_max=0, order=0):
    """orc_storm_mt: the storm on `threads` host threads (count / sum as storm())."""
    count = np.zeros(n, dtype=np.int64)
    ssum = np.zeros(n, dtype=np.uint64)
    d = lib().orc_storm_mt(n, seed, k, length, max(length, len_max), order, threads, _p(count, ctypes.c_int64),
                           _p(ssum, ctypes.c_uint64))
    if d < 0:
        raise RuntimeError("oracle storm_mt failed")
    return {"deliveries": d, "count": count, "sum": ssum}


def storm_expected(n, seed, k, length, len_max=0, order=0):
    count = np.zeros(n, dtype=np.int64)
    ssum = np.zeros(n, dtype=np.uint64)
    d = lib().orc_storm_expected2(n, seed, k, length, max(length, len_max), order, _p(count, ctypes.c_int64),
                                  _p(ssum, ctypes.c_uint64))
    return {"deliveries": d, "count": count, "sum": ssum}


def judge_cfg(kind=ORC_JUDGE_APPROVE, decline=None, isp=None, seed=0, ppm=0):
    """Returns (cfg, keepalive) -- keep the second element alive while cfg is used."""
    keep = []
    cfg = JudgeCfg()
    cfg.kind = kind
    if decline is not None:
        arr = np.ascontiguousarray(np.asarray(decline, dtype=np.uint8))
        keep.append(arr)
        cfg.decline = arr.ctypes.data
    if isp is not None:
        blob = b"".join(s.encode() + b"\0" for s in isp)
        keep.append(blob)
        cfg.isp = blob
    cfg.seed = seed
    cfg.ppm = ppm
    return cfg, keep


def iar(n, proposals, cfg, cap=1 << 16, pool=0):
    """proposals: list of (origin, pid, data bytes).  Returns list of event tuples.  pool 0: all
    submitted up front (orc_iar, the reference's one my_own_proposal); pool >= 1: the proposal pool
    (orc_iar_pool, every origin keeps up to `pool` in flight, list order)."""
    origin = np.array([p[0] for p in proposals], dtype=np.int32)
    pid = np.array([p[1] for p in proposals], dtype=np.int32)
    blob = b"".join(p[2] for p in proposals)
    off = np.cumsum([0] + [len(p[2]) for p in proposals[:-1]]).astype(np.int32)
    dl = np.array([len(p[2]) for p in proposals], dtype=np.int32)
    ev = np.zeros(6 * cap, dtype=np.int32)
    if pool:
        k = lib().orc_iar_pool(n, len(proposals), _p(origin, ctypes.c_int32), _p(pid, ctypes.c_int32), blob,
                               _p(off, ctypes.c_int32), _p(dl, ctypes.c_int32), ctypes.byref(cfg), pool,
                               _p(ev, ctypes.c_int32), cap)
    else:
        k = lib().orc_iar(n, len(proposals), _p(origin, ctypes.c_int32), _p(pid, ctypes.c_int32), blob,
                          _p(off, ctypes.c_int32), _p(dl, ctypes.c_int32), ctypes.byref(cfg), _p(ev, ctypes.c_int32), cap)
    if k < 0:
        raise RuntimeError("oracle iar failed")
    return [tuple(int(x) for x in ev[6 * i:6 * i + 6]) for i in range(k)]


def iar_rounds(n, p, cfg, cap=None, pool=1):
    """orc_iar_rounds_pool: iar_bench's workload (`pool` outstanding proposals per rank, pid = it * n + r)
    with every event: list of (ev, rank, pid, a, b, c)"""
    cap = cap or 4 * n * n * p + 1024
    ev = np.zeros(6 * cap, dtype=np.int32)
    k = lib().orc_iar_rounds_pool(n, p, pool, ctypes.byref(cfg), _p(ev, ctypes.c_int32), cap)
    if k < 0:
        raise RuntimeError("oracle iar_rounds failed")
    return [tuple(int(x) for x in r) for r in ev[:6 * k].reshape(k, 6)]


def iar_bench(n, p, cfg):
    a, j, ac = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    d = lib().orc_iar_bench(n, p, ctypes.byref(cfg), ctypes.byref(a), ctypes.byref(j), ctypes.byref(ac))
    return {"decisions": d, "approved": a.value, "judge_calls": j.value, "actions": ac.value}
