"""GPU parity of bulk messages -- bcasts longer than a ring slot (BASELINE configs[2]
and [4]): rootless like every bcast (the origin alone decides to send; receivers learn of it from the
announcement that travels the skip-ring tree), the bytes moved by the mover workgroups: on one GPU a
fan-out from the origin's copy into every receiver's heap (the direct plan), across GPUs a pipelined
scatter + all-gather (the chunked plan -- rehearsed here on one GPU with RLO_PART_CHUNKED).

Parity against the oracle (oracle/rlo_oracle.c orc_storm2, extended for messages beyond the
reference's 32,764-byte cap): per rank, the delivery set (bcast id, origin, tree parent of the
announcement), every delivered ring message's bytes, every bulk message's checksum
(orc_msg_checksum over the bytes the receiver holds), and the checksum of checksums.  In one part,
in two parts of one process and in separate processes (hipIpc), for the C5 workload (mixed sizes
64 B .. 1 MiB, every rank originating in every slot) at N = 16 and 64, and for fixed ragged sizes.
"""
import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu
LOG_DELIVER, TAG_BULK = 1, 10


@pytest.fixture(scope="module")
def rlo():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rlo as _rlo

    return _rlo


def _check(st, logs, n, k, lo, hi, seed, order, ring_cap):
    ref = orc.storm(n, seed, k, lo, want_parent=True, len_max=hi, order=order)
    assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
    assert np.array_equal(st["bcast_delivered"].astype(np.int64), ref["count"])
    par = ref["parent"]
    nbulk = 0
    for r in range(n):
        rows, payload = logs[r]
        got = sorted((row[4], row[2], row[3]) for row in rows if row[0] == LOG_DELIVER)
        want = sorted((b, orc.origin_of(seed, b, n, order), int(par[b, r])) for b in range(k)
                      if orc.origin_of(seed, b, n, order) != r)
        assert got == want, ("rank", r)
        for row in rows:
            kind, tag, origin, frm, bid, ln, vote, aux, pidx = row
            exp_len = orc.len_of(seed, bid, lo, hi)
            assert ln == exp_len, (r, bid, ln, exp_len)
            data = orc.payload(origin, bid, ln)
            if tag == TAG_BULK:  # the receiver's copy, by its checksum
                assert ln > ring_cap
                nbulk += 1
                assert aux | (pidx << 32) == orc.msg_checksum(origin, bid, 0, data), ("rank", r, "bid", bid, "len", ln)
            else:
                assert ln <= ring_cap
                assert bytes(payload[pidx][:ln]) == data, ("rank", r, "bid", bid)
    assert np.array_equal(st["bcast_sum"], ref["sum"])  # checksum of everything every rank picked up
    return nbulk


@pytest.mark.parametrize("n,k,order,seed", [(16, 96, 1, 5), (64, 192, 1, 7), (16, 80, 0, 9), (5, 40, 1, 2)])
def test_c5_mixed_storm_one_part(rlo, n, k, order, seed):
    lo, hi, cap = 64, 1 << 20, 4096
    with rlo.World(n, max_payload=cap, bulk_max=hi) as w:
        w.program_storm(k, lo, seed=seed, len_max=hi, order=order, log=True, log_cap=k + 8)
        w.run()
        st = w.stats()
        logs = [w.log(r, cap=k + 8, payload=True) for r in range(n)]
    nb = _check(st, logs, n, k, lo, hi, seed, order, cap)
    assert nb > 0


@pytest.mark.parametrize("n,bounds,k", [(16, [0, 8, 16], 96), (64, [0, 20, 64], 128)])
def test_c5_mixed_storm_two_parts(rlo, n, bounds, k):
    from rlo import sharded

    lo, hi, cap, seed = 64, 1 << 20, 4096, 11
    spec = {"kind": "storm", "k": k, "len": lo, "len_max": hi, "order": 1, "seed": seed, "log": True,
            "log_cap": k + 8}
    (st, logs, _), rcs = sharded.run_inprocess(n, bounds, spec, max_payload=cap, bulk_max=hi, movers=16)
    assert rcs == [0, 0], (st["error"], st["error_aux"])
    _check(st, logs, n, k, lo, hi, seed, 1, cap)


def test_c5_mixed_storm_processes(rlo):
    from rlo import sharded

    n, bounds, k, lo, hi, cap, seed = 16, [0, 8, 16], 64, 64, 1 << 20, 4096, 13
    spec = {"kind": "storm", "k": k, "len": lo, "len_max": hi, "order": 1, "seed": seed, "log": True,
            "log_cap": k + 8}
    (st, logs, _), rcs = sharded.run_processes(n, bounds, spec, max_payload=cap, bulk_max=hi, movers=8, uncached=True)
    assert rcs == [0, 0], (st["error"], st["error_aux"])
    _check(st, logs, n, k, lo, hi, seed, 1, cap)


@pytest.mark.parametrize("n,k,ln,slots", [(8, 32, (1 << 20) + 16, 2), (3, 12, 3 * (1 << 20) + 123, 1),
                                          (2, 8, 1 << 20, 2), (64, 64, 5000, 2), (8, 16, (4 << 20) + 80, 4)])
def test_bulk_fixed_sizes_checksums(rlo, n, k, ln, slots):
    """ragged fixed sizes from random originators (slot reuse: k >> slots per origin)"""
    with rlo.World(n, max_payload=64, bulk_max=ln, bulk_slots=slots) as w:
        w.program_storm(k, ln, seed=3)
        w.run()
        st = w.stats()
    exp = orc.storm_expected(n, 3, k, ln)
    assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
    assert np.array_equal(st["bcast_delivered"].astype(np.int64), exp["count"])
    assert np.array_equal(st["bcast_sum"], exp["sum"])


def test_bulk_64mib_latency_rounds(rlo):
    """C3 at one GPU: one 64 MiB bcast at a time from rotating originators; every round is delivered
    byte for byte (checksums) before the next starts"""
    n, ln, rounds = 8, 64 << 20, 6
    with rlo.World(n, max_payload=64, bulk_max=ln) as w:
        w.program_latency(rounds, ln, seed=5)
        w.run()
        st = w.stats()
        lat = w.latencies_ticks()
    org = [orc.origin_of(5, i, n) for i in range(rounds)]
    assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
    assert [int(x) for x in st["bcast_delivered"]] == [sum(o != r for o in org) for r in range(n)]
    data = {}
    want = np.zeros(n, dtype=np.uint64)
    for i, o in enumerate(org):
        cs = np.uint64(orc.msg_checksum(o, i, 0, orc.payload(o, i, ln)))
        for r in range(n):
            if r != o:
                want[r] += cs
    assert np.array_equal(st["bcast_sum"], want)
    assert (lat > 0).all()


def test_bulk_repeatable_and_world_reuse(rlo):
    """relaunching the same bulk world (flags and job rings reset) delivers the same bytes"""
    n, k = 16, 64
    with rlo.World(n, max_payload=1024, bulk_max=256 << 10) as w:
        w.program_storm(k, 64, seed=1, len_max=256 << 10, order=1)
        sums = []
        for _ in range(3):
            w.run()
            sums.append(w.stats()["bcast_sum"].copy())
    exp = orc.storm_expected(n, 1, k, 64, len_max=256 << 10, order=1)
    for s_ in sums:
        assert np.array_equal(s_, exp["sum"])


# ---- the chunked plan (scatter + all-gather, what an 8-GPU world runs), rehearsed on one GPU with
# RLO_PART_CHUNKED: every part of the world takes it although all share this GPU
@pytest.mark.parametrize("n,bounds,k", [(16, [0, 8, 16], 96), (8, [0, 3, 8], 48)])
def test_c5_mixed_storm_chunked_plan(rlo, n, bounds, k):
    from rlo import sharded

    lo, hi, cap, seed = 64, 1 << 20, 4096, 17
    spec = {"kind": "storm", "k": k, "len": lo, "len_max": hi, "order": 1, "seed": seed, "log": True,
            "log_cap": k + 8}
    (st, logs, _), rcs = sharded.run_inprocess(n, bounds, spec, max_payload=cap, bulk_max=hi, movers=16, chunked=True)
    assert rcs == [0, 0], (st["error"], st["error_aux"])
    assert _check(st, logs, n, k, lo, hi, seed, 1, cap) > 0


@pytest.mark.parametrize("ln", [(16 << 20) + 48, (36 << 20) + 5])
def test_bulk_chunked_plan_latency_rounds(rlo, ln):
    """one multi-chunk message at a time (chunks pipelined: each chunk's all-gather behind its scatter) in
    a two-part world on the chunked plan; every receiver's checksum of every round"""
    from rlo import sharded

    n, rounds, seed = 8, 4, 9
    assert rlo.bulk_plan(n, ln, True)["nchunks"] >= 2
    spec = {"kind": "lat", "rounds": rounds, "len": ln, "seed": seed}
    (st, _, _), rcs = sharded.run_inprocess(n, [0, 4, 8], spec, max_payload=64, bulk_max=ln, movers=16, chunked=True)
    assert rcs == [0, 0], (st["error"], st["error_aux"])
    org = [orc.origin_of(seed, i, n) for i in range(rounds)]
    want = np.zeros(n, dtype=np.uint64)
    for i, o in enumerate(org):
        cs = np.uint64(orc.msg_checksum(o, i, 0, orc.payload(o, i, ln)))
        for r in range(n):
            if r != o:
                want[r] += cs
    assert [int(x) for x in st["bcast_delivered"]] == [sum(o != r for o in org) for r in range(n)]
    assert np.array_equal(st["bcast_sum"], want)
