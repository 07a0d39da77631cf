"""Worlds created with RLO_PART_ONE_XCD (rlo_hip.h): cached rings, every rank-wave of the hop kernel on one XCD, plain
hand-off stores kept in that XCD's L2 (rlo_hop.hip LOC).  The same parity bar as the default worlds' latency and
one-proposal IAR tests (test_gpu_engine.py, test_gpu_scale.py), over several launches of one world (a line an earlier
launch left in the L2 must never be read as this launch's), and the flag's limits."""
import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu

LOG_DELIVER = 1


@pytest.fixture(scope="module")
def rlo():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rlo as _rlo

    return _rlo


@pytest.mark.parametrize("n,ln,maxp", [(4, 64, 64), (8, 64, 64), (8, 112, 112), (13, 100, 112), (32, 64, 64), (8, 1, 64),
                                        (64, 64, 64), (128, 48, 64), (256, 64, 64)])
def test_one_xcd_latency_program(rlo, n, ln, maxp):
    rounds, seed = 64, 5
    ref = orc.storm(n, seed, rounds, ln, want_parent=True)
    with rlo.World(n, max_payload=maxp, one_xcd=True) as w:
        for rep in range(3):
            w.program_latency(rounds, ln, seed=seed)
            w.run()
            assert w.info_now()["last_kernel"] == 1  # the hop kernel
            st = w.stats()
            lat = w.latencies_ticks()
            assert (st["error"] == 0).all(), (rep, st["error"], st["error_aux"])
            assert len(lat) == rounds and (lat > 0).all()
            assert np.array_equal(st["bcast_delivered"].astype(np.int64), ref["count"]), rep
            assert np.array_equal(st["bcast_sum"], ref["sum"]), rep
        w.program_latency(rounds, ln, seed=seed, log=True)
        w.run()
        st2 = w.stats()
        logs = [w.log(r, cap=rounds + 8, payload=True) for r in range(n)]
    assert (st2["error"] == 0).all()
    for r in range(n):
        rows, payload = logs[r]
        got = sorted((row[4], row[2], row[3]) for row in rows if row[0] == LOG_DELIVER)
        want = sorted((b, orc.origin_of(seed, b, n), int(ref["parent"][b, r])) for b in range(rounds)
                      if orc.origin_of(seed, b, n) != r)
        assert got == want, r
        for row in rows:
            assert row[5] == ln and bytes(payload[row[8]][:ln]) == orc.payload(row[2], row[4], ln), (r, row)


@pytest.mark.parametrize("n,p,ppm", [(8, 64, 20000), (16, 24, 3400), (5, 48, 0), (4, 40, 50000)])
def test_one_xcd_iar_exact_sets(rlo, n, p, ppm):
    """One own proposal per rank (the reference's my_own_proposal, rootless_ops.c:241), seeded declines: the
    judge-call, action, decision-pickup and result sets against the oracle, on every one of three launches"""
    import iar_sets

    kind = rlo.abi.RLO_JUDGE_HASH if ppm else rlo.abi.RLO_JUDGE_APPROVE
    cap = 3 * n * p + 64
    with rlo.World(n, max_payload=32, one_xcd=True) as w:
        for rep in range(3):
            w.program_iar(iar_sets.props(n, p), judge=kind, seed=99, ppm=ppm, log=True, log_cap=cap, pool=1)
            w.run()
            assert w.info_now()["last_kernel"] == 1
            st = w.stats()
            logs = {r: w.log(r, cap=cap) for r in range(n)}
            assert (st["error"] == 0).all(), (rep, st["error"], st["error_aux"])
            iar_sets.check(logs, n, p, ppm, 1)


def test_one_xcd_limits(rlo):
    """Only the hop kernel's programs run in a ONE_XCD world: a storm (the progress kernel, whose rank-workgroups
    spread over every XCD and would read the cached rings through other L2s) is refused at launch, not run; worlds
    of more than 256 ranks, or with bulk messages, are refused at creation"""
    with rlo.World(8, max_payload=64, one_xcd=True) as w:
        w.program_storm(64, 64, seed=3)
        with pytest.raises(Exception):
            w.run()
        w.program_latency(16, 64, seed=1)  # the world stays usable for the programs it runs
        w.run()
        assert (w.stats()["error"] == 0).all()
    with pytest.raises(Exception):
        rlo.World(257, max_payload=64, one_xcd=True)
    with pytest.raises(Exception):
        rlo.World(8, max_payload=64, bulk_max=1 << 20, one_xcd=True)
