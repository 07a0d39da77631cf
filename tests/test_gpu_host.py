"""GPU parity of the host-service program (the engine under librootless_ops.so) with every
rank of the world in this process -- the rootless_ops.h state machine at 16..256 ranks.

Bcast: every rank originates through its command ring (RLO_bcast_gen, rootless_ops.c:1581);
each rank's pickup ring must deliver exactly the other ranks' messages, each once, from the
oracle's tree parent (rootless_ops.c:1104-1225), with the sent bytes.
IAR: proposals from several ranks at once, the judge a host callback (decline mask, arg !=
NULL, as tests/golden/iar.json's cases); judge calls, actions, decision pickups and own results
must equal the oracle's (rootless_ops.c:668-917), which is pinned to the reference's fixtures.
"""
import time

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rlo():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rlo as _rlo

    return _rlo


def drain(hw, until, timeout=60.0, on_event=None):
    t0 = time.time()
    while not until():
        hw.flush()
        for r in range(hw.n):
            for ev in hw.poll(r):
                on_event(r, ev)
        if time.time() - t0 > timeout:
            st = hw.stats()
            raise AssertionError("host-service world stalled: errors %s" % st["error"][st["error"] != 0][:8])


@pytest.mark.parametrize("n,k,ln,maxp", [(16, 8, 64, 256), (64, 4, 200, 256), (13, 6, 3000, 4096), (256, 1, 48, 64)])
def test_host_bcast_matches_oracle(rlo, n, k, ln, maxp):
    from rlo import abi

    trees = [orc.tree(n, o)[0] for o in range(n)]
    got = [[] for _ in range(n)]

    def on_event(r, ev):
        assert ev["kind"] == abi.RLO_EV_DELIVER_BCAST, ev
        got[r].append((ev["origin"], ev["id"], ev["from"], ev["payload"]))

    with rlo.HostWorld(n, max_payload=maxp) as hw:
        for i in range(k):
            for o in range(n):
                hw.bcast(o, orc.payload(o, o * k + i, ln), seq=o * k + i)
        drain(hw, lambda: all(len(g) == (n - 1) * k for g in got), on_event=on_event)
        time.sleep(0.05)
        for r in range(n):  # nothing beyond the expected deliveries
            assert hw.poll(r) == []
    st = hw.final_stats
    assert (st["error"] == 0).all()
    for r in range(n):
        want = sorted((o, o * k + i, int(trees[o][r]), orc.payload(o, o * k + i, ln))
                      for o in range(n) if o != r for i in range(k))
        assert sorted(got[r]) == want, r
    assert (st["bcast_delivered"] == (n - 1) * k).all()
    assert (st["originated"] == k).all()


def _run_iar(rlo, n, proposals, decline, pool=1, pend_hbm=False):
    """proposals: (origin, pid, data); at most `pool` per origin (pool 1: one own proposal per engine,
    rootless_ops.c:241; more: the proposal pool, :30 -- all submitted at once, the kernel keeps up
    to `pool` in flight and holds the rest in the command ring)."""
    from rlo import abi

    judge, actions, pickups, results = [], [], [], []
    approved = {}
    hw_ref = []

    def on_event(r, ev):
        hw = hw_ref[0]
        k = ev["kind"]
        if k == abi.RLO_EV_JUDGE:
            data = ev["payload"][16:]
            v = 0 if decline[r] else 1
            judge.append((r, ev["id"], 0, v, ev["origin"]))
            if v:
                approved[(r, ev["origin"], ev["id"])] = data
            hw.judge(r, ev, v)
        elif k == abi.RLO_EV_OWN_JUDGE:
            judge.append((r, ev["id"], 1, 1, r))
            hw.own_judge(r, ev, 1)
        elif k == abi.RLO_EV_ACTION:
            data = approved.pop((r, ev["origin"], ev["id"]))
            actions.append((r, ev["id"], 1, len(data), ev["origin"]))
        elif k == abi.RLO_EV_DELIVER_DECISION:
            pickups.append((r, ev["id"], ev["vote"], ev["origin"], 7))
        elif k == abi.RLO_EV_RESULT:
            results.append((r, ev["id"], ev["vote"]))
        else:
            raise AssertionError(ev)

    with rlo.HostWorld(n, max_payload=256, pool=pool, pend_hbm=pend_hbm) as hw:
        assert hw.world.info["pend_hbm"] == (1 if pend_hbm else hw.world.info["pend_hbm"])
        hw_ref.append(hw)
        for o, pid, data in proposals:
            hw.propose(o, pid, data)
        drain(hw, lambda: len(results) == len(proposals) and len(pickups) == len(proposals) * (n - 1),
              on_event=on_event)
    st = hw.final_stats
    assert (st["error"] == 0).all()
    assert int(st["own_decided"].sum()) == len(proposals)
    return judge, actions, pickups, results


_HOST_IAR_CASES = [(8, [1], [4], 1, 1), (8, [0, 3, 5, 6], [], 1, 1), (16, [0, 5, 9, 15], [6, 12], 1, 1),
                   (64, list(range(0, 64, 5)), [7, 33], 1, 1), (256, [0, 77, 128, 255], [3], 1, 1),
                   (8, [0, 3, 5, 6], [], 12, 4), (16, [0, 5, 9, 15], [6, 12], 20, 16), (64, list(range(0, 64, 7)), [7, 33], 6, 8)]


# every case with the pending-proposal tables in LDS; the 16- and 256-rank ones also with them in HBM
@pytest.mark.parametrize("n,origins,mask_ranks,per,pool,pend_hbm",
                         [c + (False,) for c in _HOST_IAR_CASES] + [c + (True,) for c in _HOST_IAR_CASES if c[0] in (16, 256)])
def test_host_iar_matches_oracle(rlo, n, origins, mask_ranks, per, pool, pend_hbm):
    """pend_hbm: the same with the pending-proposal tables in HBM (the 8-GPU world's layout)"""
    decline = np.zeros(n, dtype=np.uint8)
    decline[mask_ranks] = 1
    props = [(o, 1000 + i * n + o, ("proposal-%d-from-%d" % (i, o)).encode()) for i in range(per) for o in origins]
    judge, actions, pickups, results = _run_iar(rlo, n, props, decline, pool=pool, pend_hbm=pend_hbm)
    cfg, keep = orc.judge_cfg(orc.ORC_JUDGE_MASK, decline=decline)
    ev = orc.iar(n, props, cfg, pool=pool if per > 1 else 0)
    assert not [e for e in ev if e[0] == orc.ORC_EV_ERROR]
    want_j = sorted((e[1], e[2], e[3], e[4], e[5]) for e in ev if e[0] == orc.ORC_EV_JUDGE)
    want_a = sorted((e[1], e[2], e[3], e[4], e[5]) for e in ev if e[0] == orc.ORC_EV_ACTION)
    want_p = sorted((e[1], e[2], e[3], e[4], e[5]) for e in ev if e[0] == orc.ORC_EV_PICKUP)
    want_r = sorted((e[1], e[2], e[3]) for e in ev if e[0] == orc.ORC_EV_RESULT)
    assert sorted(judge) == want_j
    assert sorted(actions) == want_a
    assert sorted(pickups) == want_p
    assert sorted(results) == want_r


def test_host_relaunch_replays_nothing(rlo):
    """a relaunched host-service world must not take the previous launch's command
    doorbells for new commands.  Launch 1 posts two bcasts (doorbell slots 0 and 1 hold tags 1 and 2)
    and quits; launch 2 must deliver nothing until the host posts, then exactly what it posts."""
    import time

    n, ln = 8, 48
    with rlo.HostWorld(n, max_payload=64) as hw:
        for i, o in enumerate((0, 5)):
            assert hw.bcast(o, orc.payload(o, i, ln), seq=i)
        got = {r: [] for r in range(n)}
        t0 = time.time()
        while sum(len(v) for v in got.values()) < 2 * (n - 1) and time.time() - t0 < 20:
            for r in range(n):
                got[r] += hw.poll(r)
        assert sum(len(v) for v in got.values()) == 2 * (n - 1)
        hw.relaunch()
        time.sleep(0.3)
        for r in range(n):
            assert hw.poll(r) == [], r  # a replayed command would deliver here
        assert hw.bcast(3, orc.payload(3, 7, ln), seq=7)
        got = {r: [] for r in range(n)}
        t0 = time.time()
        while sum(len(v) for v in got.values()) < n - 1 and time.time() - t0 < 20:
            for r in range(n):
                got[r] += hw.poll(r)
        time.sleep(0.1)
        for r in range(n):
            got[r] += hw.poll(r)
            if r == 3:
                assert got[r] == [], got[r]
            else:
                assert [(e["origin"], e["id"], e["payload"][:ln]) for e in got[r]] == [(3, 7, orc.payload(3, 7, ln))], r
