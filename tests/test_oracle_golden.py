"""The CPU restatement (oracle/) pinned against vectors captured from the compiled reference.

Fixtures come from tests/golden/gen_fixtures.py (runs oracle/_ref/ref_harness, i.e. the
reference's rootless_ops.c compiled in place, under MPICH).  Every assertion here is
bit-exact: topology integers, tree parents, FNV hashes of the delivered 32,764-byte data
region, judge-call sets, decisions, action arguments and user-visible pickups.
"""
import numpy as np
import pytest

import pyoracle as orc


def test_topology_levels_and_walls(golden):
    fx = golden("topo.json")
    nmax = fx["nmax"]
    for n in range(2, nmax + 1):
        assert orc.topology(n, 0)["level"] == fx["level0"][n - 2], n
    for r in range(1, nmax):
        t = orc.topology(nmax, r)
        assert t["level"] == fx["level"][r], r
        assert t["last_wall"] == fx["last_wall_fn"][r], r


def test_topology_rank0_last_wall_is_pow2_level():
    # rootless_ops.c:1478-1479: rank 0 uses pow(2, level), not last_wall()
    for n in (2, 3, 4, 5, 8, 13, 256, 257):
        t = orc.topology(n, 0)
        assert t["last_wall"] == 1 << t["level"]


def test_parent_trees_match_reference(golden):
    fx = golden("parents.json")
    assert fx["len"] == 64
    for ns, case in fx["by_n"].items():
        n = int(ns)
        for o in range(n):
            parent, cnt = orc.tree(n, o)
            assert cnt == n - 1, (n, o)
            assert parent.tolist() == case["parent"][o], (n, o)
            want = "%016x" % orc.region_hash(orc.payload(o, o, 64))
            assert case["hash"][o] == want, (n, o)


def test_stream_deliveries_match_reference(golden):
    for case in golden("stream.json")["cases"]:
        n, seed, k, ln = case["n"], case["seed"], case["k"], case["len"]
        res = orc.storm(n, seed, k, ln, want_parent=True)
        par = res["parent"]
        for r in range(n):
            got = []
            for b in range(k):
                o = orc.origin_of(seed, b, n)
                if o == r:
                    assert par[b, r] == -1
                    continue
                got.append([b, o, int(par[b, r]), "%016x" % orc.region_hash(orc.payload(o, b, ln))])
            assert sorted(got) == case["deliveries"][r], (n, r)
            assert res["count"][r] == len(got)


def test_storm_simulation_equals_analytic_checksums():
    for n, k, ln in ((4, 300, 64), (13, 200, 100), (64, 100, 4096), (256, 64, 8)):
        sim = orc.storm(n, 77, k, ln)
        exp = orc.storm_expected(n, 77, k, ln)
        assert sim["deliveries"] == exp["deliveries"] == k * (n - 1)
        assert np.array_equal(sim["count"], exp["count"])
        assert np.array_equal(sim["sum"], exp["sum"])


@pytest.mark.parametrize("n,k,lo,hi,order,threads", [(256, 3000, 64, 64, 0, 8), (7, 400, 64, 5000, 0, 4),
                                                     (16, 120, 64, 1 << 20, 1, 3), (3, 50, 64, 64, 0, 16)])
def test_storm_threaded_equals_single_thread(n, k, lo, hi, order, threads):
    """bench.py's multi-core cpu_baseline restatement delivers exactly what the single-thread one does"""
    a = orc.storm(n, 5, k, lo, len_max=hi, order=order)
    b = orc.storm_mt(n, 5, k, lo, threads, len_max=hi, order=order)
    assert a["deliveries"] == b["deliveries"] == k * (n - 1)
    assert np.array_equal(a["count"], b["count"]) and np.array_equal(a["sum"], b["sum"])


@pytest.mark.parametrize("n,p,ppm", [(8, 5, 0), (16, 3, 50000), (64, 2, 814)])
def test_iar_rounds_events_agree_with_totals(n, p, ppm):
    """orc_iar_rounds (the exact-set checker of tests/test_gpu_engine.py) records the same workload
    orc_iar_bench counts: one result per proposal, judge calls / actions / approvals equal, every
    non-origin rank picks up every decision"""
    kind = orc.ORC_JUDGE_HASH if ppm else orc.ORC_JUDGE_APPROVE
    cfg, keep = orc.judge_cfg(kind, seed=7, ppm=ppm)
    ev = orc.iar_rounds(n, p, cfg)
    tot = orc.iar_bench(n, p, cfg)
    res = [e for e in ev if e[0] == orc.ORC_EV_RESULT]
    assert len(res) == tot["decisions"] == n * p
    assert sum(1 for e in res if e[3] == 1) == tot["approved"]
    assert sum(1 for e in ev if e[0] == orc.ORC_EV_JUDGE) == tot["judge_calls"]
    assert sum(1 for e in ev if e[0] == orc.ORC_EV_ACTION) == tot["actions"]
    assert sum(1 for e in ev if e[0] == orc.ORC_EV_PICKUP) == (n - 1) * n * p
    assert sorted(e[2] for e in res) == sorted(it * n + r for it in range(p) for r in range(n))


@pytest.mark.parametrize("n,p,ppm,pool", [(8, 12, 0, 4), (16, 6, 50000, 16), (64, 3, 814, 8), (5, 20, 20000, 16)])
def test_iar_pool_outcomes_equal_single_proposal_rounds(n, p, ppm, pool):
    """the proposal pool (rootless_ops.c:30, :1251-1366) changes when a proposal runs, not what happens
    to it: orc_iar_rounds_pool's per-(origin, pid) judge calls, actions, decision pickups and results
    equal orc_iar_rounds' (pool 1, the reference's one my_own_proposal, which the golden IAR cases pin)"""
    kind = orc.ORC_JUDGE_HASH if ppm else orc.ORC_JUDGE_APPROVE
    cfg, keep = orc.judge_cfg(kind, seed=7, ppm=ppm)
    one = orc.iar_rounds(n, p, cfg)
    many = orc.iar_rounds(n, p, cfg, pool=pool)
    assert len(many) == len(one) and set(many) == set(one)
    assert not [e for e in many if e[0] == orc.ORC_EV_ERROR]


def test_iar_pool_one_per_origin_equals_reference_model(golden):
    """with at most one proposal per origin the pool oracle is orc_iar, case for case (iar.json)"""
    for case in golden("iar.json")["cases"]:
        n, o, mask = case["n"], case["origin"], case["mask"]
        cfg, keep = orc.judge_cfg(orc.ORC_JUDGE_MASK, decline=[(mask >> r) & 1 for r in range(n)])
        props = [(o, 100 + o, ("proposal-from-%d" % o).encode())]
        assert orc.iar(n, props, cfg, pool=4) == orc.iar(n, props, cfg)


def _iar_events(n, origin, mask):
    cfg, keep = orc.judge_cfg(orc.ORC_JUDGE_MASK, decline=[(mask >> r) & 1 for r in range(n)])
    prop = ("proposal-from-%d" % origin).encode()
    return orc.iar(n, [(origin, 100 + origin, prop)], cfg), prop


def test_iar_single_proposal_matches_reference(golden):
    for case in golden("iar.json")["cases"]:
        n, o, mask = case["n"], case["origin"], case["mask"]
        ev, prop = _iar_events(n, o, mask)
        judge = sorted([e[1], e[3], "" if e[3] else prop.decode()] for e in ev if e[0] == orc.EV_JUDGE)
        assert judge == case["judge"], case
        res = [e for e in ev if e[0] == orc.EV_RESULT]
        assert len(res) == 1 and res[0][1] == o and res[0][3] == case["decision"]
        actions = sorted([e[1], e[2], e[3], e[4], prop.decode()] for e in ev if e[0] == orc.EV_ACTION)
        assert actions == case["actions"], case
        pickups = sorted([e[1], 4, e[2], e[3], e[5], "IAR_DEC", e[4]] for e in ev if e[0] == orc.EV_PICKUP)
        assert pickups == case["pickups"], case
        assert not [e for e in ev if e[0] == orc.EV_ERROR]


def test_iar_multi_proposal_matches_reference(golden):
    for case in golden("multi.json")["cases"]:
        n, a1, mod, agree = case["n"], case["active_1"], case["mod"], case["agree"]
        isp, props = [], []
        for r in range(n):  # roles of testcases.c:417-469
            if r == a1:
                isp.append("555"); props.append((r, r, b"555"))
            elif r % mod == 0:
                s = "555" if agree else "333"
                isp.append(s); props.append((r, r, s.encode()))
            else:
                isp.append("555" if agree else "111")
        cfg, keep = orc.judge_cfg(orc.ORC_JUDGE_ISP, isp=isp)
        ev = orc.iar(n, props, cfg)
        pdata = {pid: d.decode() for (_, pid, d) in props}
        judge = sorted([e[1], e[3], "" if e[3] else pdata[e[2]], e[4]] for e in ev if e[0] == orc.EV_JUDGE)
        assert judge == case["judge"], case
        dec = sorted([e[1], e[2], e[3], e[4]] for e in ev if e[0] == orc.EV_PICKUP)
        assert dec == case["decisions"], case
        res = sorted([e[1], e[2], e[3]] for e in ev if e[0] == orc.EV_RESULT)
        assert res == case["results"], case


def test_reference_testcases_passed(golden):
    # the reference's own wrappers (testcases.c:699-740, :243, :401) passed at N=4
    fx = golden("testcases.json")
    assert fx["results"] and all(r["ret"] == 1 for r in fx["results"])


def test_hacky_sack_invariant_oracle():
    # testcases.c:691-692: every rank picks up (sent+1)*(ws-1) messages -- exact-once delivery
    for n in (2, 3, 4, 7, 8):
        for o in range(n):
            parent, cnt = orc.tree(n, o)
            assert cnt == n - 1 and parent[o] == -1 and (parent[np.arange(n) != o] >= 0).all()


@pytest.mark.parametrize("n", list(range(2, 130)) + [255, 256, 257, 512, 1000, 1024])
def test_exact_spanning_tree_property(n):
    # every origin yields an exact spanning tree (N-1 edges, no self delivery)
    for o in range(n) if n <= 64 else range(0, n, max(1, n // 16)):
        parent, cnt = orc.tree(n, o)
        assert cnt == n - 1
