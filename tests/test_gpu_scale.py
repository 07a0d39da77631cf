"""The 8-GPU world's layout on the GPU (VERDICT r3 "next" 1).

bench.py --gpus 8 builds ONE world of 2,048 ranks, 256 per part.  Every part of it is created here on
the one GPU of the box (allocation and LDS sizing only: a part's kernel needs every peer part running
to launch) and its layout checked against the host plan (rlo_layout_plan, tests/test_layout_plan.py):
8 waves, the whole 64-B slot staged (nsmall 5), doorbells on, pending-proposal tables in HBM.

The HBM tables' own code path (the PH instantiations of rlo_progress_kernel, run by every iar / host
program of such a world) is parity-tested at smaller N by forcing the layout (RLO_PART_PEND_HBM): IAR
exact sets per (origin, pid) against the pool oracle, in one part and in parts; the host-service path in
tests/test_gpu_host.py (pend_hbm cases).
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rlo():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rlo as _rlo

    return _rlo


KEYS = ("waves", "nsmall", "ll_ok", "pend_hbm", "rank_begin", "rank_end", "proposal_pool")


@pytest.mark.parametrize("n,parts", [(2048, 8), (1024, 4), (512, 2)])
def test_bench_world_parts_layout(rlo, n, parts):
    for p in (0, parts // 2, parts - 1):
        with rlo.World.part(n, parts, p, max_payload=64, device=0, uncached=True) as w:
            got = {k: w.info[k] for k in KEYS}
        plan = rlo.layout_plan(n, parts, p, max_payload=64, cus=w.info["cus"])
        assert got == {k: plan[k] for k in KEYS}, (got, plan)
        assert got["waves"] == 8 and got["nsmall"] == 5 and got["ll_ok"] == 1, got
        assert got["pend_hbm"] == (1 if n == 2048 else 0)


def test_c5_world_part_at_8_gpus(rlo):
    """bench.py's C5 leg at 8 GPUs: 512 ranks, bulk messages to 1 MiB (was refused: N x B > 256); the host plan
    (rlo_layout_plan) agrees with what the part got on the GPU (the bulk variant's model)"""
    kw = dict(max_payload=4096, bulk_max=1 << 20)
    with rlo.World.part(512, 8, 3, device=0, uncached=True, **kw) as w:
        got = {k: w.info[k] for k in KEYS + ("bulk_slots",)}
    assert got["bulk_slots"] == 2 and got["nsmall"] == 5 and got["waves"] == 4
    plan = rlo.layout_plan(512, 8, 3, cus=w.info["cus"], **kw)
    assert got == {k: plan[k] for k in got}, (got, plan)


@pytest.mark.parametrize("n,payload,pend_hbm", [(320, 256, False), (384, 1024, False), (300, 64, True)])
def test_four_wave_parts_plan_matches(rlo, n, payload, pend_hbm):
    """4-wave parts with more local ranks than CUs (two rank-workgroups per CU: doorbells only where the 4-wave
    LL instantiation keeps 2 waves per SIMD), medium and large slots, LDS and HBM tables: the host plan agrees
    with the part the GPU built (waves, staged chunks, doorbells, table placement)"""
    with rlo.World(n, max_payload=payload, device=0, pend_hbm=pend_hbm) as w:
        got = {k: w.info[k] for k in KEYS}
    plan = rlo.layout_plan(n, max_payload=payload, pend_hbm=pend_hbm, cus=w.info["cus"])
    assert got == {k: plan[k] for k in KEYS}, (got, plan)
    assert got["waves"] == 4 and (got["pend_hbm"] == 1 or not pend_hbm)


@pytest.mark.parametrize("n,p,ppm,pool", [(256, 4, 201, 1), (256, 8, 201, 16), (64, 16, 50000, 4), (8, 64, 20000, 16),
                                          (5, 48, 0, 8),
                                          # one own proposal in worlds of <= 16 ranks: the hop kernel's PH instantiation
                                          (8, 64, 20000, 1), (16, 24, 3400, 1)])
def test_iar_exact_sets_hbm_tables(rlo, n, p, ppm, pool):
    """the PH instantiation: pending entries in HBM, exact sets per (origin, pid) vs the pool oracle"""
    import iar_sets

    kind = rlo.abi.RLO_JUDGE_HASH if ppm else rlo.abi.RLO_JUDGE_APPROVE
    cap = 3 * n * p + 64
    with rlo.World(n, max_payload=32, proposal_pool=max(2, pool), pend_hbm=True) as w:
        assert w.info["pend_hbm"] == 1
        w.program_iar(iar_sets.props(n, p), judge=kind, seed=99, ppm=ppm, log=True, log_cap=cap, pool=pool)
        w.run()
        st = w.stats()
        kernel = w.info_now()["last_kernel"]
        logs = {r: w.log(r, cap=cap) for r in range(n)}
    assert (st["error"] == 0).all(), (st["error"], st["error_aux"])
    assert kernel == (1 if pool == 1 and n <= 16 else 0), kernel  # 1: the hop kernel (rlo_hop.hip)
    iar_sets.check(logs, n, p, ppm, pool)


def test_iar_hbm_tables_relaunch_and_storm(rlo):
    """a world with HBM tables runs its storm on the LDS-free instantiation and its iar on the PH one,
    back to back and relaunched (the table is zeroed by every PH launch)"""
    import numpy as np

    import iar_sets
    import pyoracle as orc

    n, p, k, seed = 64, 6, 4096, 13
    with rlo.World(n, max_payload=64, proposal_pool=2, pend_hbm=True) as w:
        for _ in range(2):
            w.program_storm(k, 64, seed=seed)
            w.run()
            st = w.stats()
            ref = orc.storm(n, seed, k, 64)
            assert (st["error"] == 0).all()
            assert np.array_equal(st["bcast_sum"], ref["sum"])
            cap = 3 * n * p + 64
            w.program_iar(iar_sets.props(n, p), judge=rlo.abi.RLO_JUDGE_HASH, seed=99, ppm=814, log=True, log_cap=cap)
            w.run()
            st = w.stats()
            assert (st["error"] == 0).all()
            iar_sets.check({r: w.log(r, cap=cap) for r in range(n)}, n, p, 814, 1)


@pytest.mark.parametrize("n,bounds,p,ppm,pool", [(64, [0, 20, 64], 8, 814, 1), (64, [0, 32, 64], 24, 814, 16)])
def test_iar_sharded_hbm_tables(rlo, n, bounds, p, ppm, pool):
    """C4 across parts with the 8-GPU layout's tables"""
    import iar_sets
    from rlo import sharded

    cap = 3 * n * p + 64
    spec = {"kind": "iar", "props": iar_sets.props(n, p), "judge": rlo.abi.RLO_JUDGE_HASH, "seed": 99, "ppm": ppm,
            "log": True, "log_cap": cap, "pool": pool}
    (st, logs, _), rcs = sharded.run_inprocess(n, bounds, spec, max_payload=32, proposal_pool=max(2, pool),
                                               uncached=True, pend_hbm=True)
    assert rcs == [0] * (len(bounds) - 1), (st["error"], st["error_aux"])
    iar_sets.check(logs, n, p, ppm, pool)
