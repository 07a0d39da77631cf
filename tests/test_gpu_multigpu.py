"""Multi-GPU readiness on a one-GPU box: the 8-GPU runs are the driver's, so the
N-part path is exercised here the way it runs there.

  * a part whose peer sits on another GPU (its exported blob names another PCI bus) switches to
    system scope (rings and heaps are uncached in every world, so peers may store into them over xGMI);
  * bench.py --gpus 2 under torch.distributed.run (gloo control plane, both ranks on this GPU via
    RLO_BENCH_DEVICE): one 128-rank world in two parts -- the storm, latency, decisions, rootless bulk
    and mixed-size legs of the driver's multi-GPU run, each part's per-rank statistics (bench.py
    --dump) compared with the oracle: delivery counts and checksums per world rank, bulk checksums per
    round, decision totals.
"""
import json
import os
import shutil
import re
import signal
import subprocess
import sys
import tempfile

import numpy as np
import pytest

import pyoracle as orc
from rlo import _lib as L

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rlo():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rlo as _rlo

    return _rlo


def _forge_bus(blob):
    m = re.search(rb"[0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-9]", blob)
    assert m, "no PCI bus id in the exported blob"
    return blob[:m.start()] + b"ffff:ff:1f.7" + blob[m.end():]


def test_cross_gpu_peer_switches_to_system_scope(rlo):
    n = 8
    w0 = rlo.World.part(n, 2, 0, max_payload=64, uncached=True)
    w1 = rlo.World.part(n, 2, 1, max_payload=64, uncached=True)
    try:
        b0, b1 = w0.export(), w1.export()
        w0.connect([b0, _forge_bus(b1)])  # part 1 "on another GPU"
        w1.connect([b0, b1])
        assert w0.info["sys_scope"] == 1 and w0.info["peers"] == L.RLO_PEER_OTHER_GPU
        assert w1.info["sys_scope"] == 0 and w1.info["peers"] == 0  # same GPU, same process
    finally:
        w0.close()
        w1.close()


def test_bulk_cross_gpu_path_system_scope(rlo):
    """the bulk leg of the 8-GPU run, on one GPU: both parts see the other "on another GPU" (forged bus), so
    both run system scope AND the chunked plan (scatter + all-gather, system-scope releases and flags) --
    every receiver's checksum of every 16-MiB round equals the oracle's"""
    from rlo import sharded

    n, rounds, seed, ln = 4, 4, 21, (16 << 20) + 32

    def forge(p, blobs):
        return [b if q == p else _forge_bus(b) for q, b in enumerate(blobs)]

    spec = {"kind": "lat", "rounds": rounds, "len": ln, "seed": seed}
    (st, _, _), rcs = sharded.run_inprocess(n, [0, 2, 4], spec, max_payload=64, bulk_max=ln, movers=16, uncached=True,
                                            blobs_for=forge)
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


def test_bulk_world_churn_processes(rlo):
    """VERDICT r3 "next" 8, the round-2 rehearsal hang: a part's bulk leg failed within 0.1 s of its
    creation.  Of the three suspects only the world's allocation and hipIpc export / import can fail that
    fast (a resident kernel elsewhere on the GPU never fails a creation -- it makes a launch wait; the bench
    legs use no shared-memory names), and what differs between legs is exactly their churn: every leg
    creates, exports, maps, runs and destroys its world again, in both processes.  Here two part processes
    do that 6 times in a row with the bulk leg's world (uncached heaps, IPC-mapped across processes), then
    6 times with a 16-rank storm world, and every repeat must map and deliver the oracle's bytes"""
    from rlo import sharded

    n, rounds, seed, ln = 4, 4, 33, (1 << 20) + 48
    spec = {"kind": "lat", "rounds": rounds, "len": ln, "seed": seed}
    runs = sharded.run_processes(n, [0, 2, 4], spec, max_payload=64, bulk_max=ln, movers=16, uncached=True, repeat=6)
    org = [orc.origin_of(seed, i, n) for i in range(rounds)]
    want = np.zeros(n, dtype=np.uint64)
    for i, o in enumerate(org):
        cs = np.uint64(orc.msg_checksum(o, i, 0, orc.payload(o, i, ln)))
        for r in range(n):
            if r != o:
                want[r] += cs
    for it, ((st, _, _), rcs) in enumerate(runs):
        assert rcs == [0, 0], (it, st["error"], st["error_aux"])
        assert np.array_equal(st["bcast_sum"], want), it
        # the peer is IPC-imported: both parts run the 8-GPU world's system-scope hand-off
        assert (st["part_peers"] == L.RLO_PEER_IMPORTED).all() and (st["part_sys_scope"] == 1).all(), it
    k = 256
    runs = sharded.run_processes(16, [0, 8, 16], {"kind": "storm", "k": k, "len": 64, "seed": seed}, max_payload=64,
                                 uncached=True, repeat=6)
    ref = orc.storm(16, seed, k, 64)
    for it, ((st, _, _), rcs) in enumerate(runs):
        bad = [(r, int(st["error"][r]), hex(int(st["error_aux"][r]))) for r in range(16) if st["error"][r]]
        assert rcs == [0, 0], (it, rcs, bad)
        assert np.array_equal(st["bcast_sum"], ref["sum"]), it


def test_bulk_world_churn_processes_pool_cap0(rlo):
    """VERDICT r5 next 5 / ADVICE r5: the pool's free path.  RLO_POOL_CAP_BYTES=0 keeps no free region: every destroyed
    world's exported regions are retired, and after each repeat the parts run the world-wide close (every part drops
    its idle imports, barrier, every part frees its retired regions -- rlo_pool_trim), so each repeat creates, exports
    and imports fresh memory; every repeat must still map and deliver the oracle's bytes"""
    from rlo import sharded

    n, rounds, seed, ln = 4, 4, 33, (1 << 20) + 48
    spec = {"kind": "lat", "rounds": rounds, "len": ln, "seed": seed}
    old = os.environ.get("RLO_POOL_CAP_BYTES")
    os.environ["RLO_POOL_CAP_BYTES"] = "0"  # read by the spawned part processes
    try:
        runs = sharded.run_processes(n, [0, 2, 4], spec, max_payload=64, bulk_max=ln, movers=16, uncached=True, repeat=4)
    finally:
        if old is None:
            os.environ.pop("RLO_POOL_CAP_BYTES", None)
        else:
            os.environ["RLO_POOL_CAP_BYTES"] = old
    org = [orc.origin_of(seed, i, n) for i in range(rounds)]
    want = np.zeros(n, dtype=np.uint64)
    for i, o in enumerate(org):
        cs = np.uint64(orc.msg_checksum(o, i, 0, orc.payload(o, i, ln)))
        for r in range(n):
            if r != o:
                want[r] += cs
    for it, ((st, _, _), rcs) in enumerate(runs):
        assert rcs == [0, 0], (it, st["error"], st["error_aux"])
        assert np.array_equal(st["bcast_sum"], want), it


def _merged(recs, name):
    """one leg's per-rank statistics of every part, by world rank"""
    parts = sorted((r[name] for r in recs), key=lambda x: x["rank_begin"])
    out = {"meta": parts[0]}
    for f in ("bcast_delivered", "bcast_sum", "originated", "own_decided", "own_approved", "actions", "judge_calls",
              "dec_delivered", "error"):
        out[f] = np.array([v for p in parts for v in p[f]], dtype=np.uint64)
    return out


def _check_dump(d, parts):
    recs = [json.load(open(os.path.join(d, "rank%d.json" % r))) for r in range(parts)]
    # the storm: per world rank, deliveries and the checksum of every byte picked up
    s = _merged(recs, "storm")
    m = s["meta"]
    exp = orc.storm_expected(m["world_ranks"], m["seed"], m["k"], m["len"])
    assert (s["error"] == 0).all()
    assert np.array_equal(s["bcast_delivered"].astype(np.int64), exp["count"])
    assert np.array_equal(s["bcast_sum"], exp["sum"])
    assert int(s["originated"].sum()) == m["k"]
    # the latency program: one bcast per round from origin_of(seed, i), the storm's payloads
    lt = _merged(recs, "latency")
    m = lt["meta"]
    exp = orc.storm_expected(len(lt["bcast_sum"]), m["seed"], m["rounds"], m["len"])
    assert np.array_equal(lt["bcast_delivered"].astype(np.int64), exp["count"])
    assert np.array_equal(lt["bcast_sum"], exp["sum"])
    # decisions: one outstanding proposal per rank, approve-all (oracle totals)
    ia = _merged(recs, "iar")
    n = len(ia["own_decided"])
    cfg, keep = orc.judge_cfg(orc.ORC_JUDGE_APPROVE)
    ref = orc.iar_bench(n, ia["meta"]["p"], cfg)
    assert int(ia["own_decided"].sum()) == ref["decisions"] and int(ia["own_approved"].sum()) == ref["approved"]
    assert int(ia["actions"].sum()) == ref["actions"] and int(ia["judge_calls"].sum()) == ref["judge_calls"]
    assert (ia["dec_delivered"] == ia["meta"]["p"] * (n - 1)).all()
    # rootless bulk rounds (one rank per part): every receiver's checksum of every round's bytes
    bulk = [k for k in recs[0] if k.startswith("bulk_")]
    assert bulk, recs[0].keys()
    for name in bulk:
        b = _merged(recs, name)
        m = b["meta"]
        g = len(b["bcast_sum"])
        want, cnt = np.zeros(g, dtype=np.uint64), np.zeros(g, dtype=np.int64)
        for i in range(m["rounds"]):
            o = orc.origin_of(m["seed"], i, g)
            cs = np.uint64(orc.msg_checksum(o, i, 0, orc.payload(o, i, m["len"])))
            for r in range(g):
                if r != o:
                    want[r] += cs
                    cnt[r] += 1
        assert (b["error"] == 0).all(), name
        assert np.array_equal(b["bcast_delivered"].astype(np.int64), cnt), name
        assert np.array_equal(b["bcast_sum"], want), name
    # C5: mixed 64 B .. 1 MiB, every rank originating in every slot
    c5 = _merged(recs, "c5")
    m = c5["meta"]
    exp = orc.storm_expected(m["world_ranks"], m["seed"], m["k"], m["lo"], len_max=m["hi"], order=m["order"])
    assert (c5["error"] == 0).all()
    assert np.array_equal(c5["bcast_delivered"].astype(np.int64), exp["count"])
    assert np.array_equal(c5["bcast_sum"], exp["sum"])


def _bench_parts(parts, per, port, limit, pool_cap=None):
    """bench.py --gpus `parts` under torch.distributed.run, every part on this GPU (RLO_BENCH_DEVICE): one world of
    parts x per ranks, every leg's per-rank statistics (--dump) checked against the oracle.  pool_cap: the parts'
    RLO_POOL_CAP_BYTES (0: every destroyed world's exported regions retire, and bench.py runs the world-wide close
    after every leg, so each leg exports and imports fresh memory)"""
    env = dict(os.environ, RLO_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    if pool_cap is not None:
        env["RLO_POOL_CAP_BYTES"] = str(pool_cap)
    dump = tempfile.mkdtemp(prefix="rlo_dump")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(parts), "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"), "--gpus", str(parts), "--steps", "2",
           "--warmup", "1", "--ranks", str(per), "--k", "16384", "--lat-rounds", "200", "--no-api", "--no-pmc",
           "--no-cpu-baseline", "--dump", dump]
    # Bounded below the suite's per-test limit, output to files (torchrun's workers outlive a killed
    # agent's pipes), so a stall fails with the bench's own progress lines instead of a bare timeout
    try:
        with tempfile.TemporaryFile() as fo, tempfile.TemporaryFile() as fe:
            p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=fo, stderr=fe, start_new_session=True)
            try:
                p.wait(timeout=limit)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGTERM)  # the agent stops its workers
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
                fe.seek(0)
                ps = subprocess.run(["ps", "-eo", "pid,ppid,etime,stat,args"], stdout=subprocess.PIPE).stdout.decode()
                pytest.fail("%d-part bench stalled after %d s; stderr tail:\n" % (parts, limit) + fe.read().decode()[-4000:] +
                            "\nprocesses:\n" + ps[-4000:])
            fo.seek(0)
            fe.seek(0)
            out, err = fo.read(), fe.read()
        lines = [ln for ln in out.decode().splitlines() if ln.startswith("{")]
        stale = "\n".join(ln for ln in err.decode().splitlines() if "as mapped here" in ln)
        assert p.returncode == 0 and lines, stale + err.decode()[-3000:]
        assert b"leg failed" not in err and b"step failed" not in err, stale + "\n" + err.decode()[-3000:]  # on any part
        line = json.loads(lines[-1])
        assert line["n_gpus"] == parts and line["mode"] == "sharded" and line["verified"], line
        assert line["world_ranks"] == parts * per and line["value"] > 0
        assert "round_p50_us" in line and line["decisions_per_s"] > 0
        bulk = line["bulk"]
        assert "error" not in bulk and all(s["verified"] for s in bulk["sizes"]), bulk
        c5 = line["c5_mixed"]
        assert "error" not in c5 and c5["verified"], c5
        _check_dump(dump, parts)  # against the oracle, not only step-to-step repeatability
        return line
    finally:
        shutil.rmtree(dump, ignore_errors=True)


def test_bench_two_parts_under_torchrun():
    _bench_parts(2, 64, 29533, 100)


def test_bench_eight_parts_under_torchrun():
    """VERDICT r4 "next" 4: the 8-part world assembled -- bench.py --gpus 8 as the driver's 8-GPU run starts it
    (8 processes, an 8-way blob exchange and ring mapping, every part's peers imported), here with 32 ranks per
    part so the 8 persistent launches are resident on one GPU together (256 eight-wave rank-workgroups, one per
    CU; parts split on multiples of 8); every leg checked against the oracle per world rank"""
    line = _bench_parts(8, 32, 29541, 140)
    assert line["bulk"]["ranks"] == 8 and line["c5_mixed"]["world_ranks"] == 128


def test_bench_eight_parts_pool_cap0():
    """the 8-part rehearsal with the pool's free path -- no free region kept, so every leg's
    destroyed world retires its exported regions and the world-wide close (rlo_pool_trim: imports dropped, barrier,
    retired regions freed) runs between legs; the next leg's fresh exports must map right in all 8 parts"""
    line = _bench_parts(8, 32, 29547, 140, pool_cap=0)
    assert line["bulk"]["ranks"] == 8


def _stale_part(part, tamper, blob_q, blobs_q, out_q, done_q):
    """one part process of a 16-rank, 2-part world on this GPU; `tamper`: before connecting, change the creation
    nonce the peer's blob carries (PartBlob.nonce, byte 480 of the blob), as a mapping of an earlier allocation
    would show it"""
    try:
        import rlo

        w = rlo.World.part(16, 2, part, part_begin=[0, 8, 16], max_payload=64, uncached=True)
        blob_q.put((part, w.export()))
        blobs = list(blobs_q.get(timeout=120))
        if tamper:
            b = bytearray(blobs[1 - part])
            b[480] ^= 0x5A
            blobs[1 - part] = bytes(b)
        try:
            w.connect(blobs)
            out_q.put((part, "ok"))
        except rlo.RloError as e:
            out_q.put((part, str(e)))
        done_q.get(timeout=120)  # the peer is done with its mapping of this part
        w.close()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        out_q.put((part, "error: %r" % e))


def test_connect_detects_stale_mapping(rlo):
    """rlo_part_connect reads every imported region's creation nonce back through its mapping: a blob whose
    nonce the mapped memory does not show (what an IPC import of an earlier allocation looks like) fails the
    connection with RLO_E_STALE, naming no wrong memory as a ring; the untampered peer connects"""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    blob_q, out_q = ctx.Queue(), ctx.Queue()
    blobs_qs = [ctx.Queue(), ctx.Queue()]
    done_qs = [ctx.Queue(), ctx.Queue()]
    procs = [ctx.Process(target=_stale_part, args=(p, p == 1, blob_q, blobs_qs[p], out_q, done_qs[p])) for p in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(blob_q.get(timeout=180) for _ in range(2))
        for q in blobs_qs:
            q.put([got[0], got[1]])
        res = dict(out_q.get(timeout=180) for _ in range(2))
        for q in done_qs:
            q.put(1)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res[0] == "ok", res
    assert "[-10]" in res[1] and "stale" in res[1], res
