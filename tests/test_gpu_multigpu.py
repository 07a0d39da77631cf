"""Multi-GPU readiness on a one-GPU box: the 8-GPU runs are the driver's, so the
N-part path is exercised here the way it runs there.

  * a part whose peer sits on another GPU (its exported blob names another PCI bus) switches to
    system scope, and a cached part refuses to join such a world (rings and heaps that peers store
    into over xGMI must be uncached);
  * bench.py --gpus 2 under torch.distributed.run (gloo control plane, both ranks on this GPU via
    RLO_BENCH_DEVICE): one 128-rank world in two parts, the storm, latency, decisions, rootless bulk
    and mixed-size legs, each verified.
"""
import json
import os
import re
import signal
import subprocess
import sys
import tempfile

import pytest

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
        assert w0.info["sys_scope"] == 1
        assert w1.info["sys_scope"] == 0
    finally:
        w0.close()
        w1.close()


def test_cached_part_refuses_a_world_spanning_gpus(rlo):
    """rings are uncached by default; the diagnostic RLO_CACHED_RINGS makes cached ones, which may
    not join a world whose parts span GPUs"""
    n = 8
    os.environ["RLO_CACHED_RINGS"] = "1"
    try:
        c0 = rlo.World.part(n, 2, 0, max_payload=64)
        c1 = rlo.World.part(n, 2, 1, max_payload=64)
    finally:
        del os.environ["RLO_CACHED_RINGS"]
    try:
        with pytest.raises(rlo.RloError):
            c0.connect([c0.export(), _forge_bus(c1.export())])
    finally:
        c0.close()
        c1.close()


def test_bench_two_parts_under_torchrun():
    env = dict(os.environ, RLO_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29533", os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--ranks", "64", "--k", "16384", "--lat-rounds", "200", "--no-api", "--no-pmc",
           "--no-cpu-baseline"]
    # Bounded below the suite's per-test limit, output to files (torchrun's workers outlive a killed
    # agent's pipes), so a stall fails with the bench's own progress lines instead of a bare timeout
    with tempfile.TemporaryFile() as fo, tempfile.TemporaryFile() as fe:
        p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=fo, stderr=fe, start_new_session=True)
        try:
            p.wait(timeout=100)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGTERM)  # the agent stops its workers
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
            fe.seek(0)
            ps = subprocess.run(["ps", "-eo", "pid,ppid,etime,stat,args"], stdout=subprocess.PIPE).stdout.decode()
            pytest.fail("two-part bench stalled after 100 s; stderr tail:\n" + fe.read().decode()[-4000:] +
                        "\nprocesses:\n" + ps[-4000:])
        fo.seek(0)
        fe.seek(0)
        out, err = fo.read(), fe.read()
    lines = [ln for ln in out.decode().splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, err.decode()[-3000:]
    line = json.loads(lines[-1])
    assert line["n_gpus"] == 2 and line["mode"] == "sharded" and line["verified"], line
    assert line["world_ranks"] == 128 and line["value"] > 0
    assert "round_p50_us" in line and line["decisions_per_s"] > 0
    bulk = line["bulk"]
    assert "error" not in bulk and all(s["verified"] for s in bulk["sizes"]), bulk
    c5 = line["c5_mixed"]
    assert "error" not in c5 and c5["verified"], c5
