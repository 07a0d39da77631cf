"""bench.py's multi-part control plane on CPU (world_size 2, gloo, no GPU): the driver's N-GPU run is
one process per GPU, each holding one part of one world; the parts exchange mapping blobs and run
barriers over torch.distributed.  A part that fails to create / connect its part, or whose step fails,
must not leave its peer waiting in a collective the failing part never joins (the round-2 rehearsal
hang).  Fake worlds stand in for librlo_hip.so's parts."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeWorld:
    def __init__(self, part, fail_export=False, fail_connect=False, fail_launch=False):
        self.part, self.fail_connect, self.fail_launch = part, fail_connect, fail_launch
        self.info = {"part": part, "n_parts": 2}
        self.closed = False
        if fail_export:
            raise RuntimeError("create failed on part %d" % part)

    def export(self):
        return b"blob%d" % self.part

    def connect(self, blobs):
        assert blobs == [b"blob0", b"blob1"]
        if self.fail_connect:
            raise RuntimeError("connect failed on part %d" % self.part)

    def import_part(self, blob, k):
        assert blob == b"blob%d" % k

    def staged_connect(self, blobs, barrier, bcast=None):
        from rlo.world import World  # the real staging logic over this fake's export / import_part / connect

        World.staged_connect(self, blobs, barrier, bcast)

    def close_imports(self):
        pass

    def reset(self, stream=None):
        pass

    def launch(self, stream=None, no_reset=False):
        if self.fail_launch:
            raise RuntimeError("launch failed on part %d" % self.part)

    def wait(self, raise_on_device_error=True):
        return 0

    def kernel_ms(self):
        return 1.0

    def close(self):
        self.closed = True


class FakeRlo:
    def __init__(self, fail):
        self.fail = fail

    @property
    def World(self):
        fail = self.fail

        class W:
            @staticmethod
            def part(R, world, rank, **kw):
                return FakeWorld(rank, **{k: True for k, v in fail.items() if v == rank})
        return W


def _worker(rank, port, fail, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=2)
    out = {}
    try:
        try:
            w = bench._world(FakeRlo(fail), dist, 16, 2, rank, 0)
            out["world"] = "ok"
        except RuntimeError as e:
            out["world"] = "raised: %s" % e
            w = FakeWorld(rank, fail_launch=fail.get("fail_launch") == rank)
        rc, ms = bench._step(w, None, dist)  # both parts reach both barriers
        out["step"] = rc
        dist.barrier()  # still in step afterwards
        out["after"] = "ok"
    finally:
        dist.destroy_process_group()
    q.put((rank, out))


def _run(fail):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, fail, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    return res


@pytest.mark.parametrize("fail", [{}, {"fail_export": 1}, {"fail_connect": 0}, {"fail_launch": 1}],
                         ids=["clean", "create", "connect", "launch"])
def test_parts_fail_together_and_stay_in_step(fail):
    res = _run(fail)
    for r in (0, 1):
        assert res[r]["after"] == "ok"
    if "fail_export" in fail or "fail_connect" in fail:
        assert all(res[r]["world"].startswith("raised") for r in (0, 1)), res  # both parts raise
    else:
        assert all(res[r]["world"] == "ok" for r in (0, 1)), res
    if "fail_launch" in fail:
        bad = fail["fail_launch"]
        assert res[bad]["step"] == -99 and res[1 - bad]["step"] == 0, res
