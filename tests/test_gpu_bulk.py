"""GPU parity of the bulk (large-message) rootless bcast (byte-exact delivery of
messages beyond the reference's 32,764-B cap to all N-1 ranks), from every kind of originator,
with ragged sizes, in one part (all ranks in one grid), in two parts of one process (two
kernels, peer mappings) and in separate processes (hipIpc)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rlo():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rlo as _rlo

    return _rlo


def _fill(t, nbytes, seed):
    import torch

    g = torch.Generator(device="cuda").manual_seed(seed)
    t[:nbytes].copy_(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g))


def _check(b, n, origin, nbytes, src, rep):
    import torch

    for r in range(n):
        if r == origin:
            continue
        got = b.tensor(r)[:nbytes]
        if not torch.equal(got, src[:nbytes]):
            bad = torch.nonzero(got != src[:nbytes]).flatten()
            stale = int((got[bad] == 0xA5).sum())
            raise AssertionError("rank %d rep %d: %d bytes differ in [%d, %d], %d still 0xA5" %
                                 (r, rep, bad.numel(), int(bad[0]), int(bad[-1]), stale))


@pytest.mark.parametrize("n,nbytes,origin,blocks,chunk,reps", [
    # chunk 0 is the library's choice (one chunk on one GPU); explicit chunks keep the pipelined
    # scatter / all-gather covered; blocks 0 is the library's choice too
    (2, 1 << 20, 1, 8, 256 << 10, 2), (3, 3 * (1 << 20) + 123, 0, 16, 0, 2), (8, 4 << 20, 5, 16, 256 << 10, 2),
    (8, 1000, 7, 4, 0, 2), (5, (1 << 20) + 16, 2, 8, 64 << 10, 2), (16, 2 << 20, 9, 8, 0, 2),
    (3, 3 * (1 << 20) + 123, 0, 16, 192 << 10, 40), (8, (4 << 20) + 80, 3, 32, 0, 40),
    (8, (4 << 20) + 80, 3, 0, 0, 4), (4, (5 << 20) + 7, 1, 0, 512 << 10, 4)])
def test_bulk_one_part(rlo, n, nbytes, origin, blocks, chunk, reps):
    import torch

    from rlo.bulk import Bulk

    with rlo.World(n, max_payload=64) as w, Bulk(w, 8 << 20) as b:
        b.connect([b.export()])
        src = b.tensor(origin)
        _fill(src, nbytes, seed=n * 1000 + origin)
        for rep in range(reps):  # reusable: flags reset between bcasts
            for r in range(n):  # stale bytes must be overwritten, not trusted
                if r != origin:
                    b.tensor(r).fill_(0xA5)
            torch.cuda.synchronize()
            b.reset()
            b.launch(origin, nbytes, blocks=blocks, chunk=chunk)
            b.wait()
            _check(b, n, origin, nbytes, src, rep)


def test_bulk_two_parts_inprocess(rlo):
    import ctypes

    import torch

    from rlo import abi
    from rlo.bulk import Bulk

    n, nbytes = 6, (6 << 20) + 48
    ws = [rlo.World.part(n, 2, p, part_begin=[0, 2, 6], max_payload=64, device=0) for p in range(2)]
    bs = [Bulk(w, 8 << 20) for w in ws]
    lib = abi.load()
    streams = []
    try:
        blobs = [w.export() for w in ws]
        for w in ws:
            w.connect(blobs)
        bblobs = [b.export() for b in bs]
        for b in bs:
            b.connect(bblobs)
        for origin in (0, 4):
            own = bs[0] if origin < 2 else bs[1]
            src = own.tensor(origin)
            _fill(src, nbytes, seed=origin)
            torch.cuda.synchronize()
            for b in bs:
                b.reset()
            if not streams:
                for _ in bs:
                    s = ctypes.c_void_p()
                    abi.check(lib.rlo_stream_create(0, ctypes.byref(s)), "rlo_stream_create")
                    streams.append(s)
            for b, s in zip(bs, streams):
                b.launch(origin, nbytes, blocks=8, stream=s)
            for b in bs:
                b.wait()
            for r in range(n):
                if r != origin:
                    b = bs[0] if r < 2 else bs[1]
                    assert torch.equal(b.tensor(r)[:nbytes], src[:nbytes]), (origin, r)
    finally:
        for b in bs:
            b.close()
        for w in ws:
            w.close()
        for s in streams:
            lib.rlo_stream_destroy(s)
