"""CPU tests of the C-ABI boundary: the library loads without a GPU, exports every function
the public headers in include/ declare, and its host-side topology equals the pinned oracle."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(REPO, "include")


def declared_functions(header):
    src = open(os.path.join(INCLUDE, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"#[^\n]*", "", src)
    names = []
    for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_]*)\s*\(([^;{}()]*(\([^()]*\)[^;{}()]*)*)\)\s*;", src):
        name = m.group(1)
        head = src[max(0, m.start() - 80):m.start()]
        if "typedef" in head.split(";")[-1] or name in ("if", "while", "return", "sizeof"):
            continue
        names.append(name)
    return sorted(set(names))


def test_library_loads_without_gpu():
    import rlo

    assert os.path.exists(rlo.LIB_PATH)


LIBS = {"rlo_hip.h": "librlo_hip.so", "rootless_ops.h": "librootless_ops.so"}


def test_every_header_has_a_library():
    assert sorted(h for h in os.listdir(INCLUDE) if h.endswith(".h")) == sorted(LIBS)


@pytest.mark.parametrize("header", sorted(LIBS))
def test_every_declared_symbol_is_exported(header):
    import rlo

    path = os.path.join(os.path.dirname(rlo.LIB_PATH), LIBS[header])
    if header == "rootless_ops.h" and not os.path.exists("/opt/conda/include/mpi.h"):
        pytest.skip("no MPI in this image: librootless_ops.so is not built")
    lib = ctypes.CDLL(path)
    names = declared_functions(header)
    assert names, header
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, (header, missing)


def test_python_export_list_matches_header():
    from rlo import _lib

    assert sorted(_lib.EXPORTS) == declared_functions("rlo_hip.h")


def test_world_create_without_gpu_fails_cleanly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import rlo

    with pytest.raises(rlo.RloError):
        rlo.World(8)


def test_topology_matches_oracle():
    import pyoracle as orc
    import rlo

    for n in list(range(2, 70)) + [127, 128, 129, 255, 256, 257, 1000, 1024, 4096]:
        ranks = range(n) if n <= 70 else range(0, n, max(1, n // 40))
        for r in ranks:
            assert rlo.topology(n, r) == orc.topology(n, r), (n, r)
            for o in range(0, n, max(1, n // 9)):
                for f in [-1] + list(range(0, n, max(1, n // 6))):
                    assert rlo.children(n, r, o, f) == orc.children(n, r, o, f), (n, r, o, f)


def test_children_cover_exact_spanning_tree():
    """Product topology alone (no GPU): BFS over rlo.children yields each rank exactly once."""
    import rlo

    for n in (2, 3, 7, 13, 64, 100, 256, 257):
        for o in range(0, n, max(1, n // 8)):
            seen = {o}
            frontier = [(c, o) for c in rlo.children(n, o, o, -1)]
            while frontier:
                r, frm = frontier.pop()
                assert r not in seen, (n, o, r)
                seen.add(r)
                frontier += [(c, r) for c in rlo.children(n, r, o, frm)]
            assert len(seen) == n


def test_bulk_plan_geometry():
    """rlo_bulk_plan (host arithmetic behind rlo_bulk_launch): stripes are whole 1-KiB blocks, a chunk
    is (n-1) stripes, the chunks cover the message, at most 4096 chunks; library defaults: one chunk
    on one GPU, floor(sqrt(bytes / 4 MiB)) chunks across GPUs, bytes / 64 KiB workgroups in [32, 128]."""
    import math

    from rlo.bulk import plan

    MiB = 1 << 20
    for n in (2, 3, 5, 8, 16, 64):
        for nbytes in (1, 1000, 1024, MiB, MiB + 16, 3 * MiB + 123, 16 * MiB, 64 * MiB, 1 << 30):
            for chunk in (0, 4096, 64 << 10, MiB):
                for cross in (False, True):
                    p = plan(n, nbytes, chunk=chunk, cross_gpu=cross)
                    assert p["stripe"] % 1024 == 0 and p["stripe"] >= 1024, (n, nbytes, p)
                    assert p["chunk"] == p["stripe"] * (n - 1)
                    assert p["nchunks"] == -(-nbytes // p["chunk"]) <= 4096
                    assert p["blocks"] == min(128, max(32, nbytes >> 16))
                    if chunk == 0:
                        want = 1 if not cross else max(1, math.isqrt(nbytes // (4 * MiB)))
                        # the stripe rounds up to whole blocks, so the chunk count can only shrink
                        assert p["nchunks"] <= want, (n, nbytes, cross, p)
                        if nbytes >= 64 * (n - 1) * 1024 and want <= 4096:
                            assert p["nchunks"] == want or p["nchunks"] == want - 1, (n, nbytes, cross, p)
    assert plan(8, 64 * MiB, cross_gpu=True)["nchunks"] == 4
    assert plan(8, 16 * MiB, cross_gpu=True)["nchunks"] == 2
    assert plan(8, 4 * MiB, cross_gpu=True)["nchunks"] == 1
    assert plan(8, 64 * MiB, cross_gpu=False)["nchunks"] == 1
    assert plan(8, MiB, blocks=7)["blocks"] == 7
    import rlo

    for bad in ((1, MiB), (65, MiB), (8, 0)):
        with pytest.raises(rlo.RloError):
            plan(*bad)
