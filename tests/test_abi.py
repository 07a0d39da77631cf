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


def test_region_pool_empty_and_trim_without_gpu():
    """rlo_pool_stats / rlo_pool_trim (the region pool's accounting and its release path) need no device when the
    pool is empty: every count 0, every trim frees nothing"""
    import rlo

    assert rlo.pool_stats() == {"live": 0, "free": 0, "free_exported": 0, "retired": 0, "imports_used": 0,
                                "imports_idle": 0}
    L = rlo.abi
    assert rlo.pool_trim(L.RLO_TRIM_IMPORTS | L.RLO_TRIM_FREE | L.RLO_TRIM_EXPORTED | L.RLO_TRIM_RETIRED) == 0
    assert rlo.abi.load().rlo_pool_stats(None, 6) == L.RLO_E_INVAL


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
    """rlo_bulk_plan (the plan every rank derives for a bulk message, rlo_device.hpp bulk_plan).
    Across GPUs: stripes are whole KiB, a chunk is N-1 stripes, ~sqrt(len / 4 MiB) <= 16 chunks cover
    the message.  One GPU: a DIRECT plan -- one chunk, one stripe holding the whole message (KiB-rounded),
    every tile fanned out from the origin's copy to every receiver.  Tiles <= 16 KiB below 8 MiB, <= 64 KiB
    from there.  The scatter tiles (every stripe of every chunk, cut into tiles) cover every byte exactly
    once, and total_tiles -- each receiver's completion count -- equals the tiles of every stripe."""
    import math

    import rlo

    MiB = 1 << 20
    for n in (2, 3, 5, 8, 16, 64, 255):
        for nbytes in (1, 1000, 1024, 5000, MiB, MiB + 16, 3 * MiB + 123, 16 * MiB, 64 * MiB + 80):
            for cross in (False, True):
                p = rlo.bulk_plan(n, nbytes, cross)
                st, ch, tile = p["stripe"], p["chunk"], p["tile"]
                assert p["direct"] == (0 if cross else 1), (n, nbytes, p)
                if not cross:
                    assert st == ch == -(-nbytes // 1024) * 1024 and p["nchunks"] == 1, (n, nbytes, p)
                else:
                    assert st % 1024 == 0 and st >= 1024 and ch == st * (n - 1), (n, nbytes, p)
                tmax = (64 << 10) if nbytes >= 8 * MiB else (16 << 10)
                assert tile % 1024 == 0 and 1024 <= tile <= min(st, tmax), (n, nbytes, p)
                assert p["nchunks"] == -(-nbytes // ch) <= 16, (n, nbytes, p)
                covered = 0
                per_stripe = [0] * (n - 1)
                for c in range(p["nchunks"]):
                    clen = min(ch, nbytes - c * ch)
                    for k in range(n - 1 if cross else 1):
                        slen = max(0, min(st, clen - k * st))
                        t = -(-slen // tile)
                        per_stripe[k] += t
                        for i in range(t):  # tile i of stripe k of chunk c: contiguous, in order
                            off = c * ch + k * st + i * tile
                            assert off == covered, (n, nbytes, c, k, i)
                            covered += min(tile, slen - i * tile)
                assert covered == nbytes
                assert sum(per_stripe) == p["total_tiles"]
                if cross and nbytes >= 16 * MiB:
                    assert p["nchunks"] >= max(1, math.isqrt(nbytes // (4 * MiB))) - 1
    assert rlo.bulk_plan(8, 64 * MiB, True)["nchunks"] == 4
    assert rlo.bulk_plan(8, 64 * MiB, False)["total_tiles"] == 1024 and rlo.bulk_plan(8, MiB, False)["total_tiles"] == 64
    for bad in ((1, MiB), (8, 0)):
        with pytest.raises(rlo.RloError):
            rlo.bulk_plan(*bad)


def test_bulk_world_config_rejected_without_gpu_or_bad_slots():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import rlo

    with pytest.raises(rlo.RloError):
        rlo.World(8, bulk_max=1 << 20, bulk_slots=3)


EPOCH = 0x9E3779B8  # the segment's pickup-tag epoch (rlo_shm.hpp ShmHdr.pk_epoch)


def _pk_tag(seq, epoch=EPOCH):
    """rlo_device.hpp pk_tag"""
    return (((seq << 1) | 1) & 0xFFFFFFFF) ^ epoch


def _pk_record(seq, kind, origin, frm, ident, length, vote, aux, slot, tagged, epoch=EPOCH):
    """a pickup record as the kernel writes it in host mode (rlo_device.hpp kPkRecBytes): LogRec's eight words with
    the 16-bit tag in the upper half of kind, from + 1, vote and the payload slot"""
    import struct

    t = (_pk_tag(seq, epoch) & 0xFFFF) << 16
    pidx = 0xFFFF if slot is None else (slot | (0x8000 if tagged else 0))
    return struct.pack("<8I", kind | t, origin & 0xFFFFFFFF, ((frm + 1) & 0xFFFF) | t, ident, length, (vote & 0xFFFF) | t,
                       aux, pidx | t)


def _fake_segment(name, nl=2, rb=4, n=8, cc=4, pc=64, stride=80, maxp=64):
    """a shared-host-service segment as rlo_program_host + rlo_host_share lay it out (rlo_shm.hpp),
    built here without a GPU so the client side can be exercised on CPU"""
    import mmap
    import struct

    import rlo

    page = lambda x: (x + 4095) & ~4095  # noqa: E731
    rec = ctypes.sizeof(rlo.abi.LogRec)
    o = 4096
    off = {}
    for key, size in (("hctl", nl * 64 * 8), ("ev", nl * pc * rec), ("evp", nl * pc * maxp), ("cli", nl * 512),
                      ("cmd", nl * cc * stride), ("stage", 0), ("llc", nl * cc * 256)):
        off[key] = o
        o = page(o + size)
    total = o
    fd = os.open("/dev/shm" + name, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
    os.ftruncate(fd, total)
    m = mmap.mmap(fd, total)
    os.close(fd)
    hdr = struct.pack("<10I10Q2I", 0, 5, nl, rb, n, 2, cc, pc, stride, maxp, 0, 0, off["hctl"], off["ev"], off["evp"],
                      off["cli"], off["cmd"], off["stage"], total, off["llc"], 0, EPOCH)
    m[:len(hdr)] = hdr
    m[0:4] = struct.pack("<I", 0x534F4C52)  # magic last
    return m, off, rec


def test_shared_service_client_protocol_without_gpu():
    """rlo_client_*: commands land in the client's shared ring with rlo_host_post's encoding and
    the client's tail; events the kernel would write are read back in order with their payload;
    the ring bounds (command capacity against the device head) hold."""
    import struct

    import rlo

    lib = rlo.abi.load()
    L = rlo.abi
    name = "/rlo.cputest.%d" % os.getpid()
    m, off, rec = _fake_segment(name)
    try:
        c = ctypes.c_void_p()
        assert lib.rlo_client_attach(b"/rlo.no-such-segment", 4, ctypes.byref(c)) == -1
        assert lib.rlo_client_attach(name.encode(), 3, ctypes.byref(c)) == -1  # rank outside the part
        assert lib.rlo_client_attach(name.encode(), 5, ctypes.byref(c)) == 0  # local rank 1
        hctl = off["hctl"] + 1 * 64 * 8
        box = off["cli"] + 1 * 512
        assert lib.rlo_client_state(c) == 0
        m[hctl + 40 * 8:hctl + 41 * 8] = struct.pack("<Q", 1)
        assert lib.rlo_client_state(c) == 1
        cmd = L.Cmd(kind=0, origin=5, id=7, pseq=0, vote=0, pad=0)
        payload = b"hello, rootless"
        for i in range(4):
            assert lib.rlo_client_post(c, ctypes.byref(cmd), payload, len(payload)) == 0
        assert lib.rlo_client_post(c, ctypes.byref(cmd), payload, len(payload)) == -8  # ring full (device head 0)
        assert struct.unpack_from("<Q", m, box)[0] == 4  # mtail
        slot = off["cmd"] + 1 * 4 * 80 + 2 * 80
        w0, w1, w2, _ = struct.unpack_from("<4I", m, slot)
        assert (w0 & 0xFFFF, (w0 >> 16) & 0xFF, w1, w2 & 0xFFFFFF) == (5, 0, 7, len(payload))
        assert bytes(m[slot + 16:slot + 16 + len(payload)]) == payload
        # ... and data-tagged in its command doorbell (rlo_shm.hpp ll_cmd_put): 8-byte halves {word, seq + 1}
        bell = off["llc"] + (1 * 4 + 2) * 256
        g = struct.unpack_from("<16I", m, bell)
        assert g[1::2] == (3,) * 8 and g[0::2][:4] == (w0, w1, w2, 0)
        assert bytes(struct.pack("<4I", *g[0::2][4:8])) == payload + b"\0"
        m[hctl + 16 * 8:hctl + 17 * 8] = struct.pack("<Q", 3)  # the device consumed 3
        consumed, posted = ctypes.c_uint64(), ctypes.c_uint64()
        lib.rlo_client_cmd_count(c, ctypes.byref(consumed), ctypes.byref(posted))
        assert (consumed.value, posted.value) == (3, 4)
        assert lib.rlo_client_post(c, ctypes.byref(cmd), payload, len(payload)) == 0
        # pickup events written "by the kernel" as tagged records (rlo_device.hpp kPkRecBytes): event 0 with a
        # tagged payload is taken as soon as its units are there, no tail; event 1's plain payload (the full path's)
        # only once the published tail covers it; a unit with a stale tag is not taken
        got = L.LogRec()
        buf = ctypes.create_string_buffer(64)
        assert lib.rlo_client_poll(c, ctypes.byref(got), buf, 64) == 0
        at0, at1 = off["ev"] + (1 * 64 + 0) * rec, off["ev"] + (1 * 64 + 1) * rec
        pat0, pat1 = off["evp"] + (1 * 64 + 0) * 64, off["evp"] + (1 * 64 + 1) * 64
        m[at0:at0 + rec] = _pk_record(0, 1, 0, 6, 11, 6, -1, 77, 0, True)
        assert lib.rlo_client_poll(c, ctypes.byref(got), buf, 64) == 0  # its payload units are not there yet
        m[pat0:pat0 + 16] = struct.pack("<2I2I", struct.unpack("<I", b"ev00")[0], _pk_tag(0),
                                        struct.unpack("<I", b"ab\0\0")[0], _pk_tag(0))
        assert lib.rlo_client_poll(c, ctypes.byref(got), buf, 64) == 1
        assert (got.kind, got.origin, got.from_, got.id, got.len, got.vote, got.aux, got.payload_idx) == (1, 0, 6, 11, 6, -1, 77, 0)
        assert buf.raw[:6] == b"ev00ab"
        stale = bytearray(_pk_record(1, 1, 1, -1, 12, 4, -1, 0, 1, False))
        stale[28:32] = struct.pack("<I", (struct.unpack_from("<I", stale, 28)[0] & 0xFFFF) | ((_pk_tag(1 + 64) & 0xFFFF) << 16))
        m[at1:at1 + rec] = bytes(stale)
        m[pat1:pat1 + 4] = b"ev01"
        m[hctl + 32 * 8:hctl + 33 * 8] = struct.pack("<Q", 2)
        assert lib.rlo_client_poll(c, ctypes.byref(got), buf, 64) == 0  # one unit carries another sequence's tag
        m[at1:at1 + rec] = _pk_record(1, 1, 1, -1, 12, 4, -1, 0, 1, False)
        m[hctl + 32 * 8:hctl + 33 * 8] = struct.pack("<Q", 1)
        assert lib.rlo_client_poll(c, ctypes.byref(got), buf, 64) == 0  # plain payload: the tail does not cover it
        m[hctl + 32 * 8:hctl + 33 * 8] = struct.pack("<Q", 2)
        assert lib.rlo_client_poll(c, ctypes.byref(got), buf, 64) == 1
        assert (got.origin, got.from_, buf.raw[:4]) == (1, -1, b"ev01")
        assert lib.rlo_client_poll(c, ctypes.byref(got), buf, 64) == 0
        # mpk: the kernel polls it here, at its pickup-head word (kHctlPkHead = 48)
        assert struct.unpack_from("<Q", m, box + 48 * 8)[0] == 2
        assert lib.rlo_client_detach(c) == 0
    finally:
        m.close()
        os.unlink("/dev/shm" + name)


def test_ctypes_structs_match_the_c_header(tmp_path):
    """every rlo_hip.h struct the Python mirror declares has the C compiler's size and field offsets
    (a field added on one side only would make the library read past the caller's struct)"""
    import subprocess

    from rlo import _lib as L

    pairs = {"rlo_world_cfg_t": L.WorldCfg, "rlo_world_info_t": L.WorldInfo, "rlo_part_cfg_t": L.PartCfg,
             "rlo_storm_cfg_t": L.StormCfg, "rlo_iar_cfg_t": L.IarCfg, "rlo_host_cfg_t": L.HostCfg,
             "rlo_cmd_t": L.Cmd, "rlo_log_rec_t": L.LogRec, "rlo_plan_cfg_t": L.PlanCfg}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rlo_hip.h"', 'int main(void) {']
    for cname, py in pairs.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for fname, _ in py._fields_:
            cf = {"from_": "from"}.get(fname, fname)
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, fname, cname, cf))
    lines += ['return 0;', '}']
    src = tmp_path / "sizes.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-I", INCLUDE, str(src), "-o", str(exe)], check=True)
    got = dict(ln.split() for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines())
    for cname, py in pairs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got["%s.%s" % (cname, fname)]) == getattr(py, fname).offset, (cname, fname)
