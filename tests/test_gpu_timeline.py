"""The latency program's per-round timeline (RLO_FLAG_TIMELINE, rlo_timeline): a diagnostics-build feature (make
DIAG=1 -> lib_diag/) that the product library refuses.  Its rows are checked against the oracle where the oracle has
an answer: every non-origin rank's tree parent per round is the skip-ring tree's (orc.tree), every rank but the
origin records an arrival, and the event clocks of a round are ordered (origination before every arrival, the last
pickup after every arrival; bulk: the scatter posted before claimed before moved)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rootless-coll-mpi-ops_amd")

CHILD = r'''
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import rlo
n, ln, rounds, seed = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
kw = dict(max_payload=64, bulk_max=1 << 20) if ln > 112 else dict(max_payload=max(64, ln))
with rlo.World(n, **kw) as w:
    w.program_latency(rounds, ln, seed=seed, timeline=True)
    w.run()
    st = w.stats()
    tl = w.timeline()
    print(json.dumps({"error": st["error"].tolist(), "tl": tl.astype(np.int64).tolist()}))
'''


def _rel(a, b):
    """a - b on the 32-bit 10-ns clock"""
    return ((np.asarray(a, np.int64) - np.asarray(b, np.int64) + (1 << 31)) % (1 << 32)) - (1 << 31)


@pytest.fixture(scope="module")
def rlo():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rlo as _rlo

    return _rlo


def test_product_library_refuses_timeline(rlo):
    if rlo.abi.LIB_PATH.endswith(os.path.join("lib_diag", "librlo_hip.so")):
        pytest.skip("this process runs the diagnostics library")
    with rlo.World(8, max_payload=64) as w:
        with pytest.raises(rlo.RloError, match=r"\[-1\]"):
            w.program_latency(8, 64, timeline=True)


@pytest.mark.parametrize("n,ln", [(8, 64), (32, 112), (8, 16384)])
def test_timeline_rows_match_the_tree(n, ln):
    if not os.path.exists(os.path.join(PKG, "lib_diag", "librlo_hip.so")):
        pytest.skip("diagnostics build (make DIAG=1) not built")
    rounds, seed = 24, 0x71
    env = dict(os.environ, RLO_DIAG_LIB="1")
    r = subprocess.run([sys.executable, "-c", CHILD, PKG, str(n), str(ln), str(rounds), str(seed)], capture_output=True,
                       text=True, timeout=150, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert not any(d["error"]), d["error"]
    tl = np.array(d["tl"], dtype=np.int64)
    assert tl.shape == (rounds, 8 + 9 * n)
    for i in range(rounds):
        o = orc.origin_of(seed, i, n)
        parent, cnt = orc.tree(n, o)
        assert cnt == n - 1
        arr = tl[i, 8:8 + n]
        par = tl[i, 8 + 2 * n:8 + 3 * n] - 1
        assert arr[o] == 0 and par[o] == -1, (i, o)
        others = [r_ for r_ in range(n) if r_ != o]
        assert (arr[others] != 0).all(), (i, arr)
        assert np.array_equal(par[others], parent[others]), (i, par, parent)
        t0 = tl[i, 0]
        assert t0 != 0
        assert (_rel(arr[others], t0) > 0).all(), i
        assert tl[i, 4] != 0 and (_rel(tl[i, 4], arr[others]) >= 0).all(), i  # the last pickup after every arrival
        if ln > 112:  # bulk: the scatter job's events in order, every receiver's copy completed
            assert 0 < _rel(tl[i, 1], t0) <= _rel(tl[i, 2], t0) <= _rel(tl[i, 3], t0), (i, tl[i, :8])
            comp = tl[i, 8 + n:8 + 2 * n]
            assert (comp[others] != 0).all(), (i, comp)


CORRUPT_CHILD = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import rlo
with rlo.World(4, max_payload=64, bulk_max=1 << 20) as w:
    w.program_latency(4, (64 << 10) + 48, seed=0x33)
    w.launch()
    rc = w.wait(raise_on_device_error=False)
    print(json.dumps({"rc": rc, "err": list(w.device_error())}))
'''


def test_bulk_verify_catches_a_stale_granule():
    """VERDICT r4 "next" 1: the bulk leg detects a corrupted tile itself.  The diagnostics build's RLO_BULK_CORRUPT
    makes the first scatter of every message zero one granule of one receiver's copy after the copy (a tile store
    that never became visible behind a complete count); the receiver's VERIFY compares every granule with the
    origin's bytes and must stop the launch with RLO_DERR_BULK, site 14 -- not return rc 0 with a wrong sum"""
    if not os.path.exists(os.path.join(PKG, "lib_diag", "librlo_hip.so")):
        pytest.skip("diagnostics build (make DIAG=1) not built")
    env = dict(os.environ, RLO_DIAG_LIB="1", RLO_BULK_CORRUPT="1")
    r = subprocess.run([sys.executable, "-c", CORRUPT_CHILD, PKG], capture_output=True, text=True, timeout=150, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["rc"] == -4, d  # RLO_E_DEVICE
    code, aux = d["err"]
    assert code == 8 and aux >> 24 == 14, (code, hex(aux))  # RLO_DERR_BULK, the VERIFY site
    assert (aux >> 16) & 0xff < 4 and aux & 0xffff == 0, hex(aux)  # a receiver, the message's first 16-KiB block


STALE_CHILD = r'''
import json, sys, time
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[2])
import rlo
import pyoracle as orc
n, ln = 8, 48
out = {}
with rlo.HostWorld(n, max_payload=64) as hw:
    for i, o in enumerate((0, 5)):
        assert hw.bcast(o, orc.payload(o, i, ln), seq=i)
    got = {r: [] for r in range(n)}
    t0 = time.time()
    while sum(len(v) for v in got.values()) < 2 * (n - 1) and time.time() - t0 < 20:
        for r in range(n):
            got[r] += hw.poll(r)
    out["first"] = sum(len(v) for v in got.values())
    hw.relaunch()
    time.sleep(0.3)
    out["phantom"] = sum(len(hw.poll(r)) for r in range(n))
    assert hw.bcast(3, orc.payload(3, 7, ln), seq=7)
    got = {r: [] for r in range(n)}
    t0 = time.time()
    while sum(len(v) for v in got.values()) < n - 1 and time.time() - t0 < 20:
        for r in range(n):
            got[r] += hw.poll(r)
    time.sleep(0.1)
    for r in range(n):
        got[r] += hw.poll(r)
    out["second"] = {r: [(e["origin"], e["id"], e["payload"][:ln].hex()) for e in got[r]] for r in range(n)}
print(json.dumps(out))
'''


def test_host_relaunch_same_epoch_takes_no_stale_pickup():
    """pickup records are tagged with 16 bits of (sequence, launch epoch), so a record a launch
    16..256 launches back left in a slot could carry the tag the running launch expects.  rlo_reset now clears the
    pickup ring.  The diagnostics build's RLO_PK_EPOCH_SAME keeps the epoch across launches -- every stale record then
    carries exactly the expected tag -- and the relaunched world must still surface nothing before the host posts,
    then exactly the new bcast"""
    if not os.path.exists(os.path.join(PKG, "lib_diag", "librlo_hip.so")):
        pytest.skip("diagnostics build (make DIAG=1) not built")
    env = dict(os.environ, RLO_DIAG_LIB="1", RLO_PK_EPOCH_SAME="1")
    r = subprocess.run([sys.executable, "-c", STALE_CHILD, PKG, os.path.join(REPO, "oracle")], capture_output=True,
                       text=True, timeout=150, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    n, ln = 8, 48
    assert d["first"] == 2 * (n - 1), d
    assert d["phantom"] == 0, d
    for r_ in range(n):
        want = [] if r_ == 3 else [[3, 7, orc.payload(3, 7, ln).hex()]]
        assert d["second"][str(r_)] == want, (r_, d["second"])
