#!/usr/bin/env python3
"""bench.py -- rootless bcast storm on MI355X (BASELINE.json configs[1], [4]).

One step = one launch of the persistent progress kernel that carries a storm of
K rootless bcasts (random originators, 64-byte payloads by default) across the
world's ranks until every rank has picked up every bcast it is owed.  Inputs
(schedule, rings) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W]

N = 1: one GPU hosts a 256-rank world (256 workgroup-ranks).
N > 1 (torch.distributed.run, one process per GPU): ONE world of 256 x N ranks,
sharded contiguously (256 ranks per GPU); every bcast's tree crosses the GPUs over
xGMI through peer-HBM ring stores (no collective on the data path; gloo only
exchanges the ring-mapping blobs and runs the barriers).  K bcasts per step at every
N, so each GPU delivers ~K x 256 messages per step: weak scaling.  `value` is
rootless bcast messages per second (BASELINE.json's metric: originated bcasts that
reached every other rank); `deliveries_per_s` (K x (R - 1) per step) is reported
beside it.  One JSON line is printed by rank 0.
"""
import argparse
import json
import os
import subprocess
import resource
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "rootless-coll-mpi-ops_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def note(msg):
    """progress on stderr (the JSON line stays the only stdout)"""
    print("[bench %.1fs] %s" % (time.time() - _T0, msg), file=sys.stderr, flush=True)


_T0 = time.time()


def percentile(a, p):
    import numpy as np

    return float(np.percentile(np.asarray(a, dtype=np.float64), p)) if len(a) else 0.0


_DUMP = {"dir": "", "recs": {}}
# storm legs (the headline and the payload-size legs) whose per-rank results the cpu_baseline leg checks against the
# oracle: each a record dict carrying "verified" and a "_check" {n, seed, k, len, count, sum}
_STORM_CHECKS = []
_DUMP_FIELDS = ("bcast_delivered", "bcast_sum", "originated", "own_decided", "own_approved", "actions", "judge_calls",
                "dec_delivered", "error")


def dump_leg(name, w, st, **extra):
    """--dump: this part's per-rank statistics of one leg (the world ranks it holds), for the test that
    compares the multi-part runs with the oracle (the bench itself never imports the oracle)"""
    if not _DUMP["dir"]:
        return
    rec = {"rank_begin": int(w.rank_begin), "n_local": int(w.n_local)}
    rec.update({f: [int(x) for x in st[f]] for f in _DUMP_FIELDS})
    rec.update(extra)
    _DUMP["recs"][name] = rec


def dump_write(rank):
    if not _DUMP["dir"]:
        return
    os.makedirs(_DUMP["dir"], exist_ok=True)
    with open(os.path.join(_DUMP["dir"], "rank%d.json" % rank), "w") as f:
        json.dump(_DUMP["recs"], f)


def cpu_baseline(n, length, seed, target_s, bulk=None):
    """The oracle's clean-room CPU restatement ("port") on the box's host cores: the same storm (n
    virtual ranks, length-byte payloads, random originators) with every tree edge copying the bytes,
    the ranks dealt to `threads` host threads (oracle/rlo_oracle.c orc_storm_mt), bounded sample.
    Beside it: the compiled reference itself under host MPI at its own 4- and 8-rank worlds.
    The oracle is also the checker of the bulk leg (`bulk`): every receiver's checksum of every round's bytes
    against orc.msg_checksum of the oracle's payload (not launch-to-launch equality alone)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle as orc
    import numpy as np

    # every storm leg's per-rank delivery counts and checksums against the oracle's analytic expectation of the same
    # (n, seed, k, length) storm (the headline's `verified` was step-to-step equality only)
    for rec in _STORM_CHECKS:
        chk = rec.pop("_check")
        want = orc.storm_expected(chk["n"], chk["seed"], chk["k"], chk["len"])
        rec["verified_oracle"] = bool(np.array_equal(np.asarray(chk["count"], dtype=np.int64), want["count"]) and
                                      np.array_equal(np.asarray(chk["sum"], dtype=np.uint64), want["sum"]))
        rec["verified"] = bool(rec["verified"] and rec["verified_oracle"])
    _STORM_CHECKS.clear()

    if bulk:
        for rec in bulk.get("sizes", []):
            chk = rec.pop("_check", None)
            if chk is None:
                continue
            got = chk["sum"]
            g = len(got)
            want = [0] * g
            for i in range(chk["rounds"]):
                o = orc.origin_of(chk["seed"], i, g)
                cs = orc.msg_checksum(o, i, 0, orc.payload(o, i, chk["len"]))
                for r in range(g):
                    if r != o:
                        want[r] = (want[r] + cs) & 0xFFFFFFFFFFFFFFFF
            rec["verified_oracle"] = [int(x) for x in got] == want
            rec["verified"] = bool(rec["verified"] and rec["verified_oracle"])

    threads = max(1, min(16, os.cpu_count() or 1))  # the box's CPU share for one GPU is 16
    t = time.perf_counter()
    orc.storm_mt(n, seed, 20000, length, threads)
    per = (time.perf_counter() - t) / 20000
    k = int(max(20000, min(4_000_000, target_s / max(per, 1e-9))))
    t = time.perf_counter()
    res = orc.storm_mt(n, seed, k, length, threads)
    dt = time.perf_counter() - t
    out = {"value": k / dt, "unit": "msgs/s", "deliveries_per_s": res["deliveries"] / dt, "cores": threads,
           "kind": "port",
           "sample": "oracle/rlo_oracle.c orc_storm_mt: %d virtual ranks, %d B, %d random-origin bcasts (%d deliveries, "
                     "bytes copied on every tree edge), %.1f s on %d host threads" % (n, length, k, res["deliveries"], dt,
                                                                                     threads)}
    refs = {}
    for nr in (4, 8):
        ref = reference_datapoint(length, nr)
        if ref:
            refs["n%d" % nr] = ref
    if refs:
        out["reference_host_mpi"] = refs
    return out


def pmc_traffic(ranks, length, k, device, timeout_s=120):
    """HBM bytes per launch of the storm kernel from rocprofv3 PMC counters, collected live in
    two separate passes (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2: they cannot share a pass).
    gfx950 corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reports half the bytes of wide
    (16 B/lane) streaming reads -> x2; WRITE_SIZE is exact for 16-B stores.  Both are in KiB."""
    import shutil

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import rocpd_summary

    vals = {}
    with tempfile.TemporaryDirectory() as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(td, ctr)
            cmd = ["timeout", "-s", "KILL", str(timeout_s), prof, "--pmc", ctr, "-d", d, "-o", "run", "--",
                   sys.executable, os.path.join(REPO, "tools", "pmc_probe.py"), "--ranks", str(ranks), "--len",
                   str(length), "--k", str(k), "--launches", "2", "--device", str(device)]
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            if r.returncode != 0:
                return None, "rocprofv3 %s pass rc=%d" % (ctr, r.returncode)
            dbs = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith(".db")]
            rows = rocpd_summary.pmc(dbs[0]) if dbs else []
            if not rows:
                return None, "no %s rows" % ctr
            vals[ctr] = rows[-1][3] * 1024.0  # last launch, KiB -> bytes
    fetch = 2.0 * vals["FETCH_SIZE"]
    write = vals["WRITE_SIZE"]
    return {"bytes": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, last of 2 launches; FETCH x2 (gfx950)"}, None


def kfd_census():
    """processes holding KFD (GPU) queues right now: /sys/class/kfd/kfd/proc/<pid>/queues/<q>/gpuid (what the
    GPUs' hardware schedulers map).  {pid: (comm, {gpuid: queues})}, every GPU of the node;
    unreadable entries are skipped"""
    root = "/sys/class/kfd/kfd/proc"
    out = {}
    try:
        pids = os.listdir(root)
    except OSError:
        return None
    for pid in pids:
        qs = {}
        try:
            for q in os.listdir(os.path.join(root, pid, "queues")):
                try:
                    g = open(os.path.join(root, pid, "queues", q, "gpuid")).read().strip()
                except OSError:
                    g = "?"
                qs[g] = qs.get(g, 0) + 1
        except OSError:
            continue
        try:
            comm = open("/proc/%s/comm" % pid).read().strip()
        except OSError:
            comm = "?"
        out[int(pid)] = (comm, qs)
    return out


def cpu_throttle():
    """(nr_throttled, throttled_usec) of this cgroup (v2 cpu.stat): the box's CPU quota throttles spinning threads"""
    try:
        kv = dict(ln.split() for ln in open("/sys/fs/cgroup/cpu.stat"))
        return int(kv.get("nr_throttled", 0)), int(kv.get("throttled_usec", 0))
    except (OSError, ValueError):
        return None


def _run_sampled(cmd, timeout_s, env=None, period=0.05):
    """run cmd; meanwhile sample the KFD census: on the GPU(s) the leg's own processes (rlo_api_bench) hold
    queues on, the most processes holding queues at once and the other processes among them; and the CPU
    quota throttling of this cgroup over the run"""
    import threading

    stop = threading.Event()
    seen = {"max_procs_our_gpu": 0, "others_our_gpu": set(), "our_gpuids": set(), "samples": 0}

    def sample():
        while not stop.is_set():
            c = kfd_census()
            if c is not None:
                seen["samples"] += 1
                ours = set(g for comm, qs in c.values() if comm == "rlo_api_bench" for g in qs)
                seen["our_gpuids"] |= ours
                on = {p: v for p, v in c.items() if any(g in seen["our_gpuids"] for g in v[1])}
                seen["max_procs_our_gpu"] = max(seen["max_procs_our_gpu"], len(on))
                seen["others_our_gpu"].update("%s:%d" % (v[0], p) for p, v in on.items() if v[0] != "rlo_api_bench")
            stop.wait(period)

    th = threading.Thread(target=sample, daemon=True)
    t0 = cpu_throttle()
    ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    w0 = time.perf_counter()
    th.start()
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=timeout_s + 20, env=env)
    finally:
        stop.set()
        th.join(timeout=2)
    wall = time.perf_counter() - w0
    ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    # core accounting: CPU seconds of every process of the run (mpiexec, its proxies, the rank processes and all
    # their threads: waited-for descendants accumulate into RUSAGE_CHILDREN), and that over the run's wall time =
    # the cores the run kept busy on average (init and teardown included)
    cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    seen["cpu_s"] = round(cpu, 2)
    seen["wall_s"] = round(wall, 2)
    seen["cores_busy"] = round(cpu / wall, 2) if wall > 0 else None
    t1 = cpu_throttle()
    if t0 and t1:
        seen["cpu_throttled_periods"] = t1[0] - t0[0]
        seen["cpu_throttled_ms"] = round((t1[1] - t0[1]) * 1e-3, 1)
    seen["others_our_gpu"] = sorted(seen["others_our_gpu"])[:8]
    seen["our_gpuids"] = sorted(seen["our_gpuids"])
    return r, seen


def dropin_api_leg(ranks=(4, 8), timeout_s=150, reps=3):
    """The drop-in rootless_ops.h path end to end: tools/api_bench.c over librootless_ops.so
    (one MPI process per rank, every rank's engine a persistent kernel on this GPU) beside the
    same driver linked against the compiled reference under host MPI on the box's cores, at the
    reference's own 4- and 8-rank worlds.  Runs with the box's environment as it is (recorded).  Every
    leg runs `reps` times, interleaved with the reference's, and reports the median with every run, and
    for ours the KFD queue census sampled during each run (processes holding GPU queues: ours should be
    one leader per GPU; another process's queues time-slice the card)."""
    mpiexec = "/opt/conda/bin/mpiexec"
    ours = os.path.join(PKG, "lib", "rlo_api_bench")
    ref = os.path.join(REPO, "oracle", "_ref", "ref_api_bench")
    if not (os.path.exists(mpiexec) and os.path.exists(ours)):
        return {"error": "mpiexec or rlo_api_bench missing"}
    out = {"driver": "tools/api_bench.c (same calls for both)",
           "env": {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)")}}
    legs = [("storm", ["storm", "20000", "64"]), ("lat", ["lat", "500", "64"]), ("iar", ["iar", "2000"])]
    # iardj: the same consensus loop with the approve-all judge registered on the device
    # (RLO_progress_engine_new_dj, an extension; the reference judges with its callback only)
    legs_ours = legs + [("iardj", ["iardj", "2000"]), ("iarpool", ["iarpool", "8000"])]
    avail = len(os.sched_getaffinity(0))
    for nr in ranks:
        # the reference: one rank per core, pinned (BASELINE.md CPU-baseline plan); ours unpinned, since a
        # GPU leader process runs the application thread beside its pump and proxy threads
        rec = {"ranks": nr, "ours": {}, "reference_host_mpi": {}, "cores": nr, "cores_available": avail,
               "pinning": {"reference_host_mpi": "mpiexec -bind-to core: one core per rank (%d cores)" % nr,
                           "ours": "RLO_NUMA_BIND=all: every thread of a rank process on the GPU's NUMA node (%d cores available)" % avail}}
        runs = {"ours": {}, "reference_host_mpi": {}}
        for rep in range(reps):
            for name, exe in (("ours", ours), ("reference_host_mpi", ref)):
                if not os.path.exists(exe):
                    rec[name] = {"error": "not built"}
                    continue
                for leg, args in (legs_ours if name == "ours" else legs):
                    note("api n=%d %s %s (%d/%d)" % (nr, name, leg, rep + 1, reps))
                    try:
                        # iarpool: the proposal pool extension, 16 own proposals in flight per rank
                        env = None
                        if name == "ours":
                            # the application opts in to having its own thread placed on the GPU's NUMA node
                            # (the reference is placed by mpiexec -bind-to core)
                            env = dict(os.environ, RLO_NUMA_BIND="all")
                            if leg == "iarpool":
                                env["RLO_PROPOSAL_POOL"] = "16"
                        bind = ["-bind-to", "core"] if name == "reference_host_mpi" else []
                        cmd = ["timeout", "-k", "5", str(timeout_s), mpiexec] + bind + ["-n", str(nr), exe] + args
                        r, seen = _run_sampled(cmd, timeout_s, env=env)
                        lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
                        res = json.loads(lines[-1]) if lines else {"error": "rc=%d" % r.returncode}
                        if name == "ours":
                            res["kfd"] = seen
                        else:
                            res["cpu_throttled_ms"] = seen.get("cpu_throttled_ms")
                        res["cpu"] = {k: seen.get(k) for k in ("cpu_s", "wall_s", "cores_busy")}
                    except Exception as e:  # noqa: BLE001 - informative leg, never fails the bench
                        res = {"error": str(e)[:200]}
                    runs[name].setdefault(leg, []).append(res)
        for name in ("ours", "reference_host_mpi"):
            if isinstance(rec[name], dict) and "error" in rec[name]:
                continue
            for leg, rs in runs[name].items():
                good = [x for x in rs if "error" not in x]
                if not good:
                    rec[name][leg] = rs[-1]
                    continue
                key = "p50_us" if leg == "lat" else ("bcast_per_s" if leg == "storm" else "decisions_per_s")
                vals = sorted(x.get(key, 0.0) for x in good)
                med = dict(sorted(good, key=lambda x: x.get(key, 0.0))[len(good) // 2])
                med["runs_" + key] = vals
                if "seconds" in good[0]:
                    med["runs_seconds"] = [x.get("seconds") for x in good]
                med["runs_cores_busy"] = [x.get("cpu", {}).get("cores_busy") for x in good]
                if name == "ours":
                    # the census of the GPU our rank processes used: processes holding queues on it at once
                    # (ours: one leader per GPU), the other processes among them, the CPU quota's throttling
                    med["kfd_max_procs_our_gpu"] = max(x["kfd"]["max_procs_our_gpu"] for x in good)
                    med["kfd_others_our_gpu"] = sorted(set(p for x in good for p in x["kfd"]["others_our_gpu"]))
                    med["runs_cpu_throttled_ms"] = [x["kfd"].get("cpu_throttled_ms") for x in good]
                    med.pop("kfd", None)
                else:
                    med["runs_cpu_throttled_ms"] = [x.get("cpu_throttled_ms") for x in good]
                rec[name][leg] = med
        # the CPU each side spent: average cores kept busy over a run (CPU seconds of all the
        # run's processes and threads / wall), median over the runs, per leg -- ours spins an application thread and a
        # pump per rank plus the leader's proxy; the reference one pinned core per rank
        rec["cores_busy"] = {}
        for name in ("ours", "reference_host_mpi"):
            for leg, rs in runs[name].items():
                cb = sorted(x["cpu"]["cores_busy"] for x in rs if x.get("cpu", {}).get("cores_busy") is not None)
                if cb:
                    rec["cores_busy"].setdefault(leg, {})[name] = cb[len(cb) // 2]
        try:
            o, f = rec["ours"], rec["reference_host_mpi"]
            rec["ratio_vs_reference"] = {
                "bcast_per_s": round(o["storm"]["bcast_per_s"] / f["storm"]["bcast_per_s"], 2),
                "decisions_per_s": round(o["iar"]["decisions_per_s"] / f["iar"]["decisions_per_s"], 2),
                "decisions_per_s_device_judge": round(o["iardj"]["decisions_per_s"] / f["iar"]["decisions_per_s"], 2),
                "decisions_per_s_pool16": round(o["iarpool"]["decisions_per_s"] / f["iar"]["decisions_per_s"], 2),
                "p50_latency": round(o["lat"]["p50_us"] / f["lat"]["p50_us"], 2)}
        except Exception:  # noqa: BLE001
            pass
        out["n%d" % nr] = rec
    return out


def size_legs(rlo, R, device, stream, sizes=(256, 1024, 4096), k=1 << 16, steps=3):
    """The headline storm at SURVEY 8(d) C2's larger payloads (one GPU): bcast/s and the HBM
    roofline fraction per size, 2(N-1)(S+16) algorithmic bytes per bcast as for `value`.  Every
    step must deliver the same bytes (per-rank checksums equal across steps)."""
    import numpy as np

    out = []
    for s in sizes:
        # the slot is the workload's payload size, as an application sizes its engine (slots of <= 24
        # chunks take the small copy path, larger ones the large-message path)
        with rlo.World(R, max_payload=s, device=device) as w:
            w.program_storm(k, s, seed=0x5EED)
            sums, kms, ok = [], [], True
            t0 = 0.0
            for i in range(steps + 1):  # first launch warms
                if i == 1:
                    t0 = time.perf_counter()
                w.reset(stream)
                w.launch(stream, no_reset=True)
                ok &= w.wait(raise_on_device_error=False) == 0
                st = w.stats()
                ok &= bool((st["error"] == 0).all()) and int(st["originated"].sum()) == k
                sums.append(st["bcast_sum"].copy())
                if i:
                    kms.append(w.kernel_ms())
            dt = (time.perf_counter() - t0) / steps
            ok &= all(np.array_equal(sums[0], x) for x in sums[1:])
            kernel_ms = float(np.mean(kms))
            gbs = k * 2.0 * (R - 1) * (s + 16) / (kernel_ms * 1e-3) / 1e9
            rec = {"payload_bytes": s, "bcasts": k, "bcast_per_s": round(k / dt, 1),
                   "deliveries_per_s": round(k * (R - 1) / dt, 1), "kernel_ms": round(kernel_ms, 3),
                   "alg_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                   "payloads": "pulled" if w.info["pull"] else "pushed", "verified": ok,
                   "_check": {"n": R, "seed": 0x5EED, "k": k, "len": s, "count": st["bcast_delivered"].tolist(),
                              "sum": st["bcast_sum"].tolist()}}
            _STORM_CHECKS.append(rec)
            out.append(rec)
    return out


def _step(w, stream, dist):
    """one launch of the loaded program; every part reset before any part launches.  Never raises
    between its two barriers: a part whose reset / launch / wait fails still joins both (its peers'
    kernels then stop at their no-progress timeout), so the parts stay in step -- an exception here
    once left one part in the next leg's collectives while its peer waited in this one's"""
    err = None
    try:
        w.reset(stream)
    except Exception as e:  # noqa: BLE001 - reported, the parts stay in step
        err = e
    if dist is not None:
        dist.barrier()
    rc = -99
    if err is None:
        try:
            w.launch(stream, no_reset=True)
            rc = w.wait(raise_on_device_error=False)
        except Exception as e:  # noqa: BLE001
            err = e
    if dist is not None:
        dist.barrier()  # no peer still stores into this part's rings / heaps
    if err is not None:
        note("part %d: step failed: %r" % (w.info.get("part", -1), err))
        return rc, 0.0
    return rc, w.kernel_ms()


def _agree(dist, world, err):
    """every part learns every part's error (None = fine); raises on all of them if any failed"""
    if world == 1:
        if err:
            raise RuntimeError(err)
        return
    errs = [None] * world
    dist.all_gather_object(errs, err)
    bad = [e for e in errs if e]
    if bad:
        raise RuntimeError("; ".join(bad))


def _bcast_blob(dist):
    """part k's blob to every part (World.staged_connect)"""
    def f(blob, k):
        obj = [blob]
        dist.broadcast_object_list(obj, src=k)
        return obj[0]
    return f


def _close(w, dist):
    """tear a world down.  Sharded: every part first drops its hipIpc imports of its peers' regions, then -- after a
    barrier -- frees its own.  A part that freed (and re-allocated, and exported) memory a peer still imported was
    seen to hand that peer a mapping of its OLD memory for the new handle (tools/probe/part_churn.py)"""
    if dist is not None and w.info.get("n_parts", 1) > 1:
        try:
            w.close_imports()
        finally:
            dist.barrier()
    w.close()
    if dist is not None:
        import rlo
        import torch

        # the world-wide close (rlo_hip.h rlo_pool_trim): regions a peer imported leave the pool only once every part
        # dropped its idle imports -- needed only when some part has retired regions (beyond RLO_POOL_CAP_BYTES)
        t = torch.tensor([float(rlo.pool_stats()["retired"])], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if t.item() > 0:
            rlo.pool_trim(rlo.abi.RLO_TRIM_IMPORTS | rlo.abi.RLO_TRIM_FREE)
            dist.barrier()
            rlo.pool_trim(rlo.abi.RLO_TRIM_RETIRED)
            dist.barrier()


def _world(rlo, dist, R, world, rank, local, **kw):
    """one R-rank world: whole on this GPU (world == 1) or this process's part of it.  In the
    one-GPU rehearsal (RLO_BENCH_DEVICE) every part shares the GPU: bulk worlds then take few mover
    workgroups, or the parts' persistent launches could not all be resident at once"""
    if world == 1:
        return rlo.World(R, device=local, **kw)
    if os.environ.get("RLO_BENCH_DEVICE") and kw.get("bulk_max") and not kw.get("movers"):
        kw["movers"] = 16
    # every part learns whether every other part was made and connected: a part that failed alone would
    # otherwise leave its peers waiting in this exchange while it moves on to the next leg's (the ranks desync)
    w, err = None, None
    try:
        w = rlo.World.part(R, world, rank, device=local, uncached=True, **kw)
        mine = w.export()
    except Exception as e:  # noqa: BLE001 - re-raised below, on every rank
        err, mine = "rank %d: create/export: %r" % (rank, e), None
    blobs = [None] * world
    dist.all_gather_object(blobs, (mine, err))
    errs = [e for _, e in blobs if e]
    if errs:
        if w is not None:
            w.close()
        raise RuntimeError("world part creation failed: " + "; ".join(errs))
    try:
        w.staged_connect([b for b, _ in blobs], dist.barrier, _bcast_blob(dist))  # one exporter at a time
    except Exception as e:  # noqa: BLE001
        err = "rank %d: connect: %r" % (rank, e)
    try:
        _agree(dist, world, err)
    except Exception:
        w.close()
        raise
    return w


def bulk_leg(rlo, dist, world, rank, local, stream, red, sizes_mib=(1, 4, 16, 64), rounds=8):
    """BASELINE configs[2] / SURVEY 8(d) C3: large-message ROOTLESS bcast through the engine -- the
    origin alone decides to send, receivers learn of it from the announcement on the skip-ring tree,
    the mover workgroups move the bytes (one GPU: a fan-out from the origin's copy into every receiver's heap;
    across GPUs: pipelined scatter + all-gather between the ranks' heaps).
    The latency program: one bcast at a time from random originators, round i+1 starts when every
    rank holds round i; algbw = S / round time (world rank 0's clock).  N > 1: one rank per GPU,
    beside rooted RCCL broadcast of the same bytes from the same root.  N = 1: 8 ranks on the GPU."""
    import numpy as np
    import torch

    G = world if world > 1 else 8
    maxb = max(sizes_mib) << 20
    w = _world(rlo, dist, G, world, rank, local, max_payload=64, bulk_max=maxb)
    # rehearsal of the N-part path on one GPU (RLO_BENCH_DEVICE): RCCL refuses two ranks per GPU
    nccl = dist.new_group(backend="nccl") if world > 1 and not os.environ.get("RLO_BENCH_DEVICE") else None
    out = []
    try:
        for mib in sizes_mib:
            nbytes = mib << 20
            w.program_latency(rounds, nbytes, seed=0xB0 + mib)
            sums, ok, kms = [], True, []
            for _ in range(2):  # the first launch warms; both must deliver the same bytes
                rc, ms = _step(w, stream, dist)
                st = w.stats()
                ok &= rc == 0 and bool((st["error"] == 0).all())
                ok &= int(red(float(st["bcast_delivered"].sum()), "sum")) == rounds * (G - 1)
                sums.append(st["bcast_sum"].copy())
                kms.append(ms)
            ok &= bool(np.array_equal(sums[0], sums[1]))
            dump_leg("bulk_%dMiB" % mib, w, st, seed=0xB0 + mib, rounds=rounds, len=nbytes)
            rt = 0.0
            if w.rank_begin == 0:  # world rank 0's clock saw every round complete
                obs = w.round_ticks().astype(np.float64)
                d = np.diff(obs[obs > 0]) * 1e-8  # 10 ns ticks -> s
                rt = float(np.median(d)) if len(d) else 0.0
            rt = red(rt, "max")
            ok = red(0.0 if ok else 1.0, "max") == 0.0
            rec = {"MiB": mib, "round_ms": round(rt * 1e3, 4), "kernel_ms_per_round": round(red(kms[1], "max") / rounds, 4),
                   "verified": bool(ok)}
            if world == 1:  # per-receiver checksums, checked against the oracle in the cpu_baseline leg
                rec["_check"] = {"seed": 0xB0 + mib, "rounds": rounds, "len": nbytes, "sum": sums[1].tolist()}
            rec["algbw_GBps"] = round(nbytes / rt / 1e9, 2) if rt > 0 else None
            if world == 1 and rt > 0:
                # one GPU (direct plan): the origin's copy written at origination and read once by the
                # fan-out (2S), every receiver's copy written once ((G-1)S) and read back to verify ((G-1)S):
                # 2G S HBM bytes
                rec["hbm_GBps"] = round(2 * G * nbytes / rt / 1e9, 1)
                rec["hbm_frac"] = round(rec["hbm_GBps"] / HBM_PEAK_GBS, 4)
                # the data movement alone, without the receivers' VERIFY read-back (the benchmark's own check):
                # the origin's copy written and read once, G-1 receiver copies written -- (G+1) S
                rec["hbm_frac_no_verify"] = round((G + 1) * nbytes / rt / 1e9 / HBM_PEAK_GBS, 4)
            if rank == 0:
                note("bulk %d MiB: %.3f ms/round" % (mib, rt * 1e3))
            if nccl is not None:
                t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                rcl = []
                for it in range(rounds + 2):
                    torch.cuda.synchronize()
                    dist.barrier()
                    e0.record()
                    dist.broadcast(t, src=it % G, group=nccl)
                    e1.record()
                    torch.cuda.synchronize()
                    if it >= 2:
                        rcl.append(red(e0.elapsed_time(e1), "max"))
                rec["rccl_ms"] = round(float(np.median(rcl)), 4)
                rec["rccl_algbw_GBps"] = round(nbytes / (rec["rccl_ms"] * 1e-3) / 1e9, 2)
                if rt > 0:
                    rec["ours_over_rccl"] = round(rec["rccl_ms"] / (rt * 1e3), 3)
            out.append(rec)
    finally:
        _close(w, dist)
    return {"ranks": G, "ranks_per_gpu": 1 if world > 1 else G, "movers_per_part": w.info.get("movers"),
            "algorithm": "rootless: announcement on the skip-ring tree, mover workgroups move the bytes between "
                         "per-rank heaps (rlo_kernel.hip mover_run): one GPU a fan-out from the origin's copy, "
                         "across GPUs scatter + all-gather",
            "timing": "median round time on world rank 0's clock (announce -> every rank holds the bytes -> "
                      "next originator starts)",
            "baseline": "torch.distributed.broadcast, nccl backend (RCCL), same root" if nccl is not None else None,
            "sizes": out}


def c5_leg(rlo, dist, world, rank, local, stream, red, per=64, k=2048, steps=3, bulk_slots=0, movers=0):
    """BASELINE configs[4] / SURVEY 8(d) C5: mixed sizes log-uniform in [64 B, 1 MiB], collision-heavy
    (slots: in every slot every rank originates, origin(b) = b mod R).  R = 64 ranks per GPU, one
    world over all GPUs, k bcasts per step (fixed: per-GPU receipts stay ~k x 64, weak scaling).
    Messages up to 4 KiB ride the rings; longer ones are bulk messages.  HBM bytes per bcast:
    ring 2(R-1)(S+16); bulk (2R-1)S + 2(R-1)32 (copies written, stripes read, copies verified,
    the announcement)."""
    import numpy as np

    R = per * world
    lo, hi, cap, seed = 64, 1 << 20, 4096, 0xC5
    w = _world(rlo, dist, R, world, rank, local, max_payload=cap, bulk_max=hi, bulk_slots=bulk_slots, movers=movers)
    try:
        w.program_storm(k, lo, seed=seed, len_max=hi, order=1)
        ok, sums, kms = True, [], []
        t0 = 0.0
        for i in range(steps + 1):
            if i == 1:
                if dist is not None:
                    dist.barrier()
                t0 = time.perf_counter()
            rc, ms = _step(w, stream, dist)
            st = w.stats()
            ok &= rc == 0 and bool((st["error"] == 0).all())
            sums.append(st["bcast_sum"].copy())
            if i:
                kms.append(ms)
        dt = red((time.perf_counter() - t0) / steps, "max")
        dump_leg("c5", w, st, seed=seed, k=k, lo=lo, hi=hi, order=1, world_ranks=R)
        ok &= int(red(float(st["originated"].sum()), "sum")) == k
        ok &= int(red(float(st["bcast_delivered"].sum()), "sum")) == k * (R - 1)
        ok &= all(np.array_equal(sums[0], x) for x in sums[1:])
        ok = red(0.0 if ok else 1.0, "max") == 0.0
        lens = rlo.storm_lengths(seed, k, lo, hi).astype(np.float64)
        ring = lens <= cap
        alg = float((2.0 * (R - 1) * (lens[ring] + 16)).sum() + ((2.0 * R - 1) * lens[~ring] + 2.0 * (R - 1) * 32).sum())
        kernel_ms = red(float(np.mean(kms)), "max")
        gbs = alg / world / (kernel_ms * 1e-3) / 1e9
        return {"world_ranks": R, "ranks_per_gpu": per, "bcasts_per_step": k, "bulk_bcasts": int((~ring).sum()),
                "payload_bytes_per_step": int(lens.sum()), "bcast_per_s": round(k / dt, 1),
                "delivered_GBps": round(float(lens.sum()) * (R - 1) / dt / 1e9, 2), "kernel_ms": round(kernel_ms, 3),
                "hbm_alg_GBps_per_gpu": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "verified": bool(ok),
                "movers_per_part": w.info.get("movers"), "bulk_slots": w.info.get("bulk_slots")}
    finally:
        _close(w, dist)


def small_n_legs(rlo, local, stream, sizes=(4, 8), rounds=2000, p=512):
    """the device engine at the reference's own small worlds (4 and 8 ranks on
    one GPU): unloaded one-way latency (origination -> last pickup) and decisions/s with every rank
    keeping one proposal outstanding (approve-all judge on the device)."""
    import numpy as np

    def lat_c4(n, **kw):
        rec = {}
        with rlo.World(n, max_payload=64, device=local, **kw) as w:
            w.program_latency(rounds, 64, seed=21)
            rc0, _ = _step(w, stream, None)
            st = w.stats()
            ok = rc0 == 0 and (st["error"] == 0).all() and int(st["bcast_delivered"].sum()) == rounds * (n - 1)
            lat = w.latencies_ticks().astype(np.float64) * 0.01
            rec["p50_us"] = round(percentile(lat, 50), 2)
            rec["p99_us"] = round(percentile(lat, 99), 2)
            w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(p) for r in range(n)])
            _step(w, stream, None)
            t = time.perf_counter()
            rc, ms = _step(w, stream, None)
            dt = time.perf_counter() - t
            st = w.stats()
            rec["decisions_per_s"] = round(n * p / dt, 1)
            rec["decisions_per_s_kernel"] = round(n * p / (ms * 1e-3), 1)
            rec["decision_us"] = round(ms * 1e3 / p, 2)  # one proposal round trip per rank, back to back
            rec["verified"] = bool(ok and rc == 0 and (st["error"] == 0).all() and int(st["own_decided"].sum()) == n * p)
        return rec

    out = {}
    for n in sizes:
        rec = lat_c4(n)
        # the same programs in a world created with RLO_PART_ONE_XCD: cached rings, every rank-wave on one XCD
        rec["one_xcd"] = lat_c4(n, one_xcd=True)
        rec["verified"] &= rec["one_xcd"]["verified"]
        # the proposal pool (rootless_ops.c:30, unfinished in the reference): 16 own proposals in flight
        # per rank instead of one (:241)
        with rlo.World(n, max_payload=32, device=local, proposal_pool=16) as w:
            pp = 4 * p
            w.program_iar([(r, it * n + r, b"0123456789abcdef") for it in range(pp) for r in range(n)], pool=16)
            _step(w, stream, None)
            t = time.perf_counter()
            rc, ms = _step(w, stream, None)
            dt = time.perf_counter() - t
            st = w.stats()
            rec["pool16_decisions_per_s"] = round(n * pp / dt, 1)
            rec["pool16_decisions_per_s_kernel"] = round(n * pp / (ms * 1e-3), 1)
            rec["verified"] &= bool(rc == 0 and (st["error"] == 0).all() and int(st["own_decided"].sum()) == n * pp)
        out["n%d" % n] = rec
    return out


def reference_datapoint(length, ranks=8):
    """The compiled reference itself (rootless_ops.c + our capture driver) under host MPI: one
    process per rank on the box's cores, 2000 random-origin bcasts."""
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    mpiexec = "/opt/conda/bin/mpiexec"
    if not (os.path.exists(exe) and os.path.exists(mpiexec)):
        return None
    try:
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "o.jsonl")
            subprocess.run(["timeout", "-k", "5", "100", mpiexec, "-bind-to", "core", "-n", str(ranks), exe, out, "bench",
                            "2000", str(length)], cwd=td, timeout=120, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL, check=True)
            rec = json.loads(open(out).read().splitlines()[0])
            rec["cores"] = ranks
            rec["pinning"] = "mpiexec -bind-to core: one core per rank"
            rec["kind"] = "reference"
            return rec
    except Exception as e:  # noqa: BLE001 - informative only
        return {"error": str(e)[:200]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ranks", type=int, default=256, help="workgroup-ranks per GPU")
    ap.add_argument("--len", type=int, default=64, help="payload bytes")
    ap.add_argument("--k", type=int, default=1 << 18, help="bcasts per step")
    ap.add_argument("--lat-rounds", type=int, default=1000)
    ap.add_argument("--iar-p", type=int, default=32, help="proposals per rank for the decisions/s leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip latency / decisions legs")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 PMC traffic passes")
    ap.add_argument("--no-api", action="store_true", help="skip the drop-in rootless_ops.h API leg")
    ap.add_argument("--no-bulk", action="store_true", help="skip the large-message leg (vs RCCL at N > 1)")
    ap.add_argument("--dump", default="", help="directory: every rank writes its ranks' per-leg statistics there "
                                                "(tests/test_gpu_multigpu.py checks them against the oracle)")
    args = ap.parse_args()
    _DUMP["dir"] = args.dump

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RLO_BENCH_DEVICE"):  # rehearsal of the N-part path on one GPU
        local = int(os.environ["RLO_BENCH_DEVICE"])

    # the drop-in API leg runs first, before this process opens the GPU: its 8 MPI ranks each keep
    # a persistent kernel resident, and idle hardware queues held here would share the card with them
    api_leg = None
    if rank == 0 and world == 1 and not args.no_api:
        note("drop-in API leg")
        api_leg = dropin_api_leg()

    import ctypes

    import numpy as np
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        import datetime

        # control plane only: blob exchange, barriers, max-reduce (bounded: a stuck peer ends the run)
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=4))

    import rlo

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    per, length, k = args.ranks, args.len, args.k
    R = per * world  # world size in ranks
    mode = "sharded"
    if world == 1:
        w = rlo.World(R, max_payload=max(64, length), device=local)
    else:
        w, err = None, ""
        try:
            w = rlo.World.part(R, world, rank, max_payload=max(64, length), device=local, uncached=True)
            blobs = [None] * world
            dist.all_gather_object(blobs, w.export())
            w.staged_connect(blobs, dist.barrier, _bcast_blob(dist))  # one exporter at a time (rlo_part_import)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line, never silent
            err = repr(e)[:300]
        errs = [None] * world
        dist.all_gather_object(errs, err)
        if any(errs):
            # the sharded world could not be mapped on this node: fall back to one independent
            # 256-rank world per GPU and SAY so in the line (mode / sharded_error)
            if w is not None:
                w.close()
            mode = "replicas"
            R = per
            w = rlo.World(R, max_payload=max(64, length), device=local)
            sharded_error = [e for e in errs if e][0]
    waves = int(w.info.get("waves", 4))  # rank-workgroup width the world was sized with (4 or 8)
    lib = rlo.abi.load()
    stream = ctypes.c_void_p()
    rlo.abi.check(lib.rlo_stream_create(local, ctypes.byref(stream)), "rlo_stream_create")

    def step():
        return _step(w, stream, dist)

    def red(x, op):
        return {"max": max_over_ranks, "sum": sum_over_ranks}[op](x)

    seed = 0x5EED
    w.program_storm(k, length, seed=seed)
    ok = True
    for _ in range(args.warmup):
        rc, _ = step()
        ok &= rc == 0
    ref_sum = w.stats()["bcast_sum"].copy() if args.warmup else None

    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        rc, ms = step()
        ok &= rc == 0
        kms.append(ms)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    st = w.stats()
    dump_leg("storm", w, st, seed=seed, k=k, len=length, world_ranks=R)
    ok &= bool((st["error"] == 0).all())
    copies = world if mode == "replicas" else 1  # independent worlds each run the whole storm
    ok &= int(sum_over_ranks(float(st["originated"].sum()))) == k * copies
    if ref_sum is not None:
        ok &= bool(np.array_equal(ref_sum, st["bcast_sum"]))  # every step delivers the same bytes

    deliveries = k * (R - 1) * args.steps * copies
    bcast_per_s = k * copies * args.steps / elapsed
    value = bcast_per_s  # BASELINE metric: rootless bcast msgs/s (each reached all R - 1 other ranks)
    kernel_ms = max_over_ranks(float(np.mean(kms)))
    # 2(N-1)(S+16) HBM bytes per bcast; this GPU's share is its ranks' receipts
    alg_bytes = k * 2.0 * (R - 1) * (length + 16) * copies / world
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9

    extras = {"deliveries_per_s": round(deliveries / elapsed, 1), "world_ranks": R, "mode": mode,
              # staged slots whose header lacked the slot mark (each one a device error; 0 expected)
              "unmarked_slots": int(sum_over_ranks(float(st["unmarked_slots"].sum())))}
    if mode == "replicas":
        extras["sharded_error"] = sharded_error
    if world > 1 and mode == "sharded":
        # cross-GPU tree edges per bcast: G-1 .. G; each moves header + payload over xGMI
        extras["xgmi_alg_GBps_per_gpu"] = round(k * (world - 1) * (length + 16) / world / (kernel_ms * 1e-3) / 1e9, 3)
    if not args.no_extras:
        if rank == 0:
            note("latency / loaded-latency / decisions legs")
        # unloaded latency: one random originator per round, round i+1 starts when every rank has
        # picked up round i
        w.program_latency(args.lat_rounds, length, seed=17)
        step()
        dump_leg("latency", w, w.stats(), seed=17, rounds=args.lat_rounds, len=length)
        if world == 1 or mode == "replicas":
            # one-way: origination -> last pickup, both on this GPU's clock
            lat_us = w.latencies_ticks().astype(np.float64) * 0.01
            extras["p50_us"] = round(percentile(lat_us, 50), 2)
            extras["p99_us"] = round(percentile(lat_us, 99), 2)
        if rank == 0:
            # closed-loop round time on ONE clock (world rank 0 observes every completion), the form
            # that stays valid when the world spans GPUs whose clocks are not synchronised
            obs = w.round_ticks().astype(np.float64)
            rt_us = np.diff(obs[obs > 0]) * 0.01
            if len(rt_us):
                extras["round_p50_us"] = round(percentile(rt_us, 50), 2)
                extras["round_p99_us"] = round(percentile(rt_us, 99), 2)
        # loaded per-delivery latency inside the storm (origination clock vs pickup clock: one
        # GPU's clock only when the world is on one GPU, so not reported for sharded N > 1)
        if world == 1 or mode == "replicas":
            w.program_storm(k, length, seed=seed, hist=True)
            step()
            hist = w.stats()["hist"].sum(axis=0).astype(np.float64)
            if dist is not None:
                t = torch.tensor(hist)
                dist.all_reduce(t)
                hist = t.numpy()
            extras["storm_delivery_p50_us"] = round(rlo.hist_percentile(hist, 50) * 0.01, 2)
            extras["storm_delivery_p99_us"] = round(rlo.hist_percentile(hist, 99) * 0.01, 2)
        # consensus: every rank keeps one outstanding proposal (approve-all)
        p = args.iar_p
        props = [(r, it * R + r, b"0123456789abcdef") for it in range(p) for r in range(R)]
        w.program_iar(props)
        step()  # warm
        barrier()
        t1 = time.perf_counter()
        rc, ims = step()
        barrier()
        idt = max_over_ranks(time.perf_counter() - t1)
        ist = w.stats()
        dump_leg("iar", w, ist, p=p)
        extras["decisions_per_s"] = round(R * p * copies / idt, 1)
        extras["decisions_kernel_ms"] = round(max_over_ranks(ims), 3)
        ok &= rc == 0 and int(sum_over_ranks(float(ist["own_decided"].sum()))) == R * p * copies
        ok &= bool((ist["error"] == 0).all())
    _close(w, dist if mode == "sharded" else None)
    if not args.no_extras and world == 1:
        # VERDICT r4 "next" 4: C4 with the pending-proposal tables in HBM (the PH kernels an 8-GPU world's parts run:
        # N x pool x 16 B per rank would crowd a 2048-rank world's LDS), beside the LDS-table number above
        p = args.iar_p
        with rlo.World(R, max_payload=max(64, length), device=local, pend_hbm=True) as wh:
            assert wh.info["pend_hbm"] == 1
            wh.program_iar([(r, it * R + r, b"0123456789abcdef") for it in range(p) for r in range(R)])
            _step(wh, stream, None)
            t1 = time.perf_counter()
            rc, ims = _step(wh, stream, None)
            idt = time.perf_counter() - t1
            ist = wh.stats()
        extras["decisions_per_s_pend_hbm"] = round(R * p / idt, 1)
        extras["decisions_kernel_ms_pend_hbm"] = round(ims, 3)
        if extras.get("decisions_per_s"):
            extras["pend_hbm_cost"] = round(1.0 - extras["decisions_per_s_pend_hbm"] / extras["decisions_per_s"], 4)
        ok &= rc == 0 and int(ist["own_decided"].sum()) == R * p and bool((ist["error"] == 0).all())
    if not args.no_extras and world == 1:
        # the proposal pool at the C4 shape: every rank keeps 16 own proposals in flight (its own world:
        # the pending table is N x 16 entries of LDS, sized at creation)
        p = 4 * args.iar_p
        with rlo.World(R, max_payload=32, device=local, proposal_pool=16) as wp:
            wp.program_iar([(r, it * R + r, b"0123456789abcdef") for it in range(p) for r in range(R)], pool=16)
            _step(wp, stream, None)
            t1 = time.perf_counter()
            rc, ims = _step(wp, stream, None)
            idt = time.perf_counter() - t1
            ist = wp.stats()
        extras["pool16_decisions_per_s"] = round(R * p / idt, 1)
        extras["pool16_decisions_kernel_ms"] = round(ims, 3)
        ok &= rc == 0 and int(ist["own_decided"].sum()) == R * p and bool((ist["error"] == 0).all())
    if not args.no_extras and world == 1:
        # SURVEY 8(d) C2's payload sizes: the same storm at 256 B .. 4 KiB (roofline per size)
        if rank == 0:
            note("payload-size legs")
        extras["payload_sizes"] = size_legs(rlo, R, local, stream)
        ok &= all(s["verified"] for s in extras["payload_sizes"])
    if not args.no_extras and world == 1:
        if rank == 0:
            note("small-world device legs (4 and 8 ranks)")
        extras["small_worlds"] = small_n_legs(rlo, local, stream)
        ok &= all(v["verified"] for v in extras["small_worlds"].values())
    if not args.no_bulk:
        if rank == 0:
            note("bulk leg (C3)")
        try:
            extras["bulk"] = bulk_leg(rlo, dist, world, rank, local, stream, red)
        except Exception as e:  # noqa: BLE001 - reported, never fails the headline line
            extras["bulk"] = {"error": repr(e)[:300]}
            note("rank %d: bulk leg failed: %r" % (rank, e))
        if rank == 0:
            note("mixed-size leg (C5)")
        # a one-GPU rehearsal of more than 2 parts (RLO_BENCH_DEVICE): every part's bulk rank-workgroups and
        # movers (one per CU) must be resident on the one GPU at once -- 16 ranks + 4 movers per part
        c5kw = {"per": 16, "movers": 4} if os.environ.get("RLO_BENCH_DEVICE") and world > 2 else {}
        try:
            extras["c5_mixed"] = c5_leg(rlo, dist, world, rank, local, stream, red, **c5kw)
        except Exception as e:  # noqa: BLE001
            extras["c5_mixed"] = {"error": repr(e)[:300]}
            note("rank %d: C5 leg failed: %r" % (rank, e))
    lib.rlo_stream_destroy(stream)
    ok = bool(sum_over_ranks(0.0 if ok else 1.0) == 0.0)

    line = {
        "metric": "rootless bcast msgs/s",
        "value": round(value, 1),
        "unit": "msgs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": "rootless bcast storm over one world of %d workgroup-ranks (%d per GPU), %d B payload, "
                               "random originators, %d bcasts per step; value = rootless bcasts/s, each delivered "
                               "to all %d other ranks" % (R, per, length, k, R - 1),
                   "ranks_per_gpu": per, "world_ranks": R, "payload_bytes": length, "bcasts_per_step": k,
                   "waves_per_rank": waves,
                   "parallelism": ("one world sharded over %d GPU(s), contiguous rank ranges" % world) if mode == "sharded"
                   else "%d independent %d-rank worlds, one per GPU" % (world, R)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": "rlo_progress_kernel", "kernel_ms": round(kernel_ms, 4),
                     "alg_bytes_per_launch": alg_bytes},
        "verified": ok,
    }
    if world == 1 or mode == "replicas":
        # the timed storm's per-rank delivery counts and checksums, checked against the oracle in the cpu_baseline leg
        line["verified_oracle"] = None
        line["_check"] = {"n": R, "seed": seed, "k": k, "len": length, "count": st["bcast_delivered"].tolist(),
                          "sum": st["bcast_sum"].tolist()}
        _STORM_CHECKS.insert(0, line)
    line.update(extras)
    if rank == 0:
        note("storm timed: %.3f ms/step" % (elapsed / args.steps * 1e3))
    if rank == 0 and world == 1 and not args.no_pmc:
        note("pmc passes")
        tr, why = pmc_traffic(per, length, k, local)
        if tr is not None:
            line["roofline"]["traffic"] = round(tr["bytes"] / 1e9, 4)
            line["roofline"]["traffic_unit"] = "GB per launch (HBM, PMC)"
            line["roofline"]["alg_GB_per_launch"] = round(alg_bytes / 1e9, 4)
            line["roofline"]["traffic_detail"] = tr
        else:
            line["roofline"]["traffic_error"] = why
    if api_leg is not None:
        line["dropin_api"] = api_leg
        # C4 at the reference's own world sizes: the device engine (one GPU) beside
        # the compiled reference under host MPI on the box's cores, same N
        sw = line.get("small_worlds") or {}
        c4 = {}
        for key, rec in sw.items():
            ref = ((api_leg.get(key) or {}).get("reference_host_mpi") or {})
            r_lat, r_dec = (ref.get("lat") or {}).get("p50_us"), (ref.get("iar") or {}).get("decisions_per_s")
            ox = rec.get("one_xcd") or {}
            c4[key] = {"device_p50_us": rec.get("p50_us"), "reference_p50_us": r_lat,
                       "device_decisions_per_s": rec.get("decisions_per_s"),
                       "device_one_xcd_p50_us": ox.get("p50_us"), "device_one_xcd_decisions_per_s": ox.get("decisions_per_s"),
                       "device_pool16_decisions_per_s": rec.get("pool16_decisions_per_s"),
                       "reference_decisions_per_s": r_dec}
            if r_dec:
                c4[key]["decisions_x_reference"] = round(rec["decisions_per_s"] / r_dec, 2)
                if ox.get("decisions_per_s"):
                    c4[key]["one_xcd_decisions_x_reference"] = round(ox["decisions_per_s"] / r_dec, 2)
                if rec.get("pool16_decisions_per_s"):
                    c4[key]["pool16_decisions_x_reference"] = round(rec["pool16_decisions_per_s"] / r_dec, 2)
        if c4:
            line["c4_vs_reference"] = c4
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        note("cpu baseline")
        line["cpu_baseline"] = cpu_baseline(R, length, seed, args.cpu_seconds, bulk=line.get("bulk"))
        if line.get("bulk", {}).get("sizes"):
            line["verified"] = bool(line["verified"] and all(s["verified"] for s in line["bulk"]["sizes"]))
        if line.get("payload_sizes"):
            line["verified"] = bool(line["verified"] and all(s["verified"] for s in line["payload_sizes"]))
    # --no-cpu-baseline: unchecked against the oracle (launch-to-launch equality only)
    for s in (line.get("bulk") or {}).get("sizes", []) + (line.get("payload_sizes") or []) + [line]:
        s.pop("_check", None)
    _STORM_CHECKS.clear()
    dump_write(rank)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
