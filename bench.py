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


def cpu_baseline(n, length, seed, target_s):
    """The oracle's clean-room CPU restatement ("port"), one host core, bounded sample."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle as orc

    t = time.perf_counter()
    orc.storm(n, seed, 2000, length)
    per = (time.perf_counter() - t) / 2000
    k = int(max(2000, min(2_000_000, target_s / max(per, 1e-9))))
    t = time.perf_counter()
    res = orc.storm(n, seed, k, length)
    dt = time.perf_counter() - t
    out = {"value": k / dt, "unit": "msgs/s", "deliveries_per_s": res["deliveries"] / dt, "cores": 1, "kind": "port",
           "sample": "oracle/rlo_oracle.c storm, %d virtual ranks, %d B, %d bcasts (%d deliveries), %.1f s, 1 thread"
                     % (n, length, k, res["deliveries"], dt)}
    ref = reference_datapoint(length)
    if ref:
        out["reference_host_mpi"] = ref
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


def dropin_api_leg(ranks=8, timeout_s=150):
    """The drop-in rootless_ops.h path end to end: tools/api_bench.c over librootless_ops.so
    (one MPI process per rank, every rank's engine a persistent kernel on this GPU) beside the
    same driver linked against the compiled reference under host MPI on the box's cores."""
    mpiexec = "/opt/conda/bin/mpiexec"
    ours = os.path.join(PKG, "lib", "rlo_api_bench")
    ref = os.path.join(REPO, "oracle", "_ref", "ref_api_bench")
    if not (os.path.exists(mpiexec) and os.path.exists(ours)):
        return {"error": "mpiexec or rlo_api_bench missing"}
    out = {"ranks": ranks, "driver": "tools/api_bench.c (same calls for both)", "ours": {}, "reference_host_mpi": {}}
    # all ranks' persistent kernels share the one GPU here: 2 hardware queues per single-engine rank
    # process keep their queues within the GPU's slots (deployment note)
    env = dict(os.environ)
    env.setdefault("GPU_MAX_HW_QUEUES", "2")
    out["env"] = {"GPU_MAX_HW_QUEUES": env["GPU_MAX_HW_QUEUES"]}
    legs = [("storm", ["storm", "20000", "64"]), ("lat", ["lat", "500", "64"]), ("iar", ["iar", "2000"])]
    for name, exe in (("ours", ours), ("reference_host_mpi", ref)):
        if not os.path.exists(exe):
            out[name] = {"error": "not built"}
            continue
        for leg, args in legs:
            note("api %s %s" % (name, leg))
            try:
                r = subprocess.run(["timeout", "-k", "5", str(timeout_s), mpiexec, "-n", str(ranks), exe] + args,
                                   stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=timeout_s + 20, env=env)
                lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
                out[name][leg] = json.loads(lines[-1]) if lines else {"error": "rc=%d" % r.returncode}
            except Exception as e:  # noqa: BLE001 - informative leg, never fails the bench
                out[name][leg] = {"error": str(e)[:200]}
    try:
        o, f = out["ours"], out["reference_host_mpi"]
        out["ratio_vs_reference"] = {
            "bcast_per_s": round(o["storm"]["bcast_per_s"] / f["storm"]["bcast_per_s"], 2),
            "decisions_per_s": round(o["iar"]["decisions_per_s"] / f["iar"]["decisions_per_s"], 2),
            "p50_latency": round(o["lat"]["p50_us"] / f["lat"]["p50_us"], 2)}
    except Exception:  # noqa: BLE001
        pass
    out["cores"] = ranks
    return out


def size_legs(rlo, R, device, stream, sizes=(256, 1024, 4096), k=1 << 16, steps=3):
    """The headline storm at SURVEY 8(d) C2's larger payloads (one GPU): bcast/s and the HBM
    roofline fraction per size, 2(N-1)(S+16) algorithmic bytes per bcast as for `value`.  Every
    step must deliver the same bytes (per-rank checksums equal across steps)."""
    import numpy as np

    out = []
    with rlo.World(R, max_payload=max(sizes), device=device) as w:
        for s in sizes:
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
            out.append({"payload_bytes": s, "bcasts": k, "bcast_per_s": round(k / dt, 1),
                        "deliveries_per_s": round(k * (R - 1) / dt, 1), "kernel_ms": round(kernel_ms, 3),
                        "alg_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "verified": ok})
    return out


def bulk_leg(dist, world, rank, local, sizes_mib=(1, 4, 16, 64), iters=5, blocks=None):
    """BASELINE configs[2]: large-message rootless bcast (pipelined scatter + all-gather over the
    ranks' HBM buffers, rlo_bulk.hip) from rotating originators vs rooted RCCL broadcast of the
    same bytes from the same root.  N > 1: one rank per GPU.  N = 1: an 8-rank world on the one
    GPU (HBM only; no RCCL counterpart).  Every receiver checks every byte."""
    import torch

    import rlo
    from rlo.bulk import Bulk

    G = world if world > 1 else 8
    maxb = max(sizes_mib) << 20
    blocks = blocks or 0  # 0: the library sizes workgroups and chunks (rlo_bulk_launch)
    if world > 1:
        w = rlo.World.part(G, G, rank, max_payload=64, device=local, uncached=True)
        blobs = [None] * world
        dist.all_gather_object(blobs, w.export())
        w.connect(blobs)
        b = Bulk(w, maxb)
        bb = [None] * world
        dist.all_gather_object(bb, b.export())
        b.connect(bb)
        mine = [rank]
        # rehearsal of the N-part path on one GPU (RLO_BENCH_DEVICE): RCCL refuses two ranks per GPU
        nccl = None if os.environ.get("RLO_BENCH_DEVICE") else dist.new_group(backend="nccl")
    else:
        w = rlo.World(G, max_payload=64, device=local)
        b = Bulk(w, maxb)
        b.connect([b.export()])
        mine = list(range(G))
        nccl = None

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    def maxr(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    out = []
    try:
        for mib in sizes_mib:
            nbytes = mib << 20
            ours, ok = [], True
            for it in range(iters + 1):
                o = it % G
                gen = torch.Generator(device="cuda").manual_seed(1000 * mib + o)
                want = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=gen)
                if o in mine:
                    b.tensor(o)[:nbytes].copy_(want)
                barrier()
                b.reset()
                barrier()
                b.launch(o, nbytes, blocks=blocks)
                ms, rc = b.wait(raise_on_error=False)
                ok &= rc == 0
                for r in mine:
                    if r != o:
                        ok &= bool(torch.equal(b.tensor(r)[:nbytes], want))
                ms = maxr(ms)
                if it:  # the first launch is a warmup
                    ours.append(ms)
            if rank == 0:
                note("bulk %d MiB ours done" % mib)
            rec = {"MiB": mib, "ours_ms": round(sorted(ours)[len(ours) // 2], 4), "verified": ok}
            rec["ours_algbw_GBps"] = round(nbytes / (rec["ours_ms"] * 1e-3) / 1e9, 2)
            if nccl is not None:
                t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                rc = []
                for it in range(iters + 2):
                    o = it % G
                    barrier()
                    e0.record()
                    dist.broadcast(t, src=o, group=nccl)
                    e1.record()
                    torch.cuda.synchronize()
                    if it >= 2:
                        rc.append(maxr(e0.elapsed_time(e1)))
                rec["rccl_ms"] = round(sorted(rc)[len(rc) // 2], 4)
                rec["rccl_algbw_GBps"] = round(nbytes / (rec["rccl_ms"] * 1e-3) / 1e9, 2)
                rec["ours_over_rccl"] = round(rec["rccl_ms"] / rec["ours_ms"], 3)
            else:  # one GPU: every receiver's copy written once (N-1)S; the originator reads S to
                # scatter, the stripe owners read S between them to all-gather: (N+1)S HBM bytes
                rec["hbm_GBps"] = round(((G + 1) * nbytes) / (rec["ours_ms"] * 1e-3) / 1e9, 1)
            out.append(rec)
    finally:
        b.close()
        w.close()
    return {"ranks": G, "ranks_per_gpu": 1 if world > 1 else G, "blocks_per_rank": blocks or "auto",
            "algorithm": "pipelined scatter + all-gather over per-rank HBM buffers (rlo_bulk.hip)",
            "baseline": "torch.distributed.broadcast, nccl backend (RCCL), same root" if world > 1 else None,
            "sizes": out}


def reference_datapoint(length):
    """The compiled reference itself under host MPI (8 ranks), if it was built and MPI exists."""
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    mpiexec = "/opt/conda/bin/mpiexec"
    if not (os.path.exists(exe) and os.path.exists(mpiexec)):
        return None
    try:
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "o.jsonl")
            subprocess.run([mpiexec, "-n", "8", exe, out, "bench", "2000", str(length)], cwd=td, timeout=120,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
            rec = json.loads(open(out).read().splitlines()[0])
            rec["cores"] = 8
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
    args = ap.parse_args()

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
            w.connect(blobs)
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
        """one launch of the loaded program; every part reset before any part launches"""
        w.reset(stream)
        if dist is not None:
            dist.barrier()
        w.launch(stream, no_reset=True)
        rc = w.wait(raise_on_device_error=False)
        if dist is not None:
            dist.barrier()  # no peer still stores into this part's rings
        return rc, w.kernel_ms()

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
        extras["decisions_per_s"] = round(R * p * copies / idt, 1)
        extras["decisions_kernel_ms"] = round(max_over_ranks(ims), 3)
        ok &= rc == 0 and int(sum_over_ranks(float(ist["own_decided"].sum()))) == R * p * copies
        ok &= bool((ist["error"] == 0).all())
    w.close()
    if not args.no_extras and world == 1:
        # SURVEY 8(d) C2's payload sizes: the same storm at 256 B .. 4 KiB (roofline per size)
        if rank == 0:
            note("payload-size legs")
        extras["payload_sizes"] = size_legs(rlo, R, local, stream)
        ok &= all(s["verified"] for s in extras["payload_sizes"])
    lib.rlo_stream_destroy(stream)
    if not args.no_bulk:
        if rank == 0:
            note("bulk leg")
        try:
            extras["bulk"] = bulk_leg(dist, world, rank, local)
        except Exception as e:  # noqa: BLE001 - reported, never fails the headline line
            extras["bulk"] = {"error": repr(e)[:300]}
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
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        note("cpu baseline")
        line["cpu_baseline"] = cpu_baseline(R, length, seed, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
