#!/usr/bin/env python3
"""bench.py -- rootless bcast storm on MI355X (BASELINE.json configs[1]).

One step = one launch of the persistent progress kernel that carries a storm of
K rootless bcasts (random originators, 64-byte payloads by default) across 256
workgroup-ranks until every rank has picked up every bcast it is owed.  Inputs
(schedule, rings) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W]

Multi-GPU (torch.distributed.run, one process per GPU): every GPU hosts its own
256-rank world (weak scaling, no data-path collective); the barrier + max over
ranks timing contract is kept.  One JSON line is printed by rank 0.
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
    out = {"value": k / dt, "unit": "bcast/s", "cores": 1, "kind": "port",
           "sample": "oracle/rlo_oracle.c storm, %d virtual ranks, %d B, %d bcasts (%d deliveries), %.1f s, 1 thread"
                     % (n, length, k, res["deliveries"], dt)}
    ref = reference_datapoint(length)
    if ref:
        out["reference_host_mpi"] = ref
    return out


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
    ap.add_argument("--k", type=int, default=1 << 18, help="bcasts per step (per GPU)")
    ap.add_argument("--lat-rounds", type=int, default=1000)
    ap.add_argument("--iar-p", type=int, default=32, help="proposals per rank for the decisions/s leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip latency / decisions legs")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import rlo

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    n, length, k = args.ranks, args.len, args.k
    stream = torch.cuda.current_stream().cuda_stream
    w = rlo.World(n, max_payload=max(64, length), device=local)
    w.program_storm(k, length, seed=0x5EED + rank)

    for _ in range(args.warmup):
        w.run(stream)
    ref_sum = w.stats()["bcast_sum"].copy() if args.warmup else None

    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        kms.append(w.run(stream))
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    st = w.stats()
    ok = bool((st["error"] == 0).all()) and int(st["originated"].sum()) == k
    if ref_sum is not None:
        ok &= bool(np.array_equal(ref_sum, st["bcast_sum"]))  # every step delivers the same bytes

    total = world * k * args.steps
    value = total / elapsed
    kernel_ms = float(np.mean(kms))
    alg_bytes = k * 2.0 * (n - 1) * (length + 16)  # 2(N-1)(S+16) per bcast
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9

    extras = {}
    if not args.no_extras:
        # unloaded latency: one random originator per round (bcast completion = last pickup)
        w.program_latency(args.lat_rounds, length, seed=17 + rank)
        w.run(stream)
        lat_us = w.latencies_ticks().astype(np.float64) * 0.01
        extras["p50_us"] = round(percentile(lat_us, 50), 2)
        extras["p99_us"] = round(percentile(lat_us, 99), 2)
        # loaded per-delivery latency inside the storm
        w.program_storm(k, length, seed=0x5EED + rank, hist=True)
        w.run(stream)
        hist = w.stats()["hist"].sum(axis=0)
        extras["storm_delivery_p50_us"] = round(rlo.hist_percentile(hist, 50) * 0.01, 2)
        extras["storm_delivery_p99_us"] = round(rlo.hist_percentile(hist, 99) * 0.01, 2)
        # consensus: every rank keeps one outstanding proposal (approve-all)
        p = args.iar_p
        props = [(r, it * n + r, b"0123456789abcdef") for it in range(p) for r in range(n)]
        w.program_iar(props)
        w.run(stream)  # warm
        barrier()
        t1 = time.perf_counter()
        ims = w.run(stream)
        barrier()
        idt = max_over_ranks(time.perf_counter() - t1)
        ist = w.stats()
        extras["decisions_per_s"] = round(world * n * p / idt, 1)
        extras["decisions_kernel_ms"] = round(ims, 3)
        ok &= int(ist["own_decided"].sum()) == n * p and bool((ist["error"] == 0).all())
    w.close()

    line = {
        "metric": "rootless bcast msgs/s",
        "value": round(value, 1),
        "unit": "bcast/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": "rootless bcast storm, %d workgroup-ranks per GPU, %d B payload, random originators, "
                               "%d bcasts per step per GPU" % (n, length, k),
                   "ranks_per_gpu": n, "payload_bytes": length, "bcasts_per_step": k,
                   "parallelism": "one %d-rank world per GPU" % n},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": "rlo_progress_kernel", "kernel_ms": round(kernel_ms, 4),
                     "alg_bytes_per_launch": alg_bytes},
        "verified": ok,
    }
    line.update(extras)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(n, length, 0x5EED, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
