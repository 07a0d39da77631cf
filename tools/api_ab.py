"""A/B of drop-in builds on one box: tools/api_bench.c (rlo_api_bench) from each build directory given
(default: the product lib/ and every tools/ab_libs/*/), legs interleaved rep by rep so box-to-box and
run-to-run drift hit every build alike, beside the compiled reference; prints the median per leg.

  python3 tools/api_ab.py [--reps 3] [--ranks 4 8] [dir ...]
"""
import argparse
import glob
import json
import os
import statistics
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = "/opt/conda/bin/mpiexec"
LEGS = [("iar", ["iar", "2000"], "decisions_per_s"), ("iardj", ["iardj", "2000"], "decisions_per_s"),
        ("lat", ["lat", "500", "64"], "p50_us"), ("storm", ["storm", "20000", "64"], "bcast_per_s")]


def run(exe, nr, args, bind=False, env=None):
    cmd = ["timeout", "-k", "5", "120", MPIEXEC] + (["-bind-to", "core"] if bind else []) + ["-n", str(nr), exe] + args
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=140, env=env)
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else {"error": "rc=%d" % r.returncode}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ranks", type=int, nargs="+", default=[4, 8])
    ap.add_argument("dirs", nargs="*")
    a = ap.parse_args()
    dirs = a.dirs or [os.path.join(REPO, "rootless-coll-mpi-ops_amd", "lib")] + sorted(glob.glob(os.path.join(REPO, "tools", "ab_libs", "*")))
    builds = {os.path.basename(os.path.dirname(d)) if d.endswith("/lib") else os.path.basename(d.rstrip("/")): os.path.join(d, "rlo_api_bench") for d in dirs}
    builds["reference"] = os.path.join(REPO, "oracle", "_ref", "ref_api_bench")
    res = {}
    for rep in range(a.reps):
        for nr in a.ranks:
            for leg, args, key in LEGS:
                for b, exe in builds.items():
                    if b == "reference" and leg == "iardj":
                        continue
                    if not os.path.exists(exe):
                        continue
                    # ours as bench.py runs it (the application thread on the GPU's NUMA node too)
                    env = None if b == "reference" else dict(os.environ, RLO_NUMA_BIND="all")
                    v = run(exe, nr, args, bind=(b == "reference"), env=env).get(key)
                    res.setdefault((nr, leg, b), []).append(v)
    for (nr, leg, b), vs in sorted(res.items()):
        ok = [v for v in vs if isinstance(v, (int, float))]
        print("n%d %-6s %-10s median %10.1f  all %s" % (nr, leg, b, statistics.median(ok) if ok else float("nan"),
                                                         [round(v, 1) if isinstance(v, float) else v for v in vs]), flush=True)


if __name__ == "__main__":
    main()
