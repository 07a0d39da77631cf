#!/usr/bin/env python3
"""Generate golden fixtures by RUNNING THE COMPILED REFERENCE under host MPI.

TEST INFRASTRUCTURE ONLY.  Needs /root/reference (this container only) and the
image's MPICH (/opt/conda).  Builds oracle/_ref/ref_harness via `make -C oracle ref`
(the reference sources are compiled where they lie; nothing is copied), runs the
capture modes of oracle/ref_harness.c and writes compact JSON fixtures next to
this script.  The fixtures are data: inputs and the reference's observed outputs.

    python tests/golden/gen_fixtures.py            # default set (~2 min on 8 cores)
    python tests/golden/gen_fixtures.py --big      # + parents at N=128/255/256/257 (slow)
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import capture  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
MPIEXEC = "/opt/conda/bin/mpiexec"


def run(n, *args, timeout=600):
    return capture.run(HARNESS, n, *args, timeout=timeout)


def dump(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, separators=(",", ":"), sort_keys=True)
        f.write("\n")
    print("wrote", os.path.relpath(path, REPO), file=sys.stderr)


def gen_topo(nmax=1024):
    recs = run(1, "topo", nmax)
    level0 = {r["n"]: r["level0"] for r in recs if "n" in r}
    levels = [None] + [r["level"] for r in recs if "rank" in r]
    walls = [None] + [r["last_wall_fn"] for r in recs if "rank" in r]
    dump("topo.json", {"nmax": nmax, "level0": [level0[n] for n in range(2, nmax + 1)], "level": levels, "last_wall_fn": walls,
                       "source": "rootless_ops.c:1427-1452 get_level/last_wall, compiled reference"})


def gen_parents(ns, length=64):
    out = {}
    for n in ns:
        out[str(n)] = capture.parents(run(n, "parents", length, timeout=3600), n)
    return out


def gen_stream(cases):
    out = []
    for n, seed, k, length in cases:
        per = capture.stream(run(n, "stream", seed, k, length), n)
        out.append({"n": n, "seed": seed, "k": k, "len": length, "deliveries": per})
    return out


def gen_iar(n, cases):
    out = []
    for origin, mask in cases:
        c = capture.iar(run(n, "iar", origin, mask))
        c.update({"n": n, "origin": origin, "mask": mask})
        out.append(c)
    return out


def gen_multi(n, cases):
    out = []
    for a1, mod, agree in cases:
        c = capture.multi(run(n, "multi", a1, mod, agree))
        c.update({"n": n, "active_1": a1, "mod": mod, "agree": agree})
        out.append(c)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    args = ap.parse_args()
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)

    gen_topo()
    ns = list(range(2, 18)) + [31, 32, 33, 64]
    if args.big:
        ns += [128, 255, 256, 257]
    dump("parents.json", {"len": 64, "by_n": gen_parents(ns),
                          "source": "receiver-side MPI_SOURCE of each delivered bcast (rootless_ops.h:115), one bcast per origin"})
    dump("stream.json", {"cases": gen_stream([(4, 7, 64, 64), (5, 3, 40, 8), (8, 11, 64, 1000), (13, 5, 52, 200)])})

    iar = []
    iar += gen_iar(4, [(o, 0) for o in range(4)] + [(1, 1 << 2), (0, 1 << 3), (2, 1 << 1), (3, 0b0101)])
    iar += gen_iar(8, [(o, 0) for o in range(8)] + [(1, 1 << 4), (5, 1 << 0), (3, 1 << 6), (0, 0b10010010), (6, 1 << 7),
                                                     (7, 1 << 3), (2, 0b01000001)])
    iar += gen_iar(16, [(0, 0), (5, 0), (15, 0), (9, 0), (5, 1 << 6), (12, 1 << 2), (0, 1 << 15), (3, 0b1000000010000000)])
    dump("iar.json", {"cases": iar, "judge": "decline iff (mask>>rank)&1 and arg!=NULL; proposal 'proposal-from-<o>', pid 100+o"})

    multi = gen_multi(4, [(1, 3, 1), (1, 3, 0)]) + gen_multi(8, [(1, 3, 1), (1, 3, 0), (5, 2, 0), (2, 4, 0)])
    dump("multi.json", {"cases": multi, "judge": "testcases.c:18-37 is_proposal_approved_cb, roles of testcases.c:401-486"})

    tests = run(4, "tests", timeout=900)
    dump("testcases.json", {"n": 4, "results": tests})
    tests2 = run(4, "tests2", timeout=900)
    dump("testcases2.json", {"n": 4, "results": tests2})


if __name__ == "__main__":
    main()
