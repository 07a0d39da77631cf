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

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
MPIEXEC = "/opt/conda/bin/mpiexec"


def run(n, *args, timeout=600):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "out.jsonl")
        cmd = [MPIEXEC, "-n", str(n), HARNESS, out] + [str(a) for a in args]
        subprocess.run(cmd, check=True, timeout=timeout, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=td)
        with open(out) as f:
            return [json.loads(line) for line in f if line.strip()]


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
        recs = run(n, "parents", length, timeout=3600)
        parent = [[-1] * n for _ in range(n)]
        hashes = [None] * n
        for r in recs:
            assert r["type"] == 0 and r["hdr_origin"] == r["origin"] and r["pid"] == -1 and r["vote"] == -1 and r["data_len"] == 0
            assert parent[r["origin"]][r["rank"]] == -1, "duplicate delivery"
            parent[r["origin"]][r["rank"]] = r["parent"]
            assert hashes[r["origin"]] in (None, r["hash"])
            hashes[r["origin"]] = r["hash"]
        assert len(recs) == n * (n - 1)
        out[str(n)] = {"parent": parent, "hash": hashes}
    return out


def gen_stream(cases):
    out = []
    for n, seed, k, length in cases:
        recs = run(n, "stream", seed, k, length)
        per = [[] for _ in range(n)]
        for r in recs:
            assert r["type"] == 0
            per[r["rank"]].append([r["bid"], r["origin"], r["parent"], r["hash"]])
        for p in per:
            p.sort()
        out.append({"n": n, "seed": seed, "k": k, "len": length, "deliveries": per})
    return out


def gen_iar(n, cases):
    out = []
    for origin, mask in cases:
        recs = run(n, "iar", origin, mask)
        judge = sorted([r["rank"], r["null"], r["arg"]] for r in recs if r["ev"] == "judge")
        actions = sorted([r["rank"], r["pid"], r["vote"], r["data_len"], r["data"]] for r in recs if r["ev"] == "action")
        pickups = sorted([r["rank"], r["type"], r["pid"], r["vote"], r["data_len"], r["data"], r["origin"]]
                         for r in recs if r["ev"] == "pickup")
        result = [r["vote"] for r in recs if r["ev"] == "result"]
        assert len(result) == 1
        out.append({"n": n, "origin": origin, "mask": mask, "judge": judge, "actions": actions, "pickups": pickups,
                    "decision": result[0]})
    return out


def gen_multi(n, cases):
    out = []
    for a1, mod, agree in cases:
        recs = run(n, "multi", a1, mod, agree)
        judge = sorted([r["rank"], r["null"], r["arg"], r["ret"]] for r in recs if r["ev"] == "judge")
        decisions = sorted([r["rank"], r["pid"], r["vote"], r["origin"]] for r in recs if r["ev"] == "decision")
        results = sorted([r["rank"], r["pid"], r["vote"]] for r in recs if r["ev"] == "result")
        out.append({"n": n, "active_1": a1, "mod": mod, "agree": agree, "judge": judge, "decisions": decisions, "results": results})
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


if __name__ == "__main__":
    main()
