"""Run the capture driver (oracle/ref_harness.c) under host MPI and reduce its JSON lines
to the fixture records of tests/golden/*.json.

TEST INFRASTRUCTURE ONLY.  The same driver source is built twice (oracle/Makefile):
  oracle/_ref/ref_harness     linked with the compiled reference -> gen_fixtures.py
  oracle/_ref/dropin_harness  linked with librootless_ops.so     -> tests/test_gpu_dropin.py
so the drop-in is checked with exactly the calls that produced the fixtures.
"""
import json
import os
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
DROPIN_HARNESS = os.path.join(REPO, "oracle", "_ref", "dropin_harness")
MPIEXEC = "/opt/conda/bin/mpiexec"


def run(exe, n, *args, timeout=600, env=None, want_stdout=False):
    """mpiexec -n N exe OUT args... -> list of JSON records (rank 0 gathers every rank's lines);
    with want_stdout, (records, combined stdout/stderr text)"""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "out.jsonl")
        cmd = ["timeout", "-k", "10", str(timeout), MPIEXEC, "-n", str(n), exe, out] + [str(a) for a in args]
        r = subprocess.run(cmd, timeout=timeout + 30, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, cwd=td, env=env)
        if r.returncode != 0:
            raise RuntimeError("%s exited %d:\n%s" % (" ".join(cmd), r.returncode, r.stdout.decode(errors="replace")[-4000:]))
        with open(out) as f:
            recs = [json.loads(line) for line in f if line.strip()]
        return (recs, r.stdout.decode(errors="replace")) if want_stdout else recs


def parents(recs, n):
    parent = [[-1] * n for _ in range(n)]
    hashes = [None] * n
    for r in recs:
        assert r["type"] == 0 and r["hdr_origin"] == r["origin"] and r["pid"] == -1 and r["vote"] == -1 and r["data_len"] == 0, r
        assert parent[r["origin"]][r["rank"]] == -1, "duplicate delivery"
        parent[r["origin"]][r["rank"]] = r["parent"]
        assert hashes[r["origin"]] in (None, r["hash"])
        hashes[r["origin"]] = r["hash"]
    assert len(recs) == n * (n - 1)
    return {"parent": parent, "hash": hashes}


def stream(recs, n):
    per = [[] for _ in range(n)]
    for r in recs:
        assert r["type"] == 0
        per[r["rank"]].append([r["bid"], r["origin"], r["parent"], r["hash"]])
    for p in per:
        p.sort()
    return per


def iar(recs):
    judge = sorted([r["rank"], r["null"], r["arg"]] for r in recs if r["ev"] == "judge")
    actions = sorted([r["rank"], r["pid"], r["vote"], r["data_len"], r["data"]] for r in recs if r["ev"] == "action")
    pickups = sorted([r["rank"], r["type"], r["pid"], r["vote"], r["data_len"], r["data"], r["origin"]]
                     for r in recs if r["ev"] == "pickup")
    result = [r["vote"] for r in recs if r["ev"] == "result"]
    assert len(result) == 1, recs
    return {"judge": judge, "actions": actions, "pickups": pickups, "decision": result[0]}


def multi(recs):
    judge = sorted([r["rank"], r["null"], r["arg"], r["ret"]] for r in recs if r["ev"] == "judge")
    decisions = sorted([r["rank"], r["pid"], r["vote"], r["origin"]] for r in recs if r["ev"] == "decision")
    results = sorted([r["rank"], r["pid"], r["vote"]] for r in recs if r["ev"] == "result")
    return {"judge": judge, "decisions": decisions, "results": results}
