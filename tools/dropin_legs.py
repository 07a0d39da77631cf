"""Where the drop-in's time goes: splits a bcast's and a host-judged proposal's time into legs
from the host traces the library writes with RLO_TRACE_DIR (rootless_ops.cpp `trace`; one CLOCK_MONOTONIC for every
rank process of the node).

  RLO_TRACE_DIR=d mpiexec -n 8 rlo_api_bench lat 500 64 ; python tools/dropin_legs.py d
  RLO_TRACE_DIR=d mpiexec -n 8 rlo_api_bench iar 2000   ; python tools/dropin_legs.py d

bcast (one at a time): command posted -> the kernel's command head seen past it on the host ("command in", as
the host sees the head), posted -> each receiver's event seen; the device's own origination -> pickup-record time
(event aux) splits the latter into device and host (command in + pickup out) parts.
proposal: submit -> every judge request seen (per tree hop: the parent's verdict or the submit -> the child's
request seen), request seen -> handled (queued behind other events) -> verdict posted, last verdict -> the
originator's judge(NULL) request seen (votes up), its verdict -> decisions seen / result seen."""
import glob
import os
import sys
from collections import defaultdict

import numpy as np

EV_BCAST, EV_DECISION, EV_RESULT, EV_JUDGE, EV_OWN = 1, 1 | (4 << 8), 4, 6, 7
CMD_BCAST, CMD_PROPOSAL, CMD_JUDGE, CMD_OWN = 0, 2, 16, 17


def load(d):
    recs = {}
    for f in sorted(glob.glob(os.path.join(d, "trace_rank*_e*.txt"))):
        rank = int(os.path.basename(f).split("_")[1][4:])
        rows = []
        for ln in open(f):
            if ln.startswith("#"):
                continue
            t, w, k, o, i, fr, aux = ln.split()
            rows.append((int(t), w, int(k), int(o), int(i), int(fr), int(aux)))
        recs[rank] = rows
    return recs


def pct(x, q):
    return round(float(np.percentile(x, q)), 2) if len(x) else float("nan")


def summary(name, x):
    x = np.asarray(x, dtype=np.float64)
    print("  %-46s p50 %8.2f  p90 %8.2f  mean %8.2f us  (%d)" % (name, pct(x, 50), pct(x, 90), x.mean() if len(x) else float("nan"), len(x)))


def bcasts(recs):
    posts = {}  # (origin, id) -> t
    for r, rows in recs.items():
        cons = [t for t, w, *_ in rows if w == "C"]
        for t, w, k, o, i, fr, aux in rows:
            if w == "P" and k == CMD_BCAST:
                c = next((tc for tc in cons if tc >= t), None)
                posts[(r, i)] = (t, c)
    seen = defaultdict(list)
    for r, rows in recs.items():
        for t, w, k, o, i, fr, aux in rows:
            if w == "S" and k == EV_BCAST:
                seen[(o, i)].append((t, aux))
    host, dev, rest, cin, first = [], [], [], [], []
    for key, (tp, tc) in posts.items():
        s = seen.get(key)
        if not s:
            continue
        tl = max(t for t, _ in s)
        host.append((tl - tp) / 1e3)
        first.append((min(t for t, _ in s) - tp) / 1e3)
        a = max(aux for _, aux in s) * 0.01
        dev.append(a)
        rest.append((tl - tp) / 1e3 - a)
        if tc is not None:
            cin.append((tc - tp) / 1e3)
    if not host:
        return
    print("bcasts: %d" % len(host))
    summary("posted -> last receiver's event seen (host)", host)
    summary("posted -> first receiver's event seen", first)
    summary("device: origination -> last pickup record", dev)
    summary("host part: command in + pickup out", rest)
    summary("posted -> command head past it (seen on host)", cin)


def proposals(recs):
    sub, verdict, jseen, jhand, own_seen, own_post, res, dec = {}, {}, {}, {}, {}, {}, {}, defaultdict(list)
    parent = {}
    for r, rows in recs.items():
        for t, w, k, o, i, fr, aux in rows:
            if w == "P" and k == CMD_PROPOSAL:
                sub[(r, i)] = t
            elif w == "P" and k == CMD_JUDGE:
                verdict[(o, i, r)] = t
            elif w == "P" and k == CMD_OWN:
                own_post[(r, i)] = t
            elif w == "S" and k == EV_JUDGE:
                jseen[(o, i, r)] = t
                parent[(o, i, r)] = fr
            elif w == "H" and k == EV_JUDGE:
                jhand[(o, i, r)] = t
            elif w == "S" and k == EV_OWN:
                own_seen[(r, i)] = t
            elif w == "S" and k == EV_RESULT:
                res[(r, i)] = t
            elif w == "S" and k == EV_DECISION:
                dec[(o, i)].append(t)
    if not sub:
        return
    # command in: a verdict posted -> the first time this rank saw the kernel's command head past it
    cin = []
    for r, rows in recs.items():
        cons = [(t, i) for t, w, k, o, i, fr, aux in rows if w == "C"]  # time order, counts non-decreasing
        ci = 0
        for t, w, k, o, i, fr, aux in rows:
            if w == "P" and k == CMD_JUDGE and fr > 0:
                while ci < len(cons) and cons[ci][0] < t:
                    ci += 1
                cj = ci
                while cj < len(cons) and cons[cj][1] < fr:
                    cj += 1
                if cj < len(cons):
                    cin.append((cons[cj][0] - t) / 1e3)
    hop, queue, cb, up, ownsvc, decl, resl, total, down = [], [], [], [], [], [], [], [], []
    for (o, pid), ts in sub.items():
        if (o, pid) not in res:
            continue
        total.append((res[(o, pid)] - ts) / 1e3)
        vs = []
        last_j = ts
        for (oo, ii, r), tj in jseen.items():
            if oo != o or ii != pid:
                continue
            p = parent[(o, pid, r)]
            tpar = ts if p == o else verdict.get((o, pid, p))
            if tpar is not None:
                hop.append((tj - tpar) / 1e3)
            if (o, pid, r) in jhand:
                queue.append((jhand[(o, pid, r)] - tj) / 1e3)
                if (o, pid, r) in verdict:
                    cb.append((verdict[(o, pid, r)] - jhand[(o, pid, r)]) / 1e3)
            if (o, pid, r) in verdict:
                vs.append(verdict[(o, pid, r)])
            last_j = max(last_j, tj)
        down.append((last_j - ts) / 1e3)
        if vs and (o, pid) in own_seen:
            up.append((own_seen[(o, pid)] - max(vs)) / 1e3)
        if (o, pid) in own_seen and (o, pid) in own_post:
            ownsvc.append((own_post[(o, pid)] - own_seen[(o, pid)]) / 1e3)
        if (o, pid) in own_post:
            if dec.get((o, pid)):
                decl.append((max(dec[(o, pid)]) - own_post[(o, pid)]) / 1e3)
            resl.append((res[(o, pid)] - own_post[(o, pid)]) / 1e3)
    print("proposals: %d decided" % len(total))
    summary("submit -> result seen (total)", total)
    summary("submit -> last judge request seen (down)", down)
    summary("one hop: parent's verdict/submit -> request seen", hop)
    summary("verdict posted -> command head past it (seen)", cin)
    summary("request seen -> handled (app thread queue)", queue)
    summary("handled -> verdict posted (judge callback)", cb)
    summary("last verdict posted -> own judge(NULL) seen (up)", up)
    summary("own judge(NULL) seen -> posted", ownsvc)
    summary("own verdict posted -> last decision seen", decl)
    summary("own verdict posted -> result seen", resl)


def main():
    recs = load(sys.argv[1])
    if not recs:
        print("no traces in", sys.argv[1])
        return
    print("%s: %d rank traces" % (sys.argv[1], len(recs)))
    bcasts(recs)
    proposals(recs)


if __name__ == "__main__":
    main()
