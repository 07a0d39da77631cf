"""Exact-set IAR parity: the device's event records against the pool oracle
(orc_iar_rounds_pool), per (origin, pid) -- TEST INFRASTRUCTURE ONLY.

Every rank runs p proposals (pid = it * n + r) keeping `pool` in flight; judge = the seeded hash judge
(ppm declines per judge call; 0 = approve-all).  The sets compared:
  judge   (rank, origin, pid, NULL arg, verdict)   -- every judge call, the originator's final one too
  action  (rank, origin, pid)                      -- action() at every rank that approved, decision 1
  pickup  (rank, origin, pid, decision)            -- every decision delivery
  result  (rank, pid, decision)                    -- every originator's result
A record seen twice fails (a set would hide it), and so does any swap of pids between two
proposals that keeps the sums equal.
"""
import pyoracle as orc

LOG_DELIVER, LOG_JUDGE, LOG_ACTION, LOG_RESULT = 1, 2, 3, 4
TAG_DECISION = 4


def props(n, p, data=b"0123456789abcdef"):
    return [(r, it * n + r, data) for it in range(p) for r in range(n)]


def check(logs, n, p, ppm, pool, seed=99):
    """logs: {rank: rows of World.log(rank)} for every world rank"""
    cfg, keep = orc.judge_cfg(orc.ORC_JUDGE_HASH if ppm else orc.ORC_JUDGE_APPROVE, seed=seed, ppm=ppm)
    ev = orc.iar_rounds(n, p, cfg, pool=pool)
    want = {"judge": set(), "action": set(), "pickup": set(), "result": set()}
    for e, rank, pid, a, b, c in ev:
        if e == orc.ORC_EV_JUDGE:
            want["judge"].add((rank, c, pid, a, b))
        elif e == orc.ORC_EV_ACTION:
            want["action"].add((rank, c, pid))
        elif e == orc.ORC_EV_PICKUP:
            want["pickup"].add((rank, b, pid, a))
        elif e == orc.ORC_EV_RESULT:
            want["result"].add((rank, pid, a))
    got = {k: set() for k in want}
    counts = {k: 0 for k in want}
    for r in range(n):
        for kind_, tag, origin, frm, pid, ln, vote, aux, _ in logs[r]:
            if kind_ == LOG_JUDGE:
                got["judge"].add((r, origin, pid, aux, vote)); counts["judge"] += 1
            elif kind_ == LOG_ACTION:
                got["action"].add((r, origin, pid)); counts["action"] += 1
            elif kind_ == LOG_DELIVER and tag == TAG_DECISION:
                got["pickup"].add((r, origin, pid, vote)); counts["pickup"] += 1
            elif kind_ == LOG_RESULT:
                got["result"].add((r, pid, vote)); counts["result"] += 1
    for k in want:
        assert counts[k] == len(got[k]), (k, "duplicate records")
        assert got[k] == want[k], (k, len(got[k]), len(want[k]), sorted(got[k] ^ want[k])[:6])
    assert len(want["result"]) == n * p
    declined = sum(1 for (_, _, d) in want["result"] if d == 0)
    if 0 < ppm < 10000:
        assert 0 < declined < n * p and want["action"], declined  # both outcomes exercised
    return declined
