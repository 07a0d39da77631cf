"""Host-service worlds: the device engine driven through its command / pickup rings, the
path librootless_ops.so (the drop-in rootless_ops.h) takes -- here with every rank of the
world in this process, so parity tests can run the API's state machine at sizes MPI
processes on one box cannot (64 / 256 ranks).

    hw = HostWorld(n)                 # launches the persistent kernel (rlo_program_host)
    hw.bcast(rank, payload)           # RLO_bcast_gen (rootless_ops.c:1581)
    hw.propose(rank, pid, data)       # RLO_submit_proposal (:876): PBuf (pid, 1, len, data)
    for ev in hw.poll(rank): ...      # RLO_make_progress_all (:538): deliveries, judge requests,
                                      # actions, own results
    hw.judge(rank, ev, vote)          # verdict of judge(data) (:698) for an RLO_EV_JUDGE event
    hw.own_judge(rank, ev, vote)      # verdict of judge(NULL) (:773) for an RLO_EV_OWN_JUDGE event
    hw.close()                        # RLO_CMD_QUIT to every rank, wait for the kernel
"""
import ctypes
import struct

from . import _lib as L
from ._lib import check
from .world import World


def pbuf(pid, vote, data):
    """pbuf_serialize (rootless_ops.c:1369-1396): [pid i32][vote i32][data_len u64][data]"""
    return struct.pack("<iiQ", pid, vote, len(data)) + data


class HostWorld:
    def __init__(self, n, max_payload=256, device=-1, cmd_slots=0, pickup_slots=0, idle_timeout_s=60, pool=1,
                 pend_hbm=False, **world_kw):
        """pool: own proposals a rank may keep in flight (the proposal pool; 1 = my_own_proposal);
        pend_hbm: the pending-proposal tables in HBM (the 8-GPU layout, rehearsed); world_kw: World's other
        arguments (bulk_max, movers, ring_slots ... -- the drop-in's world shape)"""
        self.world = World(n, max_payload=max_payload, device=device, proposal_pool=max(2, 1 << (pool - 1).bit_length()),
                           pend_hbm=pend_hbm, **world_kw)
        self.lib = self.world.lib
        self.h = self.world.h
        self.n = n
        self.max_payload = self.world.info["slot_stride"] - 16
        cfg = L.HostCfg(cmd_slots, pickup_slots, idle_timeout_s, 0, pool, 0)
        check(self.lib.rlo_program_host(self.h, ctypes.byref(cfg)), "rlo_program_host")
        self.stream = ctypes.c_void_p()
        dev = device if device >= 0 else 0
        check(self.lib.rlo_stream_create(dev, ctypes.byref(self.stream)), "rlo_stream_create")
        check(self.lib.rlo_launch_ex(self.h, self.stream, 0), "rlo_launch_ex")
        self.backlog = [[] for _ in range(n)]
        self.pool = pool
        self.inflight = [0] * n    # own proposals posted whose result has not arrived
        self.held = [[] for _ in range(n)]  # proposals beyond the pool, posted as results free slots
        self._rec = L.LogRec()
        self._buf = ctypes.create_string_buffer(self.max_payload + 16)
        self.closed = False

    # ---------------------------------------------------------------- commands
    def _post(self, rank, cmd, payload=b""):
        q = self.backlog[rank]
        q.append((cmd, payload))
        while q:
            c, p = q[0]
            rc = self.lib.rlo_host_post(self.h, rank, ctypes.byref(c), p if p else None, len(p))
            if rc == L.RLO_E_AGAIN:
                return False
            check(rc, "rlo_host_post")
            q.pop(0)
        return True

    def flush(self):
        for r in range(self.n):
            if self.backlog[r]:
                c, p = self.backlog[r].pop(0)
                self._post(r, c, p)

    def bcast(self, rank, payload, seq=0):
        return self._post(rank, L.Cmd(L.RLO_CMD_BCAST, 0, seq, 0, 0, 0), bytes(payload))

    def propose(self, rank, pid, data):
        """RLO_submit_proposal; beyond `pool` in flight the proposal waits here (as librootless_ops.so
        does), not in the command ring, where it would hold up the judge verdicts behind it"""
        if self.inflight[rank] >= self.pool:
            self.held[rank].append((pid, bytes(data)))
            return True
        self.inflight[rank] += 1
        return self._post(rank, L.Cmd(L.RLO_CMD_PROPOSAL, 0, pid, 0, 1, 0), pbuf(pid, 1, bytes(data)))

    def judge(self, rank, ev, vote):
        return self._post(rank, L.Cmd(L.RLO_CMD_JUDGE, ev["origin"], ev["id"], ev["aux"], int(vote), 0))

    def own_judge(self, rank, ev, vote):
        """verdict of judge(NULL) for an RLO_EV_OWN_JUDGE event (its pid and pool slot)"""
        return self._post(rank, L.Cmd(L.RLO_CMD_OWN_JUDGE, 0, ev["id"], ev["aux"], int(vote), 0))

    # ---------------------------------------------------------------- events
    def poll(self, rank, limit=1 << 16):
        out = []
        r, buf = self._rec, self._buf
        for _ in range(limit):
            got = self.lib.rlo_host_poll(self.h, rank, ctypes.byref(r), buf, len(buf))
            if got != 1:
                check(got, "rlo_host_poll")
                break
            ev = {"kind": r.kind, "origin": r.origin, "from": r.from_, "id": r.id, "len": r.len, "vote": r.vote,
                  "aux": r.aux}
            if r.payload_idx != 0xFFFFFFFF:
                ev["payload"] = buf.raw[:min(r.len, len(buf))]
            out.append(ev)
            if r.kind == L.RLO_EV_RESULT:  # a pool slot is free again
                self.inflight[rank] -= 1
                if self.held[rank]:
                    self.propose(rank, *self.held[rank].pop(0))
        return out

    def running(self):
        return check(self.lib.rlo_host_running(self.h), "rlo_host_running") == 1

    def stats(self):
        """per-rank counters; complete only after close() (see final_stats)"""
        return self.world.stats()

    def relaunch(self):
        """QUIT every rank, wait for the kernel, and launch the same world again (rings, counters and
        command doorbells restart at 0: rlo_reset)"""
        for r in range(self.n):
            self.backlog[r].clear()
            q = L.Cmd(L.RLO_CMD_QUIT, 0, 0, 0, 0, 0)
            while self.lib.rlo_host_post(self.h, r, ctypes.byref(q), None, 0) == L.RLO_E_AGAIN:
                self.poll(r)
        self.world.wait()
        self.inflight = [0] * self.n
        self.held = [[] for _ in range(self.n)]
        check(self.lib.rlo_launch_ex(self.h, self.stream, 0), "rlo_launch_ex")

    def close(self, raise_on_device_error=True):
        if self.closed:
            return
        self.closed = True
        for r in range(self.n):
            self.backlog[r].clear()
            q = L.Cmd(L.RLO_CMD_QUIT, 0, 0, 0, 0, 0)
            while self.lib.rlo_host_post(self.h, r, ctypes.byref(q), None, 0) == L.RLO_E_AGAIN:
                self.poll(r)
        try:
            self.world.wait(raise_on_device_error=raise_on_device_error)
            self.final_stats = self.world.stats()  # per-rank counters are flushed when the kernel ends
        finally:
            self.lib.rlo_stream_destroy(self.stream)
            self.world.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close(raise_on_device_error=a[0] is None)
