// rootless_ops.cpp -- the drop-in rootless_ops.h API (librootless_ops.so) over the device
// engine's host-service program (rlo_hip.h).
//
// One engine = one rank of a device world whose parts are the ranks of the engine's
// communicator (one part per process).  RLO_progress_engine_new builds the part on this
// process' GPU, exchanges the ring mappings with MPI_Allgather and launches the rank's
// persistent progress kernel.  From then on the kernel forwards, merges votes and
// broadcasts decisions by itself; this library only
//   * posts originations (RLO_bcast_gen, RLO_submit_proposal) and judge verdicts into the
//     rank's command ring, and
//   * drains the rank's pickup ring in RLO_make_progress_all: deliveries become
//     RLO_user_msg pickups, judge / action callbacks run on this thread
//     (rootless_ops.c:698, :773, :842), own results update my_own_proposal.
// Everything here is the reference's host-visible state machine; nothing on the data path
// runs on the CPU.
#include "rootless_ops.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <cstring>
#include <pthread.h>
#include <sched.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <string>
#include <map>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <utility>
#include <vector>

#include "rlo_hip.h"
#include "rlo_trace.hpp"

int total_pickup = 0;  // rootless_ops.h:46

struct RLO_msg_generic {  // first member = the user view, so RLO_user_msg* and RLO_msg_t* convert
    RLO_user_msg msg_usr;
    int send_len;         // bytes given to RLO_msg_new_bc
    uint8_t* ext;         // a bulk message's bytes (longer than the data area), malloc'd; else null
    size_t ext_len;
    int source;           // tree parent (MPI_SOURCE in the reference), -1 for local messages
    uint64_t seq;         // command sequence number once posted
    int posted;           // 1: in the command ring (or backlog), 2: consumed by the device
    int pickup_done, fwd_done;
    size_t dirty;         // bytes of buf written since the last clear (pool reuse)
};

struct Proposal_state {  // rootless_ops.c:184-194
    RLO_ID pid;
    int recv_proposal_from;
    RLO_Vote vote;
    int votes_needed, votes_recved;
    RLO_Req_stat state;
    RLO_msg_t* proposal_msg;
    RLO_msg_t* decision_msg;
};

namespace {

struct Cmd {  // a command waiting for room in the command ring
    rlo_cmd_t c;
    std::vector<uint8_t> payload;
    RLO_msg_t* msg;
};

struct RawEv {  // a pickup-ring event pulled off the device, not yet handled on the app thread
    rlo_log_rec_t ev;
    std::vector<uint8_t> payload;
    int64_t t_seen = 0;  // RLO_TRACE_DIR: when the pump took it off the pickup ring
};

}  // namespace

struct progress_engine {
    MPI_Comm comm = MPI_COMM_NULL;
    MPI_Comm group = MPI_COMM_NULL;  // the ranks sharing my GPU (one part of the device world)
    int rank = 0, size = 0, id = 0, device = 0;
    bool leader = false;             // group rank 0: owns the part, its kernel and the proxy
    bool caller_bound = false;       // RLO_NUMA_BIND=all moved the creating thread: its mask to restore at cleanup
    cpu_set_t caller_mask;
    rlo_world_t* w = nullptr;        // leader only
    void* stream = nullptr;          // leader only
    rlo_client_t* cl = nullptr;      // every rank: its rank of the part, through the shared segment
    iar_cb_func_t judge = nullptr, action = nullptr;
    void* ctx = nullptr;
    uint32_t slot_bytes = 0;      // device payload capacity
    uint32_t deliver_max = 0;     // bytes a receiver sees (reference: msg_size_max - 4, :1588)
    uint64_t bulk_max = 0;        // extension: bcasts up to this many bytes (bulk messages), 0 = off
    int send_list_len = 0;
    std::deque<RLO_msg_t*> pickup;   // queue_pickup (:938)
    std::deque<Cmd> backlog;         // commands the ring had no room for yet
    std::deque<RLO_msg_t*> wait;     // my bcasts until the device took them (queue_wait, :1594)
    uint64_t bcast_seq = 0;
    RLO_proposal_state own{};        // my_own_proposal (:241): the most recently submitted one
    int pool_depth = 1;              // extension: own proposals in flight (RLO_PROPOSAL_POOL)
    std::map<int, RLO_proposal_state> props;  // pool_depth > 1: every own proposal by pid
    int own_inflight = 0;            // own proposals posted whose result has not arrived
    std::deque<std::pair<int, std::vector<char>>> held_props;  // submitted beyond the pool: (pid, PBuf)
    std::map<std::pair<int, int>, std::vector<char>> approved;  // (origin, pid) -> PBuf bytes (queue_iar_pending)
    // the zero-padded receive buffer a judge / action callback reads (the reference's calloc'd buffer): kept
    // zeroed between calls -- only the bytes written for a call are cleared after it -- so a judge request
    // costs no 32-KiB allocation on the proposal's path
    std::vector<char> cbuf;
    long sent_bcast = 0, recved_bcast = 0;  // :1600, :586
    bool failed = false;
    uint32_t poll_tick = 0;
    std::vector<uint8_t> evbuf;
    // the device side of the engine (command ring producer, pickup ring consumer, backlog, evq)
    // is shared with the pump thread, which keeps both rings moving while the application is
    // not calling progress (MPI's sends complete without it: testcases.c:690-697 relies on that)
    std::mutex mu;
    std::deque<RawEv> evq;
    std::atomic<int64_t> app_ns{0};  // last time the application thread made progress
    // RLO_TRACE=1: counters printed at cleanup (diagnostics)
    uint64_t n_progress = 0, n_events = 0, n_pumped = 0, n_judge = 0, n_result = 0;
    int64_t t_submit = 0, sum_prop_ns = 0, max_prop_ns = 0;
    // RLO_TRACE: my proposal's two legs, as seen here -- submit -> the kernel consumed the command
    // (the host -> device path), then -> my result event (the device rounds + device -> host path);
    // histogram buckets < 0.2, 0.5, 1, 2 ms and beyond
    uint64_t d_sub_idx = 0;
    int64_t d_cons_ns = 0, d_fwd_ns = 0;
    uint32_t d_hist[2][5] = {}, d_fh[2][5] = {};  // d_fh: submit -> forwarded by the proxy, forwarded -> consumed
    int64_t t_moved = 0, t_dump = 0;  // RLO_WATCHDOG: last event / last state dump
    rlo::TraceLog tr;                 // RLO_TRACE_DIR (the app and pump threads both append)
    uint64_t tr_consumed = 0;
    progress_engine* next = nullptr;
};

namespace {

progress_engine* g_engines = nullptr;  // Active_Engines (:40)
int g_engines_ever = 0;
int g_fault_attach_rank = -1;  // rlo_dropin_test_fault
std::vector<RLO_msg_t*> g_pool;         // recycled received messages

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

const char* trace_dir() {
    static const char* d = std::getenv("RLO_TRACE_DIR");
    return d && *d ? d : nullptr;
}

void trace(progress_engine* e, char what, uint32_t kind, int32_t origin, int32_t id, int32_t from, uint32_t aux,
           int64_t t = 0) {
    e->tr.add(rlo::TraceRec{t ? t : now_ns(), what, kind, origin, id, from, aux});
}

void trace_write(progress_engine* e) {
    char path[4096], hdr[128];
    std::snprintf(path, sizeof path, "%s/trace_rank%d_e%d.txt", trace_dir(), e->rank, e->id);
    std::snprintf(hdr, sizeof hdr, "# rank %d size %d engine %d\n", e->rank, e->size, e->id);
    (void)e->tr.write(path, hdr);
}

// RLO_TRACE_SETUP=1: engine construction steps with timestamps on stderr (diagnostics)
void setup_trace(int rank, const char* step) {
    static const bool on = std::getenv("RLO_TRACE_SETUP") != nullptr;
    if (on) std::fprintf(stderr, "rlo setup rank %d t=%.6f %s\n", rank, now_ns() * 1e-9, step);
}

void proposal_init(RLO_proposal_state* ps) {  // proposal_state_init :1235-1248
    ps->pid = -1;
    ps->recv_proposal_from = -1;
    ps->vote = 1;
    ps->votes_needed = -1;
    ps->votes_recved = 0;
    ps->state = RLO_INVALID;
    ps->proposal_msg = nullptr;
    ps->decision_msg = nullptr;
}

RLO_msg_t* msg_alloc(int origin) {
    RLO_msg_t* m;
    if (!g_pool.empty()) {
        m = g_pool.back();
        g_pool.pop_back();
        std::memset(m->msg_usr.buf, 0, m->dirty);  // the data area reads as calloc'd (:290)
    } else {
        m = (RLO_msg_t*)std::calloc(1, sizeof(RLO_msg_t));
        if (!m) return nullptr;
    }
    m->msg_usr.type = -1;  // RLO_msg_new_generic :292-294
    m->msg_usr.pid = -1;
    m->msg_usr.vote = -1;
    m->msg_usr.data_len = 0;
    m->msg_usr.data = m->msg_usr.buf + sizeof(int);
    std::memcpy(m->msg_usr.buf, &origin, sizeof(int));
    m->send_len = 0;
    m->ext = nullptr;
    m->ext_len = 0;
    m->source = -1;
    m->seq = 0;
    m->posted = 0;
    m->pickup_done = 0;
    m->fwd_done = 0;
    m->dirty = sizeof(int);
    return m;
}

void msg_release(RLO_msg_t* m) {
    if (!m) return;
    std::free(m->ext);
    m->ext = nullptr;
    m->ext_len = 0;
    if (g_pool.size() < 256) g_pool.push_back(m);
    else std::free(m);
}

// PBuf [pid i32][vote i32][data_len u64][data] (pbuf_serialize :1369-1396)
size_t pbuf_put(char* out, RLO_ID pid, RLO_Vote vote, uint64_t len, const void* data) {
    std::memcpy(out, &pid, 4);
    std::memcpy(out + 4, &vote, 4);
    std::memcpy(out + 8, &len, 8);
    if (len) std::memcpy(out + 16, data, len);
    return 16 + len;
}

int post(progress_engine* e, const rlo_cmd_t& c, const void* payload, uint32_t len, RLO_msg_t* msg) {
    std::lock_guard<std::mutex> lk(e->mu);
    if (trace_dir()) {  // with the command's index in this rank's command stream (the kernel's head passes it)
        uint64_t posted = 0;
        rlo_client_cmd_count(e->cl, nullptr, &posted);
        trace(e, 'P', c.kind, c.origin, c.id, (int32_t)(posted + e->backlog.size() + 1), c.pseq);
    }
    if (e->backlog.empty()) {
        int rc = rlo_client_post(e->cl, &c, payload, len);
        if (rc == RLO_OK) {
            if (msg) {
                uint64_t posted = 0;
                rlo_client_cmd_count(e->cl, nullptr, &posted);
                msg->seq = posted;  // consumed once the device head reaches it
                msg->posted = 1;
            }
            return 0;
        }
        if (rc != RLO_E_AGAIN) {
            std::fprintf(stderr, "rlo: rank %d: command post failed: %s\n", e->rank, rlo_strerror(rc));
            return -1;
        }
    }
    Cmd q;
    q.c = c;
    q.payload.assign((const uint8_t*)payload, (const uint8_t*)payload + len);
    q.msg = msg;
    if (msg) msg->posted = 1;
    e->backlog.push_back(std::move(q));
    return 0;
}

// RLO_CMD_PROPOSAL with the serialized PBuf (:876-906); counts it in flight until its result
int post_proposal(progress_engine* e, int pid, const std::vector<char>& pb) {
    rlo_cmd_t c;
    std::memset(&c, 0, sizeof c);
    c.kind = RLO_CMD_PROPOSAL;
    c.id = pid;
    c.vote = 1;
    if (post(e, c, pb.data(), (uint32_t)pb.size(), nullptr)) return -1;
    e->own_inflight++;
    return 0;
}

// [e->mu held]
void flush_backlog(progress_engine* e) {
    while (!e->backlog.empty()) {
        Cmd& q = e->backlog.front();
        int rc = rlo_client_post(e->cl, &q.c, q.payload.data(), (uint32_t)q.payload.size());
        if (rc == RLO_E_AGAIN) return;
        if (rc != RLO_OK) {
            std::fprintf(stderr, "rlo: rank %d: command post failed: %s\n", e->rank, rlo_strerror(rc));
            e->failed = true;
            return;
        }
        if (q.msg) {
            uint64_t posted = 0;
            rlo_client_cmd_count(e->cl, nullptr, &posted);
            q.msg->seq = posted;
        }
        e->backlog.pop_front();
    }
}

// frees my sent bcasts once the device has taken them (_wait_only_queue_cleanup :1015-1034)
// [e->mu held]
void reap_sent(progress_engine* e) {
    if (e->wait.empty()) return;
    uint64_t consumed = 0;
    rlo_client_cmd_count(e->cl, &consumed, nullptr);
    while (!e->wait.empty()) {
        RLO_msg_t* m = e->wait.front();
        if (m->seq == 0 || m->seq > consumed) break;
        e->wait.pop_front();
        m->posted = 2;
        m->fwd_done = 1;
        std::free(m->ext);
        std::free(m);
    }
}

int leg_bucket(int64_t ns) { return ns < 200000 ? 0 : ns < 500000 ? 1 : ns < 1000000 ? 2 : ns < 2000000 ? 3 : 4; }

void check_alive(progress_engine* e) {
    if (e->failed) return;
    const int st = rlo_client_state(e->cl);
    if (st == 1) return;
    std::fprintf(stderr, "rlo: rank %d engine %d: this rank's progress workgroup stopped serving (state %d%s)\n", e->rank,
                 e->id, st, st == RLO_E_DEVICE ? ": the GPU leader marked the engine failed" : "");
    e->failed = true;
}

void handle_event(progress_engine* e, const rlo_log_rec_t& ev, const uint8_t* payload) {
    switch (ev.kind) {
        case RLO_EV_DELIVER_BCAST: {  // :583-589 -> pickup
            RLO_msg_t* m = msg_alloc(ev.origin);
            if (!m) return;
            const uint32_t n = ev.len < e->deliver_max ? ev.len : e->deliver_max;
            std::memcpy(m->msg_usr.buf + sizeof(int), payload, n);
            m->dirty = sizeof(int) + n;
            m->msg_usr.type = RLO_BCAST;
            m->source = ev.from;
            m->fwd_done = 1;  // forwarded by the device before this event was written
            e->recved_bcast++;
            e->pickup.push_back(m);
            break;
        }
        case RLO_EV_DELIVER_BULK: {  // extension: a bcast beyond the data area, copied out of the heap
            RLO_msg_t* m = msg_alloc(ev.origin);
            if (!m) return;
            m->ext = (uint8_t*)std::malloc(ev.len ? ev.len : 1);
            if (!m->ext || rlo_client_bulk_get(e->cl, &ev, m->ext) != RLO_OK) {
                std::fprintf(stderr, "rlo: rank %d: bulk delivery of %u bytes from %d failed\n", e->rank, ev.len, ev.origin);
                e->failed = true;
                msg_release(m);
                return;
            }
            rlo_cmd_t c;  // the heap slot can take the origin's next bulk message
            std::memset(&c, 0, sizeof c);
            c.kind = RLO_CMD_BULK_RELEASE;
            c.origin = ev.origin;
            c.pseq = ev.aux;
            post(e, c, nullptr, 0, nullptr);
            m->ext_len = ev.len;
            m->msg_usr.type = RLO_BCAST;
            m->msg_usr.data = (char*)m->ext;
            m->msg_usr.data_len = ev.len;  // extension: the size (reference bcasts leave 0, :920-932)
            m->source = ev.from;
            m->fwd_done = 1;
            e->recved_bcast++;
            e->pickup.push_back(m);
            break;
        }
        case RLO_EV_DELIVER_DECISION: {  // _iar_decision_handler :814-859 + _user_msg_mock :920-932
            e->approved.erase(std::make_pair(ev.origin, (int)ev.id));  // declined: proposal dropped (:833-837)
            RLO_msg_t* m = msg_alloc(ev.origin);
            if (!m) return;
            char* d = m->msg_usr.buf + sizeof(int);
            m->dirty = sizeof(int) + pbuf_put(d, (RLO_ID)ev.id, ev.vote, 7, "IAR_DEC");
            m->msg_usr.type = RLO_IAR_DECISION;
            m->msg_usr.pid = (RLO_ID)ev.id;
            m->msg_usr.vote = ev.vote;
            m->msg_usr.data_len = 7;
            m->msg_usr.data = d + 16;
            m->source = ev.from;
            m->fwd_done = 1;
            e->recved_bcast++;
            e->pickup.push_back(m);
            break;
        }
        case RLO_EV_ACTION: {  // decision 1 for a proposal I approved: action(PBuf) (:842)
            auto it = e->approved.find(std::make_pair(ev.origin, (int)ev.id));
            if (it != e->approved.end()) {
                const size_t n = it->second.size();
                std::memcpy(e->cbuf.data(), it->second.data(), n);
                if (e->action) e->action(e->cbuf.data(), e->ctx);
                std::memset(e->cbuf.data(), 0, n);
                e->approved.erase(it);
            }
            break;
        }
        case RLO_EV_RESULT: {  // my decision went out (:560-563 + _iar_decision_bcast :908-917)
            if (e->own_inflight > 0) e->own_inflight--;
            if (!e->held_props.empty() && e->own_inflight < e->pool_depth) {  // its pool slot is free again
                auto hp = std::move(e->held_props.front());
                e->held_props.pop_front();
                if (post_proposal(e, hp.first, hp.second)) e->failed = true;
            }
            if (e->pool_depth > 1) {
                auto it = e->props.find((int)ev.id);
                if (it != e->props.end()) {
                    it->second.vote = ev.vote;
                    it->second.votes_recved = it->second.votes_needed;
                    it->second.state = RLO_COMPLETED;
                }
                e->n_result++;
                e->sent_bcast++;  // a decision counts as a sent bcast (:1600)
                if ((int)ev.id != e->own.pid) break;  // own mirrors the most recent submission
                e->own.vote = ev.vote;
                e->own.votes_recved = e->own.votes_needed;
                e->own.state = RLO_COMPLETED;
                break;
            }
            if (e->d_cons_ns) {
                e->d_hist[1][leg_bucket(now_ns() - e->d_cons_ns)]++;
                e->d_cons_ns = 0;
            }
            e->d_sub_idx = 0;
            if (e->t_submit) {
                const int64_t d = now_ns() - e->t_submit;
                e->sum_prop_ns += d;
                e->max_prop_ns = std::max(e->max_prop_ns, d);
            }
            e->n_result++;
            e->sent_bcast++;  // a decision counts as a sent bcast (:1600)
            // only the result of the proposal my_own_proposal holds: a second submission while the first
            // is in flight overwrote it (:878-883), and the reference counts votes only for that pid (:756)
            if ((int)ev.id != e->own.pid) break;
            e->own.vote = ev.vote;
            e->own.votes_recved = e->own.votes_needed;
            e->own.state = RLO_COMPLETED;
            break;
        }
        case RLO_EV_JUDGE: {  // judge(proposal data, ctx) (:698); data is zero-padded like the
            e->n_judge++;
                              // reference's calloc'd receive buffer
            const uint32_t n = ev.len < (uint32_t)RLO_MSG_SIZE_MAX ? ev.len : (uint32_t)RLO_MSG_SIZE_MAX;
            std::memcpy(e->cbuf.data(), payload, n);
            int v = e->judge ? e->judge(e->cbuf.data() + 16, e->ctx) : 1;
            std::memset(e->cbuf.data(), 0, n);
            if (v != 0 && v != 1) {
                std::printf("%s:%u - rank = %03d: unknown judgment received: %d\n", __func__, __LINE__, e->rank, v);
                v = 0;
            }
            if (v == 1) e->approved[std::make_pair(ev.origin, (int)ev.id)].assign((const char*)payload, (const char*)payload + n);
            rlo_cmd_t c;
            std::memset(&c, 0, sizeof c);
            c.kind = RLO_CMD_JUDGE;
            c.origin = ev.origin;
            c.id = (int32_t)ev.id;
            c.pseq = ev.aux;
            c.vote = v;
            post(e, c, nullptr, 0, nullptr);
            break;
        }
        case RLO_EV_JUDGED: {  // extension: the device judged a proposal here; keep the PBuf for action()
            e->n_judge++;
            if (ev.vote == 1) {
                const uint32_t n = ev.len < (uint32_t)RLO_MSG_SIZE_MAX ? ev.len : (uint32_t)RLO_MSG_SIZE_MAX;
                e->approved[std::make_pair(ev.origin, (int)ev.id)].assign((const char*)payload, (const char*)payload + n);
            }
            break;
        }
        case RLO_EV_OWN_JUDGE: {  // every vote was 1: vote = judge(my_proposal = NULL, ctx) (:770-775)
            int v = e->judge ? e->judge(nullptr, e->ctx) : 1;
            if (v != 0 && v != 1) v = 0;
            rlo_cmd_t c;
            std::memset(&c, 0, sizeof c);
            c.kind = RLO_CMD_OWN_JUDGE;
            c.id = (int32_t)ev.id;
            c.pseq = ev.aux;  // the proposal's pool slot
            c.vote = v;
            post(e, c, nullptr, 0, nullptr);
            break;
        }
        default:
            std::fprintf(stderr, "rlo: rank %d: unexpected event kind %u\n", e->rank, ev.kind);
            break;
    }
}

// [e->mu held] commands into the command ring, events off the pickup ring into evq
bool pump(progress_engine* e) {
    const size_t backlog0 = e->backlog.size();
    flush_backlog(e);
    rlo_log_rec_t ev;
    int got = 0;
    for (; got < 4096; got++) {
        int r = rlo_client_poll(e->cl, &ev, e->evbuf.data(), (uint32_t)e->evbuf.size());
        if (r != 1) break;
        RawEv q;
        q.ev = ev;
        if (trace_dir()) q.t_seen = now_ns();
        if (ev.payload_idx != 0xffffffffu) {
            const uint32_t n = ev.len < (uint32_t)e->evbuf.size() ? ev.len : (uint32_t)e->evbuf.size();
            q.payload.assign(e->evbuf.data(), e->evbuf.data() + n);
        }
        e->evq.push_back(std::move(q));
    }
    if (got) flush_backlog(e);
    if (trace_dir()) {
        uint64_t consumed = 0;
        rlo_client_cmd_count(e->cl, &consumed, nullptr);
        if (consumed != e->tr_consumed) trace(e, 'C', 0, -1, (int32_t)consumed, -1, 0);
        e->tr_consumed = consumed;
    }
    return got || e->backlog.size() != backlog0;
}

// RLO_WATCHDOG=seconds (diagnostics): an engine whose application keeps calling progress but
// sees no event for that long prints its host- and ring-side state once per period
void watchdog(progress_engine* e, bool moved, int64_t period_ns) {
    const int64_t t = now_ns();
    if (moved || e->t_moved == 0) { e->t_moved = t; return; }
    if (t - e->t_moved < period_ns || t - e->t_dump < period_ns) return;
    e->t_dump = t;
    std::lock_guard<std::mutex> lk(e->mu);  // backlog / evq are shared with the pump thread
    uint64_t consumed = 0, posted = 0;
    rlo_client_cmd_count(e->cl, &consumed, &posted);
    uint64_t d[9] = {0};
    rlo_client_debug(e->cl, d);
    std::fprintf(stderr, "rlo watchdog rank %d engine %d: commands posted %llu forwarded %llu consumed %llu (kernel saw "
                 "tail %llu); pickups consumed %llu written %llu (kernel saw head %llu); kernel beat %llu state %llu\n",
                 e->rank, e->id, (unsigned long long)d[0], (unsigned long long)d[1], (unsigned long long)d[2],
                 (unsigned long long)d[3], (unsigned long long)d[4], (unsigned long long)d[5], (unsigned long long)d[6],
                 (unsigned long long)d[7], (unsigned long long)d[8]);
    std::fprintf(stderr, "rlo watchdog rank %d engine %d: %.1f s without events; sent %ld recved %ld pickup %zu "
                 "backlog %zu wait %zu evq %zu commands consumed %llu / posted %llu, kernel running %d, "
                 "progress calls %llu events %llu\n", e->rank, e->id, (t - e->t_moved) * 1e-9, e->sent_bcast,
                 e->recved_bcast, e->pickup.size(), e->backlog.size(), e->wait.size(), e->evq.size(),
                 (unsigned long long)consumed, (unsigned long long)posted, rlo_client_state(e->cl),
                 (unsigned long long)e->n_progress, (unsigned long long)e->n_events);
}

// make_progress_gen (:551-641): everything the device finished since the last call
void progress(progress_engine* e) {
    if (!e->cl || e->failed) return;
    e->app_ns.store(now_ns(), std::memory_order_relaxed);
    // like make_progress_gen, which completes at most one receive per call (its single posted
    // ANY_SOURCE irecv, :569-624), a call surfaces at most one received message (a delivery or a
    // proposal to judge); applications pace on that (testcases.c:666-686 stops sending exactly
    // when its count is reached only because each progress call yields one pickup)
    std::deque<RawEv> local;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        pump(e);
        if (e->d_sub_idx && !e->d_cons_ns) {  // RLO_TRACE: has the kernel taken my proposal yet?
            if (!e->d_fwd_ns) {  // has the leader's proxy forwarded it?
                uint64_t f = 0;
                int64_t fns = 0;
                rlo_client_fwd(e->cl, &f, &fns);
                if (f >= e->d_sub_idx) {
                    e->d_fwd_ns = fns;
                    e->d_fh[0][leg_bucket(fns - e->t_submit)]++;
                }
            }
            uint64_t consumed = 0;
            rlo_client_cmd_count(e->cl, &consumed, nullptr);
            if (consumed >= e->d_sub_idx) {
                e->d_cons_ns = now_ns();
                e->d_hist[0][leg_bucket(e->d_cons_ns - e->t_submit)]++;
                if (e->d_fwd_ns) e->d_fh[1][leg_bucket(e->d_cons_ns - e->d_fwd_ns)]++;
            }
        }
        while (!e->evq.empty()) {
            const uint32_t k = e->evq.front().ev.kind;
            local.push_back(std::move(e->evq.front()));
            e->evq.pop_front();
            if (k == RLO_EV_DELIVER_BCAST || k == RLO_EV_DELIVER_BULK || k == RLO_EV_DELIVER_DECISION || k == RLO_EV_JUDGE)
                break;
        }
        reap_sent(e);
    }
    e->n_progress++;
    e->n_events += local.size();
    for (const RawEv& q : local) {
        if (trace_dir()) {
            trace(e, 'S', q.ev.kind, q.ev.origin, (int32_t)q.ev.id, q.ev.from, q.ev.aux, q.t_seen);
            trace(e, 'H', q.ev.kind, q.ev.origin, (int32_t)q.ev.id, q.ev.from, q.ev.aux);
        }
        handle_event(e, q.ev, q.payload.data());
    }
    if (local.empty() && (++e->poll_tick & 255u) == 0) check_alive(e);
    static const double wd = std::getenv("RLO_WATCHDOG") ? std::atof(std::getenv("RLO_WATCHDOG")) : 0.0;
    if (wd > 0) watchdog(e, !local.empty(), (int64_t)(wd * 1e9));
}

// ---- the pump thread: one per process while engines exist; it only moves ring entries
std::mutex g_list_mu;  // guards g_engines against the pump thread
std::thread g_pump;
std::atomic<bool> g_pump_stop{false};

// The pump steps in only for engines whose application thread has not made progress for a
// while: a busy application moves its own rings, and the pump would only compete for its core.
void pump_loop() {
    constexpr int64_t kQuiet = 200000;  // ns without an application progress call
    unsigned idle = 0;
    while (!g_pump_stop.load(std::memory_order_relaxed)) {
        bool did = false;
        {
            std::lock_guard<std::mutex> lg(g_list_mu);
            const int64_t t = now_ns();
            for (progress_engine* e = g_engines; e; e = e->next) {
                if (t - e->app_ns.load(std::memory_order_relaxed) < kQuiet) continue;
                std::unique_lock<std::mutex> lk(e->mu, std::try_to_lock);
                if (!lk.owns_lock() || e->failed || !e->cl) continue;  // the app thread is on it
                if (pump(e)) { did = true; e->n_pumped++; }
            }
        }
        if (did) idle = 0;
        else if (++idle > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
        else std::this_thread::yield();
    }
}

// The engine's own threads onto the NUMA node of their part's GPU.  The shared segment's per-rank lines are written
// by the rank's CPU and read by the GPU and the proxy, so a thread on the far socket pays remote-socket latency on
// every command and pickup: 8 ranks unpinned ran the storm at 0.27-0.47 M bcast/s and the host-judge decisions at
// 34.6-40.8 K/s from run to run, on the GPU's node 0.48-0.50 M and 41.3 K, on the other node 0.30 M and 34.6 K
// (profiles/r4_dropin_numa_ab.txt).  RLO_NUMA_BIND:
//   unset / 1  the pump and proxy threads this library starts, and nothing else: the application's threads keep
//              the affinity the launcher gave them (the reference library changes no affinity at all);
//   all        the calling application thread too, for the engine's lifetime (its mask is restored at cleanup);
//   0          no thread.
// A process the launcher already placed within one node (mpiexec -bind-to ..., taskset) is left alone, as is an
// unknown node or one with none of the process's CPUs.
static std::vector<int> node_cpus(int node) {
    std::vector<int> out;
    char path[96];
    std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE* f = std::fopen(path, "r");
    if (!f) return out;
    char buf[4096] = {0};
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    for (char* tok = std::strtok(buf, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {
        int a = 0, b = 0;
        if (std::sscanf(tok, "%d-%d", &a, &b) == 2) {
            for (int c = a; c <= b; c++) out.push_back(c);
        } else if (std::sscanf(tok, "%d", &a) == 1) {
            out.push_back(a);
        }
    }
    return out;
}
enum NumaMode { kNumaOff = 0, kNumaEngine = 1, kNumaAll = 2 };
static NumaMode numa_mode() {
    const char* v = std::getenv("RLO_NUMA_BIND");
    if (!v || !*v || std::strcmp(v, "1") == 0) return kNumaEngine;
    if (std::strcmp(v, "all") == 0) return kNumaAll;
    return kNumaOff;
}
// the CPUs of `node` within `cur`, or false when `cur` already lies within one node (the launcher placed the
// process), the node is unknown or holds none of `cur`'s CPUs
static bool numa_mask(int node, const cpu_set_t& cur, cpu_set_t* want) {
    if (node < 0) return false;
    int touched = 0;
    for (int nd = 0; nd < 64 && touched < 2; nd++) {
        bool any = false;
        for (int c : node_cpus(nd))
            if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &cur)) { any = true; break; }
        touched += any ? 1 : 0;
    }
    if (touched < 2) return false;
    CPU_ZERO(want);
    int k = 0;
    for (int c : node_cpus(node))
        if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &cur)) { CPU_SET(c, want); k++; }
    return k > 0;
}
int g_numa_node = -1;        // the NUMA node of the latest engine's GPU (engine threads follow it)
cpu_set_t g_proc_mask;       // the process's affinity before this library changed any thread's
bool g_proc_mask_ok = false;
static void bind_engine_thread(std::thread& t) {
    if (!t.joinable() || !g_proc_mask_ok || numa_mode() == kNumaOff) return;
    cpu_set_t want;
    if (numa_mask(g_numa_node, g_proc_mask, &want)) (void)pthread_setaffinity_np(t.native_handle(), sizeof want, &want);
}

void pump_start() {
    if (g_pump.joinable() || std::getenv("RLO_NO_PUMP")) return;
    g_pump_stop = false;
    g_pump = std::thread(pump_loop);
    bind_engine_thread(g_pump);
}

void pump_stop() {
    if (!g_pump.joinable()) return;
    g_pump_stop = true;
    g_pump.join();
}

// ---- the proxy thread: one per leader process while it serves parts.  It moves the clients'
// commands into the parts' VRAM command rings and their pickup heads into the counters the
// kernels poll, and runs their bulk copies (rlo_host_proxy); it spins, since every command of every
// rank on this GPU passes through it
// (the thread works on its own copy of the list, refreshed when the generation moves, so it never
// holds a lock the application threads wait for)
std::mutex g_served_mu;
std::vector<rlo_world_t*> g_served;  // [g_served_mu]
std::atomic<uint64_t> g_served_gen{0}, g_proxy_seen{0};
std::thread g_proxy;
std::atomic<bool> g_proxy_stop{false};

void proxy_loop() {
    unsigned idle = 0;
    uint64_t seen = ~0ull;
    std::vector<rlo_world_t*> mine;
    // RLO_PROXY_DIAG: the largest gap between two passes (a descheduled proxy stalls every rank)
    static const bool diag = std::getenv("RLO_PROXY_DIAG") != nullptr;
    int64_t t_prev = diag ? now_ns() : 0, gap_max = 0, gaps_1ms = 0, passes = 0;
    while (!g_proxy_stop.load(std::memory_order_relaxed)) {
        if (diag) {
            const int64_t tn = now_ns();
            gap_max = std::max(gap_max, tn - t_prev);
            gaps_1ms += tn - t_prev > 1000000;
            t_prev = tn;
            passes++;
        }
        const uint64_t gen = g_served_gen.load(std::memory_order_acquire);
        if (gen != seen) {
            {
                std::lock_guard<std::mutex> lg(g_served_mu);
                mine = g_served;
            }
            seen = gen;
            g_proxy_seen.store(gen, std::memory_order_release);
        }
        int acted = 0;
        for (rlo_world_t* w : mine) {
            const int a = rlo_host_proxy(w);
            if (a > 0) acted += a;
        }
        if (acted) idle = 0;
        else if (++idle > (1u << 20)) std::this_thread::sleep_for(std::chrono::microseconds(20));  // long idle only
        else __builtin_ia32_pause();
    }
    if (diag)
        std::fprintf(stderr, "proxy diag: passes %lld, max gap %.1f us, gaps > 1 ms %lld\n", (long long)passes,
                     gap_max * 1e-3, (long long)gaps_1ms);
}

void served_add(rlo_world_t* w) {
    {
        std::lock_guard<std::mutex> lg(g_served_mu);
        g_served.push_back(w);
    }
    g_served_gen.fetch_add(1, std::memory_order_acq_rel);
}

// after this returns the proxy no longer touches w
void served_remove(rlo_world_t* w) {
    {
        std::lock_guard<std::mutex> lg(g_served_mu);
        g_served.erase(std::remove(g_served.begin(), g_served.end(), w), g_served.end());
    }
    const uint64_t g = g_served_gen.fetch_add(1, std::memory_order_acq_rel) + 1;
    while (g_proxy.joinable() && g_proxy_seen.load(std::memory_order_acquire) < g) std::this_thread::yield();
}

void proxy_start() {
    if (g_proxy.joinable()) return;
    g_proxy_stop = false;
    g_proxy = std::thread(proxy_loop);
    bind_engine_thread(g_proxy);
}

void proxy_stop() {
    if (!g_proxy.joinable()) return;
    g_proxy_stop = true;
    g_proxy.join();
}

std::vector<std::pair<rlo_world_t*, void*>> g_grave;  // stopped engines' worlds / streams

void bury() {
    for (auto& g : g_grave) {
        rlo_world_destroy(g.first);
        rlo_stream_destroy(g.second);
    }
    g_grave.clear();
}

// The reference never frees the engine's dup'd communicator (:1461, :1524-1527) and its tests
// use it after RLO_progress_engine_cleanup.  Keep it alive until MPI_Finalize, which deletes
// MPI_COMM_SELF's attributes first (MPI standard, "Allowing User Functions at Process
// Termination") -- there the retired communicators are freed.
std::vector<MPI_Comm> g_retired;
int g_retire_key = MPI_KEYVAL_INVALID;

int free_retired(MPI_Comm, int, void*, void*) {
    bury();
    for (MPI_Comm& c : g_retired) MPI_Comm_free(&c);
    g_retired.clear();
    return MPI_SUCCESS;
}

void retire_comm(MPI_Comm c) {
    if (g_retire_key == MPI_KEYVAL_INVALID) {
        MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, free_retired, &g_retire_key, nullptr);
        MPI_Comm_set_attr(MPI_COMM_SELF, g_retire_key, nullptr);
    }
    g_retired.push_back(c);
}

}  // namespace

extern "C" {

RLO_user_msg* RLO_user_msg_new(RLO_msg_t* gen_msg_in) { return gen_msg_in ? &gen_msg_in->msg_usr : nullptr; }

RLO_msg_t* RLO_msg_new_generic(RLO_engine_t* eng) {
    assert(eng);
    RLO_msg_t* m = (RLO_msg_t*)std::calloc(1, sizeof(RLO_msg_t));
    if (!m) return nullptr;
    m->msg_usr.type = -1;
    m->msg_usr.pid = -1;
    m->msg_usr.vote = -1;
    m->msg_usr.data = m->msg_usr.buf + sizeof(int);
    std::memcpy(m->msg_usr.buf, &eng->rank, sizeof(int));
    m->source = -1;
    m->dirty = sizeof(m->msg_usr.buf);
    return m;
}

RLO_msg_t* RLO_msg_new_bc(RLO_engine_t* eng, void* buf_in, int send_size) {
    RLO_msg_t* m = RLO_msg_new_generic(eng);
    if (!m) return nullptr;
    if (send_size < 0) send_size = 0;
    if ((uint64_t)send_size > eng->deliver_max && eng->bulk_max) {
        // extension: longer than the data area -> a bulk bcast (RLO_bcast_gen moves it through the heap)
        if ((uint64_t)send_size > eng->bulk_max) {
            std::fprintf(stderr, "rlo: RLO_msg_new_bc: %d bytes exceed RLO_BULK_MAX (%llu)\n", send_size,
                         (unsigned long long)eng->bulk_max);
            std::free(m);
            return nullptr;
        }
        m->ext = (uint8_t*)std::malloc((size_t)send_size);
        if (!m->ext) { std::free(m); return nullptr; }
        std::memcpy(m->ext, buf_in, (size_t)send_size);
        m->ext_len = (size_t)send_size;
        m->send_len = send_size;
        return m;
    }
    if (send_size > RLO_MSG_SIZE_MAX) send_size = RLO_MSG_SIZE_MAX;  // the data area (:295)
    if (send_size) std::memcpy(m->msg_usr.buf + sizeof(int), buf_in, (size_t)send_size);
    m->send_len = send_size;
    return m;
}

int RLO_msg_free(RLO_msg_t* msg_in) {
    if (msg_in) std::free(msg_in->ext);
    std::free(msg_in);
    return 0;
}

int RLO_msg_test_isends(RLO_engine_t* eng, RLO_msg_t* msg_in) {
    assert(eng && msg_in);
    if (msg_in->posted == 2) return 1;
    if (msg_in->posted == 0) return 1;  // never sent: nothing pending
    std::lock_guard<std::mutex> lk(eng->mu);
    uint64_t consumed = 0;
    rlo_client_cmd_count(eng->cl, &consumed, nullptr);
    return msg_in->seq != 0 && consumed >= msg_in->seq;
}

}  // extern "C"

namespace {

RLO_engine_t* engine_new(MPI_Comm mpi_comm, size_t msg_size_max, void* approv_cb_func, void* app_ctx,
                         void* app_proposal_action, const RLO_device_judge* dj) {
    progress_engine* e = new progress_engine();
    MPI_Comm_dup(mpi_comm, &e->comm);  // bcomm_init :1461
    MPI_Comm_rank(e->comm, &e->rank);
    MPI_Comm_size(e->comm, &e->size);
    e->judge = (iar_cb_func_t)approv_cb_func;
    e->action = (iar_cb_func_t)app_proposal_action;
    e->ctx = app_ctx;
    if (e->size < 2) {  // bcomm_init returns NULL for N < 2 (:1464-1467)
        std::fprintf(stderr, "rlo: a rootless engine needs at least 2 ranks\n");
        MPI_Comm_free(&e->comm);
        delete e;
        return nullptr;
    }
    size_t cap = msg_size_max ? msg_size_max : RLO_MSG_SIZE_MAX;
    if (cap > RLO_MSG_SIZE_MAX) cap = RLO_MSG_SIZE_MAX;
    if (cap < 64) cap = 64;
    e->slot_bytes = (uint32_t)((cap + 15) & ~(size_t)15);
    e->deliver_max = (uint32_t)cap - (uint32_t)sizeof(int);  // bytes [0, msg_size_max - 4) arrive (:1588)
    e->evbuf.assign(e->slot_bytes + 16, 0);
    e->cbuf.assign(RLO_MSG_SIZE_MAX + 16, 0);
    int level = 0, lw = 0, scc = 0, sl[16];
    rlo_topology(e->size, e->rank, &level, &lw, &scc, &e->send_list_len, sl);
    proposal_init(&e->own);

    // One part per GPU.  The ranks are dealt to the GPUs in contiguous blocks; the first rank of
    // each block (the leader) owns the part -- all of the block's ranks -- with its persistent
    // kernel, and is the only process on that GPU that touches HIP.  Every rank (the leader's own
    // too) drives its rank through the shared host segment (rlo_client_*), which the leader's proxy
    // thread serves.  So exactly one process per GPU holds hardware queues, however many ranks
    // share it (DESIGN.md "one queue-holding process per GPU").
    int node_size = 0;
    {
        MPI_Comm node;
        MPI_Comm_split_type(e->comm, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node);
        MPI_Comm_size(node, &node_size);
        MPI_Comm_free(&node);
    }
    int ndev = 0;
    if (e->rank == 0 && node_size == e->size) ndev = rlo_device_count();  // rank 0 leads a GPU anyway
    MPI_Bcast(&ndev, 1, MPI_INT, 0, e->comm);
    if (node_size != e->size || ndev <= 0) {
        if (e->rank == 0)
            std::fprintf(stderr, "rlo: %s\n", ndev <= 0 ? "no HIP device" : "the communicator must stay inside one node (hipIpc mappings)");
        MPI_Comm_free(&e->comm);
        delete e;
        return nullptr;
    }
    auto dev_of = [&](int r) {
        if (const char* sd = std::getenv("RLO_DEVICE")) return std::atoi(sd) % ndev;
        return e->size <= ndev ? r : (int)((int64_t)r * ndev / e->size);
    };
    // RLO_PARTS=k: deal the ranks into k contiguous parts (k leaders, k persistent kernels, ring
    // mappings exchanged between the leaders) even where they share a GPU -- the multi-part engine an
    // 8-GPU node runs, exercised on one GPU.  Every rank must see the same k (the largest is taken)
    int kparts = 0;
    {
        int mine = 0;
        if (const char* sp = std::getenv("RLO_PARTS")) mine = std::max(0, std::atoi(sp));
        MPI_Allreduce(&mine, &kparts, 1, MPI_INT, MPI_MAX, e->comm);
        kparts = std::min(kparts, e->size);
    }
    std::vector<int> part_begin;  // contiguous blocks of ranks: one per GPU, or RLO_PARTS of them
    if (kparts > 0) {
        for (int p = 0; p < kparts; p++) part_begin.push_back((int)((int64_t)e->size * p / kparts));
    } else {
        for (int r = 0; r < e->size; r++)
            if (r == 0 || dev_of(r) != dev_of(r - 1)) part_begin.push_back(r);
    }
    const int n_parts = (int)part_begin.size();
    part_begin.push_back(e->size);
    int part = 0;
    while (part_begin[part + 1] <= e->rank) part++;
    e->device = dev_of(part_begin[part]);  // a part's ranks share its leader's GPU
    e->leader = e->rank == part_begin[part];
    MPI_Comm_split(e->comm, part, e->rank, &e->group);
    {  // the engine's threads onto its GPU's NUMA node (the leader asks HIP; group rank 0 is the leader)
        int numa = e->leader ? rlo_device_numa_node(e->device) : -1;
        MPI_Bcast(&numa, 1, MPI_INT, 0, e->group);
        if (!g_proc_mask_ok) {
            CPU_ZERO(&g_proc_mask);
            g_proc_mask_ok = sched_getaffinity(0, sizeof g_proc_mask, &g_proc_mask) == 0;
        }
        g_numa_node = numa;
        bind_engine_thread(g_pump);  // already running for an earlier engine
        bind_engine_thread(g_proxy);
        cpu_set_t want, cur;
        if (numa_mode() == kNumaAll && pthread_getaffinity_np(pthread_self(), sizeof cur, &cur) == 0 &&
            numa_mask(numa, cur, &want) && pthread_setaffinity_np(pthread_self(), sizeof want, &want) == 0) {
            e->caller_mask = cur;  // restored at cleanup
            e->caller_bound = true;
        }
    }
    MPI_Comm leaders;
    MPI_Comm_split(e->comm, e->leader ? 0 : MPI_UNDEFINED, e->rank, &leaders);
    // extension: device judges -- the kinds must agree; ISP strings go to the part's leader
    int djk = dj ? dj->kind : -1, djmin = 0, djmax = 0;
    MPI_Allreduce(&djk, &djmin, 1, MPI_INT, MPI_MIN, e->comm);
    MPI_Allreduce(&djk, &djmax, 1, MPI_INT, MPI_MAX, e->comm);
    std::vector<std::string> isp_local;
    if (djmin != djmax || (dj && dj->kind != RLO_DJUDGE_APPROVE && dj->kind != RLO_DJUDGE_ISP &&
                           dj->kind != RLO_DJUDGE_HASH)) {  // the same on every rank: all leave here
        if (e->rank == 0) std::fprintf(stderr, "rlo: RLO_progress_engine_new_dj: every rank must pass the same known judge kind\n");
        if (leaders != MPI_COMM_NULL) MPI_Comm_free(&leaders);
        MPI_Comm_free(&e->group);
        MPI_Comm_free(&e->comm);
        delete e;
        return nullptr;
    }
    {
        const std::string mine = dj && dj->kind == RLO_DJUDGE_ISP && dj->isp ? std::string(dj->isp) : std::string();
        int gsz = 0, grank = 0;
        MPI_Comm_size(e->group, &gsz);
        MPI_Comm_rank(e->group, &grank);
        int len = (int)mine.size() + 1;
        std::vector<int> lens(gsz, 0), offs(gsz, 0);
        MPI_Gather(&len, 1, MPI_INT, lens.data(), 1, MPI_INT, 0, e->group);
        int tot = 0;
        for (int i = 0; i < gsz; i++) { offs[i] = tot; tot += lens[i]; }
        std::vector<char> buf(e->leader ? (size_t)std::max(tot, 1) : 1, 0);
        MPI_Gatherv(mine.c_str(), len, MPI_CHAR, buf.data(), lens.data(), offs.data(), MPI_CHAR, 0, e->group);
        if (e->leader)
            for (int i = 0; i < gsz; i++) isp_local.emplace_back(buf.data() + offs[i]);
    }
    std::vector<int> devs(n_parts);
    for (int p = 0; p < n_parts; p++) devs[p] = dev_of(part_begin[p]);
    bool multi = false;
    for (int d : devs) multi |= d != devs[0];

    {  // extension: the proposal pool depth, the largest any rank asks for (RLO_PROPOSAL_POOL)
        int mine = 1, depth = 1;
        if (const char* pp = std::getenv("RLO_PROPOSAL_POOL")) mine = std::max(1, std::min(16, std::atoi(pp)));
        MPI_Allreduce(&mine, &depth, 1, MPI_INT, MPI_MAX, e->comm);
        e->pool_depth = depth;
    }
    // extension, opt-in: bcasts beyond the data area up to RLO_BULK_MAX bytes.  Off by default, as the reference
    // caps a bcast at its data area (:295): a world without bulk messages runs the host-service kernel without the
    // bulk code and its mover workgroups -- the drop-in's 8-rank p50 20.0 vs 21.9 us with it
    // (profiles/r5_dropin_legs_bulk_ab.txt)
    e->bulk_max = 0;
    if (const char* bm = std::getenv("RLO_BULK_MAX")) e->bulk_max = std::strtoull(bm, nullptr, 10);
    int rc = RLO_OK;
    char shm_name[96] = {0};
    auto agree = [&](int ok_local) {  // every rank of the engine learns whether every step worked
        int g = 0;
        MPI_Allreduce(&ok_local, &g, 1, MPI_INT, MPI_MIN, e->comm);
        return g != 0;
    };
    bool ok = true, launched = false;
    if (e->leader) {
        rlo_part_cfg_t pc;
        std::memset(&pc, 0, sizeof pc);
        pc.n_ranks = e->size;
        pc.n_parts = n_parts;
        pc.part = part;
        pc.part_begin = part_begin.data();
        pc.max_payload = e->slot_bytes;
        // 512 slots for small slots (the library default is 2048 there, tuned for device storms; the
        // drop-in's few ranks per GPU gain nothing from it: profiles/r1s5_api_slots.jsonl); RLO_RING_SLOTS
        // overrides it for diagnostics
        pc.ring_slots = e->slot_bytes > 4096 ? 128u : 512u;
        if (const char* rs = std::getenv("RLO_RING_SLOTS")) pc.ring_slots = (uint32_t)std::strtoul(rs, nullptr, 10);
        pc.device = e->device;
        pc.flags = multi ? RLO_PART_UNCACHED : 0u;
        pc.bulk_max = e->bulk_max;
        pc.bulk_slots = 2;
        pc.proposal_pool = 2;  // pending entries per origin: a power of two >= the pool depth
        while (pc.proposal_pool < (uint32_t)e->pool_depth) pc.proposal_pool *= 2;
        pc.movers = 4;  // RLO_BULK_MOVERS: mover workgroups of the part
        if (const char* mv = std::getenv("RLO_BULK_MOVERS")) pc.movers = (uint32_t)std::strtoul(mv, nullptr, 10);
        rc = rlo_part_create(&pc, &e->w);
    }
    setup_trace(e->rank, "part created");
    std::vector<uint8_t> blob(RLO_PART_BLOB_BYTES, 0), blobs((size_t)RLO_PART_BLOB_BYTES * n_parts, 0);
    if (e->leader && rc == RLO_OK && rlo_part_export(e->w, blob.data(), RLO_PART_BLOB_BYTES) < 0) rc = RLO_E_HIP;
    ok = agree(rc == RLO_OK);
    if (ok && e->leader) {
        MPI_Allgather(blob.data(), RLO_PART_BLOB_BYTES, MPI_BYTE, blobs.data(), RLO_PART_BLOB_BYTES, MPI_BYTE, leaders);
        // the mappings in n_parts stages (rlo_hip.h rlo_part_import): in stage k part k exports its handles afresh
        // and every other leader imports them while part k imports nothing -- a handle exported before its exporter
        // imported anything (later imports by the exporter were seen to make an earlier handle map another region)
        for (int k = 0; k < n_parts && n_parts > 1; k++) {
            std::vector<uint8_t> bk(RLO_PART_BLOB_BYTES, 0);
            if (k == part && rlo_part_export(e->w, bk.data(), RLO_PART_BLOB_BYTES) < 0 && rc == RLO_OK) rc = RLO_E_HIP;
            MPI_Bcast(bk.data(), RLO_PART_BLOB_BYTES, MPI_BYTE, k, leaders);
            if (k != part && rc == RLO_OK) rc = rlo_part_import(e->w, bk.data(), k);
            MPI_Barrier(leaders);
        }
        if (rc == RLO_OK) rc = rlo_part_connect(e->w, blobs.data(), n_parts);
        setup_trace(e->rank, "connected");
        if (rc == RLO_OK) {
            std::snprintf(shm_name, sizeof shm_name, "/rlo.%d.%d.%d", (int)getpid(), g_engines_ever + 1, part);
            rc = rlo_host_share(e->w, shm_name, 4ull << 20);
        }
        if (rc == RLO_OK) {
            rlo_host_cfg_t hc;
            std::memset(&hc, 0, sizeof hc);
            hc.pickup_slots = 512;
            hc.pool = (uint32_t)e->pool_depth;
            rc = rlo_program_host(e->w, &hc);
        }
        if (rc == RLO_OK && dj) {  // extension: the device judges (every local rank's string for ISP)
            rlo_iar_cfg_t jc;
            std::memset(&jc, 0, sizeof jc);
            jc.judge_kind = (uint32_t)dj->kind;
            jc.judge_ppm = dj->ppm;
            jc.judge_seed = dj->seed;
            std::string all;
            for (int r = 0; r < e->size; r++) {
                const int lrk = r - part_begin[part];
                if (lrk >= 0 && lrk < (int)isp_local.size()) all += isp_local[lrk];
                all.push_back('\0');
            }
            jc.judge_isp = all.data();
            rc = rlo_host_device_judge(e->w, &jc);
        }
        setup_trace(e->rank, "programmed (shared segment)");
        if (rc == RLO_OK) rc = rlo_stream_create(e->device, &e->stream);
        if (rc == RLO_OK) rc = rlo_reset(e->w, e->stream);
    }
    setup_trace(e->rank, "connected+programmed+shared+reset");
    ok = ok && agree(rc == RLO_OK);  // every part reset before any part launches
    if (ok && e->leader) {
        rc = rlo_launch_ex(e->w, e->stream, RLO_LAUNCH_NO_RESET);
        launched = rc == RLO_OK;
        setup_trace(e->rank, "launch returned");
        // the kernel is resident and serving: a launch queued behind other work on a shared hardware
        // queue would otherwise look like a running engine that never answers
        if (rc == RLO_OK) rc = rlo_host_wait_started(e->w, 20000);
        if (rc != RLO_OK)
            std::fprintf(stderr, "rlo: rank %d: the progress kernel on GPU %d did not start serving (%s)\n", e->rank,
                         e->device, rlo_strerror(rc));
    }
    ok = ok && agree(rc == RLO_OK);
    setup_trace(e->rank, "launched+started");
    if (ok) {  // members map their ranks through the leader's segment
        MPI_Bcast(shm_name, (int)sizeof shm_name, MPI_CHAR, 0, e->group);
        // fault injection, armed only by a test calling rlo_dropin_test_fault (no environment switch in the
        // product library): rank r's attach fails after every kernel was launched -- the path on which the
        // leaders must stop their serving kernels cleanly
        if (g_fault_attach_rank >= 0 && g_fault_attach_rank == e->rank) shm_name[1] = '!';
        rc = rlo_client_attach(shm_name, e->rank, &e->cl);
        ok = agree(rc == RLO_OK);
        if (e->leader) rlo_host_unlink(e->w);  // every client attached (or gave up): drop the name
    }
    setup_trace(e->rank, "attached");
    if (ok && e->leader) {  // the proxy serves this part from now on
        served_add(e->w);
        proxy_start();
    }
    if (!ok) {
        std::fprintf(stderr, "rlo: rank %d: engine setup failed (%s, hip %d)\n", e->rank, rlo_strerror(rc),
                     rlo_last_hip_error());
        if (e->w && e->leader) {
            rlo_host_fail(e->w);
            if (launched && rlo_host_running(e->w) == 1) {  // stop every local rank of the kernel
                rlo_cmd_t q;
                std::memset(&q, 0, sizeof q);
                q.kind = RLO_CMD_QUIT;
                for (int r = part_begin[part]; r < part_begin[part + 1]; r++) rlo_host_post(e->w, r, &q, nullptr, 0);
                rlo_wait(e->w);
            }
        }
        MPI_Barrier(e->comm);
        if (e->cl) rlo_client_detach(e->cl);
        if (e->w) rlo_world_destroy(e->w);
        if (e->stream) rlo_stream_destroy(e->stream);
        if (leaders != MPI_COMM_NULL) MPI_Comm_free(&leaders);
        MPI_Comm_free(&e->group);
        MPI_Comm_free(&e->comm);
        delete e;
        return nullptr;
    }
    if (leaders != MPI_COMM_NULL) MPI_Comm_free(&leaders);
    e->id = ++g_engines_ever;  // engine ids 1, 2, ... (:515-517)
    {
        std::lock_guard<std::mutex> lg(g_list_mu);
        progress_engine** tail = &g_engines;
        while (*tail) tail = &(*tail)->next;
        *tail = e;
    }
    pump_start();
    return e;
}

}  // namespace

extern "C" {

// test hook (tests/test_gpu_dropin.py::test_engine_setup_failure_is_clean through oracle/ref_harness.c):
// what 1 = the next engine setup's attach of `rank` fails; rank -1 disarms.  Not in the reference API
int rlo_dropin_test_fault(int what, int rank) {
    if (what != 1) return -1;
    g_fault_attach_rank = rank;
    return 0;
}

RLO_engine_t* RLO_progress_engine_new(MPI_Comm mpi_comm, size_t msg_size_max, void* approv_cb_func, void* app_ctx,
                                      void* app_proposal_action) {
    return engine_new(mpi_comm, msg_size_max, approv_cb_func, app_ctx, app_proposal_action, nullptr);
}

RLO_engine_t* RLO_progress_engine_new_dj(MPI_Comm mpi_comm, size_t msg_size_max, const RLO_device_judge* judge,
                                         void* app_ctx, void* app_proposal_action) {
    if (!judge) return nullptr;
    return engine_new(mpi_comm, msg_size_max, nullptr, app_ctx, app_proposal_action, judge);
}

int RLO_progress_engine_cleanup(RLO_engine_t* eng) {
    assert(eng);
    if (std::getenv("RLO_TRACE"))
        std::fprintf(stderr, "rlo trace rank %d engine %d: progress %llu events %llu pumped %llu judge %llu results %llu "
                     "proposal->result avg %.1f us max %.1f us\n", eng->rank, eng->id, (unsigned long long)eng->n_progress,
                     (unsigned long long)eng->n_events, (unsigned long long)eng->n_pumped, (unsigned long long)eng->n_judge,
                     (unsigned long long)eng->n_result, eng->n_result ? eng->sum_prop_ns / 1e3 / eng->n_result : 0.0,
                     eng->max_prop_ns / 1e3);
    if (std::getenv("RLO_TRACE"))
        std::fprintf(stderr, "rlo trace rank %d legs (<0.2/0.5/1/2/>2 ms): submit->consumed %u %u %u %u %u | consumed->result %u %u %u %u %u\n",
                     eng->rank, eng->d_hist[0][0], eng->d_hist[0][1], eng->d_hist[0][2], eng->d_hist[0][3], eng->d_hist[0][4],
                     eng->d_hist[1][0], eng->d_hist[1][1], eng->d_hist[1][2], eng->d_hist[1][3], eng->d_hist[1][4]);
    if (std::getenv("RLO_TRACE"))
        std::fprintf(stderr, "rlo trace rank %d split: submit->forwarded %u %u %u %u %u | forwarded->consumed %u %u %u %u %u\n",
                     eng->rank, eng->d_fh[0][0], eng->d_fh[0][1], eng->d_fh[0][2], eng->d_fh[0][3], eng->d_fh[0][4],
                     eng->d_fh[1][0], eng->d_fh[1][1], eng->d_fh[1][2], eng->d_fh[1][3], eng->d_fh[1][4]);
    if (trace_dir()) trace_write(eng);
    // collective quiescence (:1607-1627): every bcast and decision sent anywhere has arrived here
    int sent = (int)eng->sent_bcast, total = 0, done = 0;
    MPI_Request req;
    MPI_Iallreduce(&sent, &total, 1, MPI_INT, MPI_SUM, eng->comm, &req);
    do {
        MPI_Test(&req, &done, MPI_STATUS_IGNORE);
        if (!done) RLO_make_progress_all();
    } while (!done);
    while (!eng->failed && eng->recved_bcast + eng->sent_bcast < total) RLO_make_progress_all();
    RLO_user_msg* u = nullptr;
    while (RLO_user_pickup_next(eng, &u)) {  // :1628-1631
        total_pickup++;
        RLO_user_msg_recycle(eng, u);
    }
    // every rank quiescent -> stop the kernels -> nobody stores into anyone's rings any more
    MPI_Ibarrier(eng->comm, &req);
    done = 0;
    do {
        MPI_Test(&req, &done, MPI_STATUS_IGNORE);
        if (!done) RLO_make_progress_all();
    } while (!done);
    rlo_cmd_t q;
    std::memset(&q, 0, sizeof q);
    q.kind = RLO_CMD_QUIT;
    post(eng, q, nullptr, 0, nullptr);
    while (!eng->failed && rlo_client_state(eng->cl) == 1) {  // keep both rings moving until my rank stops
        std::lock_guard<std::mutex> lk(eng->mu);
        pump(eng);
        eng->evq.clear();
    }
    if (std::getenv("RLO_HOST_DIAG") && !eng->failed) {
        uint64_t d[8] = {};
        rlo_client_hdiag(eng->cl, d);
        std::fprintf(stderr, "rlo hdiag rank %d: pending iters %llu held %llu pk-blocked %llu host iters %llu | seen->drained "
                     "<20us %llu <100us %llu <500us %llu >=500us %llu\n", eng->rank, (unsigned long long)d[0],
                     (unsigned long long)d[1], (unsigned long long)d[2], (unsigned long long)d[3], (unsigned long long)d[4],
                     (unsigned long long)d[5], (unsigned long long)d[6], (unsigned long long)d[7]);
    }
    MPI_Barrier(eng->group);  // every rank of my GPU's part stopped: the kernel ends
    if (eng->leader) {
        served_remove(eng->w);
        int rc = rlo_wait(eng->w);
        if (rc != RLO_OK && !eng->failed)
            std::fprintf(stderr, "rlo: rank %d engine %d: kernel ended with %s\n", eng->rank, eng->id, rlo_strerror(rc));
        if (std::getenv("RLO_HOP_PROF")) {  // diagnostics build: the part's doorbell-pass profile (tools/hop_prof.py)
            rlo_world_info_t wi;
            if (rlo_world_query(eng->w, &wi) == RLO_OK) {
                const int nl = wi.rank_end - wi.rank_begin;
                std::vector<rlo_rank_stats_t> st((size_t)nl);
                if (rlo_stats(eng->w, st.data(), nl) == RLO_OK) {
                    uint64_t pr[8] = {}, db[8] = {}, it = 0, busy = 0;
                    for (const auto& x : st) {
                        for (int k = 0; k < 8; k++) { pr[k] += x.prof[k]; db[k] += x.dbg[k]; }
                        it += x.iterations;
                        busy += x.busy_iterations;
                    }
                    std::fprintf(stderr, "rlo hopprof part %d: hops %llu, cycles per hop", wi.part, (unsigned long long)db[0]);
                    for (int k = 0; k < 8; k++) std::fprintf(stderr, " %.0f", db[0] ? (double)pr[k] / db[0] : 0.0);
                    std::fprintf(stderr, " | passes %llu, to full: busy %llu cmd %llu lone %llu | held %llu pk-room %llu | "
                                 "iterations %llu busy %llu\n", (unsigned long long)db[4], (unsigned long long)db[1],
                                 (unsigned long long)db[2], (unsigned long long)db[3], (unsigned long long)db[6],
                                 (unsigned long long)db[7], (unsigned long long)it, (unsigned long long)busy);
                }
            }
        }
    }
    MPI_Barrier(eng->comm);
    for (RLO_msg_t* m : eng->pickup) msg_release(m);
    for (RLO_msg_t* m : eng->wait) std::free(m);
    retire_comm(eng->comm);  // callers keep using RLO_get_my_comm's comm after cleanup (testcases.c:329-331)
    {
        std::lock_guard<std::mutex> lg(g_list_mu);
        progress_engine** p = &g_engines;  // engine_remove (:445-466)
        while (*p && *p != eng) p = &(*p)->next;
        if (*p) *p = eng->next;
    }
    if (!g_engines) pump_stop();
    bool none_served;
    {
        std::lock_guard<std::mutex> lg(g_served_mu);
        none_served = g_served.empty();
    }
    if (none_served) proxy_stop();
    rlo_client_detach(eng->cl);
    eng->cl = nullptr;
    // hipFree / hipIpcCloseMemHandle may wait for the whole device, i.e. for the persistent
    // kernel of another engine of this process: free the world once no engine kernel runs
    if (eng->leader) g_grave.push_back(std::make_pair(eng->w, eng->stream));
    if (!g_engines) {
        bury();
        // the process's last engine: the device memory only this process ever mapped goes back to HIP, and its idle
        // imports of peers' regions close (regions it exported stay pooled: RLO_device_memory_release)
        (void)rlo_pool_trim(RLO_TRIM_IMPORTS | RLO_TRIM_FREE, nullptr);
    }
    MPI_Comm_free(&eng->group);
    if (eng->caller_bound) (void)pthread_setaffinity_np(pthread_self(), sizeof eng->caller_mask, &eng->caller_mask);
    delete eng;
    return 0;
}

int RLO_make_progress_all(void) {
    if (!g_engines) return -1;  // :540-543
    for (progress_engine* e = g_engines; e; e = e->next) progress(e);
    return 0;
}

int RLO_get_engine_id(RLO_engine_t* eng) {
    assert(eng);
    return eng->id;
}

MPI_Comm RLO_get_my_comm(RLO_engine_t* eng) {
    assert(eng);
    return eng->comm;
}

int RLO_bcast_gen(RLO_engine_t* eng, RLO_msg_t* msg_in, enum RLO_COMM_TAGS tag) {
    assert(eng && msg_in);
    if (tag != RLO_BCAST) {  // proposals / decisions are originated by the engine itself
        std::fprintf(stderr, "rlo: RLO_bcast_gen: only RLO_BCAST is originated by callers (tag %d)\n", (int)tag);
        return -1;
    }
    const uint32_t n = (uint32_t)msg_in->send_len < eng->deliver_max ? (uint32_t)msg_in->send_len : eng->deliver_max;
    msg_in->pickup_done = 1;  // :1584
    rlo_cmd_t c;
    std::memset(&c, 0, sizeof c);
    c.kind = RLO_CMD_BCAST;
    c.id = (int32_t)++eng->bcast_seq;
    if (msg_in->ext) {  // extension: a bulk bcast -- its bytes into my heap slot once the slot is free
        uint32_t q = 0;
        int rc;
        // my heap slot is free once every receiver released its previous message; they do so while they
        // make progress, which they may be waiting on me for (a bounded wait, then the engine fails)
        const int64_t t0 = now_ns();
        while ((rc = rlo_client_bulk_put(eng->cl, msg_in->ext, msg_in->ext_len, 0, &q)) == RLO_E_AGAIN) {
            RLO_make_progress_all();
            if (eng->failed) return -1;
            if (now_ns() - t0 > 60ll * 1000000000ll) { rc = RLO_E_TIMEOUT; break; }
        }
        if (rc != RLO_OK) {
            std::fprintf(stderr, "rlo: rank %d: bulk bcast of %zu bytes failed: %s\n", eng->rank, msg_in->ext_len,
                         rlo_strerror(rc));
            if (rc != RLO_E_INVAL) eng->failed = true;  // the service itself failed (a bad argument leaves it usable)
            return -1;
        }
        const uint32_t desc[4] = {(uint32_t)msg_in->ext_len, q, 0u, 0u};
        c.kind = RLO_CMD_BULK;
        if (post(eng, c, desc, sizeof desc, msg_in)) return -1;
        eng->wait.push_back(msg_in);
        eng->sent_bcast++;
        RLO_make_progress_all();  // :1602
        return 0;
    }
    if (post(eng, c, msg_in->msg_usr.buf + sizeof(int), n, msg_in)) return -1;
    eng->wait.push_back(msg_in);
    eng->sent_bcast++;
    RLO_make_progress_all();  // :1602
    return 0;
}

int RLO_user_pickup_next(RLO_engine_t* eng, RLO_user_msg** msg_out) {
    assert(eng);
    if (eng->pickup.empty()) return 0;
    RLO_msg_t* m = eng->pickup.front();
    eng->pickup.pop_front();
    *msg_out = &m->msg_usr;
    return 1;
}

int RLO_user_msg_recycle(RLO_engine_t* eng, RLO_user_msg* msg_in) {
    assert(eng && msg_in);
    RLO_msg_t* m = (RLO_msg_t*)msg_in;
    m->pickup_done = 1;
    if (m->fwd_done) {  // always: the device forwarded before the pickup event existed
        msg_release(m);
        return 1;
    }
    return 0;
}

int RLO_submit_proposal(RLO_engine_t* eng, char* proposal, size_t prop_size, RLO_ID my_proposal_id) {
    assert(eng);
    eng->own.pid = my_proposal_id;  // :878-883
    eng->own.proposal_msg = nullptr;
    eng->own.vote = 1;
    eng->own.votes_needed = eng->send_list_len;
    eng->own.votes_recved = 0;
    eng->own.decision_msg = nullptr;
    if (prop_size == 0 && proposal != nullptr) {  // pbuf_serialize rejects it (:1372-1375)
        std::printf("pbuf_serialize failed.\n");
        return -1;
    }
    if (16 + prop_size > eng->deliver_max) {
        std::fprintf(stderr, "rlo: proposal of %zu bytes exceeds the engine's message size\n", prop_size);
        return -1;
    }
    std::vector<char> pb(16 + prop_size);
    pbuf_put(pb.data(), my_proposal_id, 1, prop_size, proposal);
    eng->t_submit = now_ns();
    eng->own.state = RLO_IN_PROGRESS;
    if (eng->pool_depth > 1) eng->props[my_proposal_id] = eng->own;  // application thread only
    // a proposal beyond the pool waits HERE, not in the command ring: there it would hold up the
    // judge verdicts behind it, which other ranks' proposals -- and so my own -- wait for
    if (eng->own_inflight >= eng->pool_depth) {
        eng->held_props.emplace_back(my_proposal_id, std::move(pb));
        return -1;
    }
    if (post_proposal(eng, my_proposal_id, pb)) return -1;
    static const bool trace = std::getenv("RLO_TRACE") != nullptr;
    if (trace) {
        std::lock_guard<std::mutex> lk(eng->mu);
        if (eng->backlog.empty()) rlo_client_cmd_count(eng->cl, nullptr, &eng->d_sub_idx);
        eng->d_cons_ns = 0;
        eng->d_fwd_ns = 0;
    }
    RLO_make_progress_all();
    return eng->own.state == RLO_COMPLETED ? eng->own.vote : -1;
}

int RLO_check_proposal_state(RLO_engine_t* eng, int pid) {
    RLO_make_progress_all();
    if (eng->pool_depth > 1) {  // extension: the proposal pool reports the pid asked for
        auto it = eng->props.find(pid);
        if (it != eng->props.end()) return it->second.state;
    }
    return eng->own.state;  // pid ignored (or unknown), as in the reference (:869-872)
}

int RLO_proposal_pool_depth(RLO_engine_t* eng) { return eng ? eng->pool_depth : 0; }

int RLO_get_vote_proposal(RLO_engine_t* eng, RLO_ID pid) {
    assert(eng);
    if (eng->pool_depth <= 1) return eng->own.pid == pid ? RLO_get_vote_my_proposal(eng) : -1;
    auto it = eng->props.find(pid);
    if (it == eng->props.end() || it->second.state != RLO_COMPLETED) return -1;
    const int ret = it->second.vote;
    eng->props.erase(it);
    if (eng->own.pid == pid) RLO_proposal_reset(&eng->own);
    return ret;
}

int RLO_get_vote_my_proposal(RLO_engine_t* eng) {
    if (eng->own.state != RLO_COMPLETED) return -1;
    int ret = eng->own.vote;
    if (eng->pool_depth > 1) eng->props.erase(eng->own.pid);
    RLO_proposal_reset(&eng->own);
    return ret;
}

int RLO_proposal_reset(RLO_proposal_state* ps) {  // :1649-1664
    assert(ps);
    if (ps->decision_msg) RLO_msg_free(ps->decision_msg);
    ps->decision_msg = nullptr;
    if (ps->proposal_msg) RLO_msg_free(ps->proposal_msg);
    ps->proposal_msg = nullptr;
    ps->pid = -1;
    ps->recv_proposal_from = -1;
    ps->state = RLO_INVALID;
    ps->vote = -1;
    ps->votes_needed = 0;
    ps->votes_recved = 0;
    return 0;
}

unsigned long RLO_get_time_usec(void) {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return 1000000ul * (unsigned long)tv.tv_sec + (unsigned long)tv.tv_usec;
}

void RLO_get_time_str(char* str_out) {
    time_t raw;
    time(&raw);
    struct tm* t = localtime(&raw);
    std::sprintf(str_out, "%d:%d:%d", t->tm_hour, t->tm_min, t->tm_sec);
}

int RLO_get_my_rank(void) {  // MPI_COMM_WORLD, as in the reference (:148-152)
    int r = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &r);
    return r;
}

int RLO_get_world_size(void) {
    int n = -1;
    MPI_Comm_size(MPI_COMM_WORLD, &n);
    return n;
}

int RLO_user_msg_source(const RLO_user_msg* msg) { return msg ? ((const RLO_msg_t*)msg)->source : -1; }

int RLO_engine_device(RLO_engine_t* eng) { return eng ? eng->device : -1; }

int RLO_device_memory_release(MPI_Comm comm) {
    // the world-wide close (rlo_hip.h rlo_pool_trim): every process drops its idle imports before any frees a region a
    // peer may have imported
    int live = g_engines ? 1 : 0, any = 0;
    MPI_Allreduce(&live, &any, 1, MPI_INT, MPI_MAX, comm);
    if (any) return -1;
    bury();
    (void)rlo_pool_trim(RLO_TRIM_IMPORTS | RLO_TRIM_FREE | RLO_TRIM_EXPORTED, nullptr);
    MPI_Barrier(comm);
    (void)rlo_pool_trim(RLO_TRIM_RETIRED, nullptr);
    MPI_Barrier(comm);
    return 0;
}

}  // extern "C"
