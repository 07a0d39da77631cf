// rlo_world.cpp -- host side of the engine: overlay topology, HBM layout of the
// mailbox rings, programs (storm / latency / iar), launch and result readout.
// Exposes the C ABI of include/rlo_hip.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rlo_device.hpp"
#include "rlo_hip.h"

extern "C" hipError_t rlo_launch_progress(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream);
extern "C" size_t rlo_kernel_static_lds(void);
extern "C" hipError_t rlo_occupancy(int* blocks, size_t dyn_lds);

static_assert(sizeof(rlo_rank_stats_t) == sizeof(rlo::RankStats), "stats ABI");
static_assert(sizeof(rlo_log_rec_t) == sizeof(rlo::LogRec), "log ABI");

namespace {

thread_local int g_last_hip = 0;

#define HIPCHK(x)                                  \
    do {                                           \
        hipError_t e_ = (x);                       \
        if (e_ != hipSuccess) {                    \
            g_last_hip = (int)e_;                  \
            return RLO_E_HIP;                      \
        }                                          \
    } while (0)

// ------------------------------------------------------------------ topology
// Integer restatement of bcomm_init (rootless_ops.c:1454-1522), get_level (:1427-1441),
// last_wall (:1444-1452); pow()/log2() become shifts.
struct Topo {
    int level, last_wall, scc, sll;
    int send_list[rlo::kMaxFanout];
};

bool is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }
int floor_log2(int n) {
    int l = 0;
    while ((n >> (l + 1)) != 0) l++;
    return l;
}

int topo_of(int n, int rank, Topo* t) {
    if (n < 2 || rank < 0 || rank >= n) return RLO_E_INVAL;
    if (rank == 0) t->level = is_pow2(n) ? floor_log2(n) - 1 : floor_log2(n);
    else t->level = __builtin_ctz((unsigned)rank);
    t->last_wall = rank == 0 ? (1 << t->level) : (rank & (rank - 1));
    t->scc = t->level;
    t->sll = t->scc + 1;
    if (t->sll > rlo::kMaxFanout) return RLO_E_INVAL;
    for (int i = 0; i < t->sll; i++) {
        int dest = rank + (1 << i);
        if (is_pow2(n)) {
            t->send_list[i] = dest % n;
        } else if (dest >= n) {
            if (rank == n - 1) { t->scc = 0; t->send_list[0] = 0; }
            else { t->scc = i; t->send_list[i] = 0; }
            t->sll = t->scc + 1;
            break;
        } else {
            t->send_list[i] = dest;
        }
    }
    return RLO_OK;
}

bool passed(int me, int origin, int to) {  // rootless_ops.c:1534-1556
    if (to == origin) return true;
    if (me >= origin) return !(to > me || (to >= 0 && to < origin));
    return !(to > me && to < origin);
}

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint32_t pow2_ceil(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}
uint32_t pow2_floor(uint64_t x) {
    uint32_t p = 1;
    while ((uint64_t)p * 2 <= x && p < (1u << 30)) p <<= 1;
    return p;
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    int alloc(size_t count) {
        release();
        if (count == 0) count = 1;
        if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) { p = nullptr; return RLO_E_HIP; }
        n = count;
        return RLO_OK;
    }
    int upload(const std::vector<T>& v) {
        int rc = alloc(v.size());
        if (rc) return rc;
        if (!v.empty() && hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return RLO_E_HIP;
        return RLO_OK;
    }
};

}  // namespace

struct rlo_world {
    int n = 0, device = 0;
    uint32_t max_payload = 0, stride = 0, fwd_cap = 0, vote_cap = 0;
    int edges = 0, max_in = 0, max_fan = 0;
    int cus = 0, blocks_per_cu = 0;
    std::vector<rlo::RankTopo> topo;
    uint8_t* fwd = nullptr;
    uint8_t* vote = nullptr;
    uint64_t* ctrl = nullptr;
    uint64_t fwd_bytes = 0, vote_bytes = 0, ctrl_words = 0;
    DevBuf<rlo::RankTopo> d_topo;
    DevBuf<rlo::RankStats> d_stats;
    DevBuf<uint32_t> d_err;
    // program
    uint32_t mode = 0;
    bool have_program = false;
    rlo::Params P{};
    DevBuf<int64_t> d_sched_off, d_expect_bcast, d_prop_off, d_expect_dec;
    DevBuf<uint32_t> d_sched_ids, d_prop_data_off, d_prop_data_len, d_isp_off, d_lat_count, d_lat_round;
    DevBuf<int32_t> d_lat_origin, d_prop_pid;
    DevBuf<uint64_t> d_lat_out;
    DevBuf<uint8_t> d_mask, d_prop_data, d_log_payload;
    DevBuf<char> d_isp;
    DevBuf<rlo::LogRec> d_log;
    uint32_t lat_rounds = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipStream_t last_stream = nullptr;
    float last_ms = 0.f;
    size_t dyn_lds = 0;
    uint32_t nsmall = 8, stage2 = 1024;
};

// ====================================================================== C ABI

extern "C" {

int rlo_last_hip_error(void) { return g_last_hip; }

const char* rlo_strerror(int code) {
    switch (code) {
        case RLO_OK: return "ok";
        case RLO_E_INVAL: return "invalid argument";
        case RLO_E_HIP: return "HIP runtime error";
        case RLO_E_OCCUPANCY: return "ranks cannot all be co-resident";
        case RLO_E_DEVICE: return "device-side engine error";
        case RLO_E_NOPROGRAM: return "no program loaded";
        case RLO_E_NODEVICE: return "no HIP device";
        default: return "unknown";
    }
}

int rlo_topology(int n, int rank, int* level, int* last_wall, int* scc, int* sll, int* send_list) {
    Topo t;
    int rc = topo_of(n, rank, &t);
    if (rc) return rc;
    if (level) *level = t.level;
    if (last_wall) *last_wall = t.last_wall;
    if (scc) *scc = t.scc;
    if (sll) *sll = t.sll;
    if (send_list) std::memcpy(send_list, t.send_list, sizeof(int) * t.sll);
    return RLO_OK;
}

int rlo_children(int n, int rank, int origin, int from, int* out) {
    Topo t;
    int rc = topo_of(n, rank, &t);
    if (rc) return rc;
    int c = 0;
    if (from < 0) {
        for (int i = t.sll - 1; i >= 0; i--) out[c++] = t.send_list[i];
    } else if (t.level > 0) {
        if (from > t.last_wall) {
            for (int j = t.scc; j >= 0; j--) out[c++] = t.send_list[j];
        } else {
            for (int j = t.scc - 1; j >= 0; j--)
                if (!passed(rank, origin, t.send_list[j])) out[c++] = t.send_list[j];
        }
    }
    return c;
}

int rlo_world_create(const rlo_world_cfg_t* cfg, rlo_world_t** out) {
    if (!cfg || !out || cfg->n_ranks < 2 || cfg->n_ranks > 4096) return RLO_E_INVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return RLO_E_NODEVICE;
    rlo_world* w = new rlo_world();
    const int n = cfg->n_ranks;
    w->n = n;
    if (cfg->device >= 0) {
        if (hipSetDevice(cfg->device) != hipSuccess) { delete w; return RLO_E_HIP; }
    }
    (void)hipGetDevice(&w->device);
    w->max_payload = (std::max<uint32_t>(cfg->max_payload ? cfg->max_payload : 4096u, 16u) + 15u) & ~15u;
    w->stride = rlo::kHdr + w->max_payload;

    // ---- overlay: nodes, directed edges, in-edge lists
    std::vector<Topo> T(n);
    for (int r = 0; r < n; r++)
        if (topo_of(n, r, &T[r])) { delete w; return RLO_E_INVAL; }
    struct Edge { int src, dst, j, k; };
    std::vector<Edge> E;
    std::vector<std::vector<int>> in_edges(n);
    std::vector<std::vector<int>> out_edge(n);
    for (int r = 0; r < n; r++) {
        out_edge[r].resize(T[r].sll);
        for (int j = 0; j < T[r].sll; j++) {
            int e = (int)E.size();
            E.push_back({r, T[r].send_list[j], j, 0});
            out_edge[r][j] = e;
            in_edges[T[r].send_list[j]].push_back(e);
        }
    }
    for (int c = 0; c < n; c++) {
        if ((int)in_edges[c].size() > rlo::kMaxIn) { delete w; return RLO_E_INVAL; }
        w->max_in = std::max(w->max_in, (int)in_edges[c].size());
        for (int k = 0; k < (int)in_edges[c].size(); k++) E[in_edges[c][k]].k = k;
    }
    for (int r = 0; r < n; r++) w->max_fan = std::max(w->max_fan, T[r].sll);
    w->edges = (int)E.size();

    // ---- ring sizing: the whole forward region must fit one 32-bit buffer resource
    const uint64_t nrings = 2ull * E.size();
    uint32_t cap = cfg->ring_slots ? pow2_ceil(cfg->ring_slots) : 512u;
    const uint64_t limit = 0xFFFF0000ull;
    if (nrings * cap * w->stride > limit) cap = pow2_floor(limit / (nrings * w->stride));
    if (cap < 16) { delete w; return RLO_E_INVAL; }
    w->fwd_cap = cap;
    w->vote_cap = std::max<uint32_t>(64u, pow2_ceil(2u * (uint32_t)n));
    w->fwd_bytes = nrings * cap * w->stride;
    w->vote_bytes = (uint64_t)E.size() * w->vote_cap * rlo::kVoteSlot;

    // ---- control words: per rank an inbox block (tails) and an outbox block (heads)
    std::vector<uint32_t> inbox(n), outbox(n);
    uint64_t words = 0;
    for (int r = 0; r < n; r++) {
        inbox[r] = (uint32_t)words;
        words += (2 * in_edges[r].size() + T[r].sll + 15) & ~15ull;  // 128-byte blocks
        outbox[r] = (uint32_t)words;
        words += (2 * T[r].sll + in_edges[r].size() + 15) & ~15ull;
    }
    w->ctrl_words = words;

    w->topo.assign(n, rlo::RankTopo{});
    for (int r = 0; r < n; r++) {
        rlo::RankTopo& t = w->topo[r];
        t.level = T[r].level;
        t.last_wall = T[r].last_wall;
        t.scc = T[r].scc;
        t.sll = T[r].sll;
        for (int j = 0; j < T[r].sll; j++) t.send_list[j] = T[r].send_list[j];
        t.n_in = (int)in_edges[r].size();
        t.inbox_ctrl = inbox[r];
        t.n_inbox = 2 * t.n_in + t.sll;
        t.outbox_ctrl = outbox[r];
        t.n_outbox = 2 * t.sll + t.n_in;
    }
    const uint64_t ring_bytes = (uint64_t)cap * w->stride;
    for (int e = 0; e < (int)E.size(); e++) {
        const Edge& ed = E[e];
        rlo::RankTopo& P = w->topo[ed.src];  // producer of forward rings, consumer of votes
        rlo::RankTopo& C = w->topo[ed.dst];  // consumer of forward rings, producer of votes
        for (int vc = 0; vc < 2; vc++) {
            uint32_t data = (uint32_t)((2ull * e + vc) * ring_bytes);
            uint32_t tail = inbox[ed.dst] + 2 * ed.k + vc;
            uint32_t head = outbox[ed.src] + 2 * ed.j + vc;
            P.out_data[ed.j][vc] = data; P.out_tail[ed.j][vc] = tail; P.out_head[ed.j][vc] = head;
            C.in_data[ed.k][vc] = data; C.in_tail[ed.k][vc] = tail; C.in_head[ed.k][vc] = head;
        }
        C.in_src[ed.k] = ed.src;
        uint32_t vdata = (uint32_t)((uint64_t)e * w->vote_cap * rlo::kVoteSlot);
        uint32_t vtail = inbox[ed.src] + 2 * P.n_in + ed.j;
        uint32_t vhead = outbox[ed.dst] + 2 * C.sll + ed.k;
        C.vout_data[ed.k] = vdata; C.vout_tail[ed.k] = vtail; C.vout_head[ed.k] = vhead;
        P.vin_data[ed.j] = vdata; P.vin_tail[ed.j] = vtail; P.vin_head[ed.j] = vhead;
    }

    // ---- residency: every rank-workgroup must be resident at once (persistent kernel).
    // Dynamic LDS = [pend 2N x 16 B][olist 2 max_fan x 256 x 2 B][stage 256 x nsmall x 16 B][stage2].
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, w->device) != hipSuccess) { delete w; return RLO_E_HIP; }
    w->cus = prop.multiProcessorCount;
    {
        // Largest small-path stage (nsmall chunks per message, <= 8) and then the largest stage2
        // (<= 64 KiB) at which the occupancy calculator (LDS allocation granularity, registers,
        // waves) still co-schedules need_bpc rank-workgroups per CU.
        const size_t lds_cu = 163840;  // 160 KiB per CU (MI355X_MICROARCH.md)
        const int need_bpc = (n + w->cus - 1) / w->cus;
        const size_t per_block = lds_cu / need_bpc;
        int api = 0;
        bool ok = false;
        for (uint32_t ns = std::min<uint32_t>(8u, w->stride / 16u); ns >= 1 && !ok; ns--) {
            const size_t fixed = rlo_kernel_static_lds() + (size_t)32 * n + (size_t)2 * w->max_fan * 256 * 2 +
                                 (size_t)rlo::kMaxCand * ns * 16;
            if (per_block < fixed + 1024 + 512) continue;
            size_t s2 = std::min<size_t>(64 * 1024, (per_block - fixed - 512) & ~(size_t)1023);
            for (;;) {
                w->dyn_lds = fixed - rlo_kernel_static_lds() + s2;
                if (rlo_occupancy(&api, w->dyn_lds) != hipSuccess) api = 0;
                if (api >= need_bpc) { ok = true; break; }
                if (s2 <= 1024) break;
                s2 -= 1024;
            }
            w->nsmall = ns;
            w->stage2 = (uint32_t)s2;
        }
        if (!ok) { delete w; return RLO_E_OCCUPANCY; }
        w->blocks_per_cu = std::max(1, api);
        if (n > w->blocks_per_cu * w->cus) { delete w; return RLO_E_OCCUPANCY; }
    }

    // ---- allocate
    if (hipMalloc(&w->fwd, w->fwd_bytes) != hipSuccess ||
        hipMalloc(&w->vote, w->vote_bytes) != hipSuccess ||
        hipMalloc(&w->ctrl, w->ctrl_words * 8) != hipSuccess) {
        g_last_hip = (int)hipGetLastError();
        rlo_world_destroy(w);
        return RLO_E_HIP;
    }
    if (w->d_topo.upload(w->topo) || w->d_stats.alloc(n) || w->d_err.alloc(4)) {
        rlo_world_destroy(w);
        return RLO_E_HIP;
    }
    (void)hipMemset(w->fwd, 0, w->fwd_bytes);
    (void)hipMemset(w->vote, 0, w->vote_bytes);
    (void)hipEventCreate(&w->ev0);
    (void)hipEventCreate(&w->ev1);
    *out = w;
    return RLO_OK;
}

int rlo_world_destroy(rlo_world_t* w) {
    if (!w) return RLO_E_INVAL;
    if (w->fwd) (void)hipFree(w->fwd);
    if (w->vote) (void)hipFree(w->vote);
    if (w->ctrl) (void)hipFree(w->ctrl);
    w->d_topo.release(); w->d_stats.release(); w->d_err.release();
    w->d_sched_off.release(); w->d_expect_bcast.release(); w->d_prop_off.release(); w->d_expect_dec.release();
    w->d_sched_ids.release(); w->d_prop_data_off.release(); w->d_prop_data_len.release(); w->d_isp_off.release();
    w->d_lat_count.release(); w->d_lat_round.release(); w->d_lat_origin.release(); w->d_prop_pid.release();
    w->d_lat_out.release(); w->d_mask.release(); w->d_prop_data.release(); w->d_log_payload.release();
    w->d_isp.release(); w->d_log.release();
    if (w->ev0) (void)hipEventDestroy(w->ev0);
    if (w->ev1) (void)hipEventDestroy(w->ev1);
    delete w;
    return RLO_OK;
}

int rlo_world_query(const rlo_world_t* w, rlo_world_info_t* o) {
    if (!w || !o) return RLO_E_INVAL;
    std::memset(o, 0, sizeof *o);
    o->n_ranks = w->n;
    o->max_in_degree = w->max_in;
    o->max_fanout = w->max_fan;
    o->edges = w->edges;
    o->ring_slots = w->fwd_cap;
    o->slot_stride = w->stride;
    o->vote_slots = w->vote_cap;
    o->fwd_bytes = w->fwd_bytes;
    o->vote_bytes = w->vote_bytes;
    o->ctrl_bytes = w->ctrl_words * 8;
    o->cus = w->cus;
    o->blocks_per_cu = w->blocks_per_cu;
    return RLO_OK;
}

static void base_params(rlo_world* w) {
    rlo::Params& P = w->P;
    std::memset(&P, 0, sizeof P);
    P.n = w->n;
    P.rank_begin = 0;
    P.rank_end = w->n;
    P.topo = w->d_topo.p;
    P.fwd_region = w->fwd;
    P.fwd_region_bytes = (uint32_t)w->fwd_bytes;
    P.fwd_cap = w->fwd_cap;
    P.fwd_stride = w->stride;
    P.vote_region = w->vote;
    P.vote_region_bytes = (uint32_t)w->vote_bytes;
    P.vote_cap = w->vote_cap;
    P.ctrl = w->ctrl;
    P.stats = w->d_stats.p;
    P.error_flag = w->d_err.p;
    P.nsmall = w->nsmall;
    P.nout_max = 2u * (uint32_t)w->max_fan;
    P.stage2_bytes = w->stage2;
    P.timeout_ticks = 100000000ull * 10;   // 10 s without progress on a rank
    P.deadline_ticks = 100000000ull * 120; // 120 s per launch
    P.window = 32;
    // harmless non-null defaults for unused arrays
    static_assert(sizeof(int64_t) == 8, "");
}

static int setup_log(rlo_world* w, uint32_t flags, uint32_t log_cap, bool payload) {
    rlo::Params& P = w->P;
    if (!(flags & RLO_FLAG_LOG)) return RLO_OK;
    if (log_cap == 0) log_cap = 1024;
    if (w->d_log.alloc((size_t)w->n * log_cap)) return RLO_E_HIP;
    P.log = w->d_log.p;
    P.log_cap = log_cap;
    P.mode |= rlo::MODE_LOG;
    if (payload) {
        P.log_stride = w->max_payload;
        if (w->d_log_payload.alloc((size_t)w->n * log_cap * P.log_stride)) return RLO_E_HIP;
        P.log_payload = w->d_log_payload.p;
    }
    return RLO_OK;
}

int rlo_program_storm(rlo_world_t* w, const rlo_storm_cfg_t* cfg) {
    if (!w || !cfg || cfg->k < 0 || cfg->len > w->max_payload || cfg->k > 0xFFFFFFFFll) return RLO_E_INVAL;
    base_params(w);
    rlo::Params& P = w->P;
    const int n = w->n;
    std::vector<int64_t> off(n + 1, 0), expect(n, 0);
    std::vector<uint32_t> ids((size_t)std::max<int64_t>(cfg->k, 1));
    std::vector<uint32_t> org((size_t)std::max<int64_t>(cfg->k, 1));
    for (int64_t b = 0; b < cfg->k; b++) {
        org[b] = (uint32_t)(splitmix64(cfg->seed + (uint64_t)b) % (uint64_t)n);
        off[org[b] + 1]++;
    }
    for (int r = 0; r < n; r++) off[r + 1] += off[r];
    std::vector<int64_t> fill(off.begin(), off.end() - 1);
    for (int64_t b = 0; b < cfg->k; b++) ids[fill[org[b]]++] = (uint32_t)b;
    for (int r = 0; r < n; r++) expect[r] = cfg->k - (off[r + 1] - off[r]);
    if (w->d_sched_off.upload(off) || w->d_sched_ids.upload(ids) || w->d_expect_bcast.upload(expect)) return RLO_E_HIP;
    P.mode = rlo::MODE_STORM | ((cfg->flags & RLO_FLAG_HIST) ? rlo::MODE_HIST : 0u) |
             ((cfg->flags & RLO_FLAG_PROF) ? rlo::MODE_PROF : 0u);
    P.seed = cfg->seed;
    P.len = cfg->len;
    P.window = std::min<uint32_t>(cfg->window ? cfg->window : 32, 64u);  // one wave prefetches the ids
    P.sched_off = w->d_sched_off.p;
    P.sched_ids = w->d_sched_ids.p;
    P.expect_bcast = w->d_expect_bcast.p;
    int rc = setup_log(w, cfg->flags, cfg->log_cap, true);
    if (rc) return rc;
    w->have_program = true;
    return RLO_OK;
}

int rlo_program_latency(rlo_world_t* w, uint32_t rounds, uint32_t len, uint64_t seed, uint32_t flags) {
    if (!w || rounds == 0 || len > w->max_payload) return RLO_E_INVAL;
    base_params(w);
    rlo::Params& P = w->P;
    const int n = w->n;
    std::vector<int32_t> org(rounds);
    std::vector<int64_t> expect(n, 0);
    for (uint32_t i = 0; i < rounds; i++) org[i] = (int32_t)(splitmix64(seed + i) % (uint64_t)n);
    for (int r = 0; r < n; r++)
        for (uint32_t i = 0; i < rounds; i++) expect[r] += org[i] != r;
    if (w->d_lat_origin.upload(org) || w->d_expect_bcast.upload(expect) || w->d_lat_count.alloc(rounds) ||
        w->d_lat_out.alloc(rounds) || w->d_lat_round.alloc(1))
        return RLO_E_HIP;
    P.mode = rlo::MODE_LAT | ((flags & RLO_FLAG_HIST) ? rlo::MODE_HIST : 0u);
    P.len = len;
    P.seed = seed;
    P.lat_rounds = rounds;
    P.lat_origin = w->d_lat_origin.p;
    P.lat_count = w->d_lat_count.p;
    P.lat_out = w->d_lat_out.p;
    P.lat_round = w->d_lat_round.p;
    P.expect_bcast = w->d_expect_bcast.p;
    w->lat_rounds = rounds;
    int rc = setup_log(w, flags, 0, true);
    if (rc) return rc;
    w->have_program = true;
    return RLO_OK;
}

int rlo_program_iar(rlo_world_t* w, const rlo_iar_cfg_t* cfg, int64_t nprop, const int32_t* origin, const int32_t* pid,
                    const uint8_t* data, const uint32_t* data_off, const uint32_t* data_len) {
    if (!w || !cfg || nprop < 0 || (nprop && (!origin || !pid || !data_off || !data_len))) return RLO_E_INVAL;
    base_params(w);
    rlo::Params& P = w->P;
    const int n = w->n;
    std::vector<int64_t> off(n + 1, 0), expect(n, 0);
    for (int64_t i = 0; i < nprop; i++) {
        if (origin[i] < 0 || origin[i] >= n) return RLO_E_INVAL;
        if (16ull + data_len[i] > w->max_payload) return RLO_E_INVAL;
        off[origin[i] + 1]++;
    }
    for (int r = 0; r < n; r++) off[r + 1] += off[r];
    std::vector<int64_t> fill(off.begin(), off.end() - 1);
    std::vector<int32_t> ppid((size_t)std::max<int64_t>(nprop, 1));
    std::vector<uint32_t> pdo((size_t)std::max<int64_t>(nprop, 1)), pdl((size_t)std::max<int64_t>(nprop, 1));
    std::vector<uint8_t> blob;
    for (int64_t i = 0; i < nprop; i++) {
        int64_t at = fill[origin[i]]++;
        ppid[at] = pid[i];
        pdo[at] = (uint32_t)blob.size();
        pdl[at] = data_len[i];
        blob.insert(blob.end(), data + data_off[i], data + data_off[i] + data_len[i]);
    }
    if (blob.empty()) blob.push_back(0);
    for (int r = 0; r < n; r++) expect[r] = nprop - (off[r + 1] - off[r]);
    if (w->d_prop_off.upload(off) || w->d_prop_pid.upload(ppid) || w->d_prop_data_off.upload(pdo) ||
        w->d_prop_data_len.upload(pdl) || w->d_prop_data.upload(blob) || w->d_expect_dec.upload(expect))
        return RLO_E_HIP;
    P.mode = rlo::MODE_IAR | ((cfg->flags & RLO_FLAG_PROF) ? rlo::MODE_PROF : 0u);
    P.judge_kind = cfg->judge_kind;
    P.judge_ppm = cfg->judge_ppm;
    P.judge_seed = cfg->judge_seed;
    std::vector<uint8_t> mask(n, 0);
    if (cfg->judge_kind == RLO_JUDGE_MASK) {
        if (!cfg->judge_mask) return RLO_E_INVAL;
        std::memcpy(mask.data(), cfg->judge_mask, n);
    }
    if (w->d_mask.upload(mask)) return RLO_E_HIP;
    P.judge_mask = w->d_mask.p;
    std::vector<char> isp;
    std::vector<uint32_t> isp_off(n, 0);
    if (cfg->judge_kind == RLO_JUDGE_ISP) {
        if (!cfg->judge_isp) return RLO_E_INVAL;
        const char* s = cfg->judge_isp;
        for (int r = 0; r < n; r++) {
            isp_off[r] = (uint32_t)isp.size();
            size_t l = std::strlen(s);
            isp.insert(isp.end(), s, s + l + 1);
            s += l + 1;
        }
    } else {
        isp.push_back(0);
    }
    if (w->d_isp.upload(isp) || w->d_isp_off.upload(isp_off)) return RLO_E_HIP;
    P.judge_isp = w->d_isp.p;
    P.judge_isp_off = w->d_isp_off.p;
    P.prop_off = w->d_prop_off.p;
    P.prop_pid = w->d_prop_pid.p;
    P.prop_data_off = w->d_prop_data_off.p;
    P.prop_data_len = w->d_prop_data_len.p;
    P.prop_data = w->d_prop_data.p;
    P.expect_dec = w->d_expect_dec.p;
    int rc = setup_log(w, cfg->flags, cfg->log_cap, false);
    if (rc) return rc;
    w->have_program = true;
    return RLO_OK;
}

int rlo_launch(rlo_world_t* w, void* stream) {
    if (!w) return RLO_E_INVAL;
    if (!w->have_program) return RLO_E_NOPROGRAM;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipMemsetAsync(w->ctrl, 0, w->ctrl_words * 8, s));
    HIPCHK(hipMemsetAsync(w->d_stats.p, 0, sizeof(rlo::RankStats) * w->n, s));
    HIPCHK(hipMemsetAsync(w->d_err.p, 0, sizeof(uint32_t) * 4, s));
    if (w->P.mode & rlo::MODE_LAT) {
        HIPCHK(hipMemsetAsync(w->d_lat_count.p, 0, sizeof(uint32_t) * w->lat_rounds, s));
        HIPCHK(hipMemsetAsync(w->d_lat_out.p, 0, sizeof(uint64_t) * w->lat_rounds, s));
        HIPCHK(hipMemsetAsync(w->d_lat_round.p, 0, sizeof(uint32_t), s));
    }
    HIPCHK(hipEventRecord(w->ev0, s));
    hipError_t e = rlo_launch_progress(&w->P, w->n, w->dyn_lds, s);
    if (e != hipSuccess) { g_last_hip = (int)e; return RLO_E_HIP; }
    HIPCHK(hipEventRecord(w->ev1, s));
    w->last_stream = s;
    return RLO_OK;
}

int rlo_wait(rlo_world_t* w) {
    if (!w) return RLO_E_INVAL;
    HIPCHK(hipEventSynchronize(w->ev1));
    HIPCHK(hipEventElapsedTime(&w->last_ms, w->ev0, w->ev1));
    uint32_t err = 0;
    HIPCHK(hipMemcpy(&err, w->d_err.p, sizeof err, hipMemcpyDeviceToHost));
    return err ? RLO_E_DEVICE : RLO_OK;
}

int rlo_run(rlo_world_t* w, void* stream, float* ms) {
    int rc = rlo_launch(w, stream);
    if (rc) return rc;
    rc = rlo_wait(w);
    if (ms) *ms = w->last_ms;
    return rc;
}

int rlo_last_kernel_ms(rlo_world_t* w, float* ms) {
    if (!w || !ms) return RLO_E_INVAL;
    *ms = w->last_ms;
    return RLO_OK;
}

int rlo_stats(rlo_world_t* w, rlo_rank_stats_t* out, int n) {
    if (!w || !out || n < 0 || n > w->n) return RLO_E_INVAL;
    HIPCHK(hipMemcpy(out, w->d_stats.p, sizeof(rlo::RankStats) * n, hipMemcpyDeviceToHost));
    return RLO_OK;
}

int rlo_log(rlo_world_t* w, int rank, rlo_log_rec_t* out, uint32_t cap, uint8_t* payload, uint32_t payload_stride) {
    if (!w || rank < 0 || rank >= w->n || !out) return RLO_E_INVAL;
    if (!w->d_log.p) return RLO_E_NOPROGRAM;
    rlo::RankStats st;
    HIPCHK(hipMemcpy(&st, w->d_stats.p + rank, sizeof st, hipMemcpyDeviceToHost));
    uint32_t cnt = (uint32_t)std::min<uint64_t>(st.log_count, w->P.log_cap);
    cnt = std::min(cnt, cap);
    if (cnt) HIPCHK(hipMemcpy(out, w->d_log.p + (size_t)rank * w->P.log_cap, sizeof(rlo::LogRec) * cnt, hipMemcpyDeviceToHost));
    if (payload && w->d_log_payload.p && cnt) {
        const uint32_t ls = w->P.log_stride;
        std::vector<uint8_t> tmp((size_t)cnt * ls);
        HIPCHK(hipMemcpy(tmp.data(), w->d_log_payload.p + (size_t)rank * w->P.log_cap * ls, tmp.size(), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < cnt; i++)
            std::memcpy(payload + (size_t)i * payload_stride, tmp.data() + (size_t)i * ls, std::min(ls, payload_stride));
    }
    return (int)cnt;
}

int rlo_latencies(rlo_world_t* w, uint64_t* ticks, uint32_t cap) {
    if (!w || !ticks || !w->d_lat_out.p) return RLO_E_INVAL;
    uint32_t n = std::min(cap, w->lat_rounds);
    HIPCHK(hipMemcpy(ticks, w->d_lat_out.p, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
    return (int)n;
}

}  // extern "C"
