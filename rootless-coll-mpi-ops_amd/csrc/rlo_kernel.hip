// rlo_kernel.hip -- the persistent progress kernel (gfx950 / CDNA4).
//
// One 256-thread workgroup = one virtual rank.  Each progress iteration is the
// device restatement of make_progress_gen (rootless_ops.c:551-641), batched:
//
//   A  poll     : one relaxed agent-scope load per in-ring tail / out-ring head
//                 (replaces MPI_Test of the single ANY_SOURCE irecv, :643-650)
//   B  votes    : drain every vote ring; LDS-atomic AND-merge (_iar_vote_handler :743-812)
//   C  select   : up to 256 messages: the in-ring backlog (FIFO per ring), then
//                 local originations (RLO_bcast_gen :1581, own proposal / decision)
//   D  classify : header load, skip-ring child set relative to the dynamic origin
//                 (_bc_forward :1104-1225), device judge for proposals (:698)
//   E  admit    : per out-ring positions by wave ballots; credit check; FIFO prefix
//   F  effects  : deliveries (pickup), proposal state, decisions + actions (:814-859), votes up (:728)
//   G  copy     : wave-wide 16-byte chunks: one write-through (sc1) load, one sc1 store per child
//   H  publish  : every wave drains vmcnt, barrier, relaxed agent-scope tail/head stores
//
// Memory ordering (MI355X_MICROARCH.md "Valid forms", row 1): payload stores and
// loads are all sc1 (L1-bypassing, written through), each storing wave drains
// vmcnt(0) before the workgroup barrier, then one lane stores the counter.
#include <hip/hip_runtime.h>

#include "rlo_device.hpp"

namespace rlo {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static constexpr int kAuxSc1 = 16;  // cache policy: sc1 (agent scope, write-through / L1 bypass)
static constexpr uint32_t kGolden32 = 0x9E3779B9u;
static constexpr uint64_t kGolden64 = 0x9E3779B97F4A7C15ull;

enum CandKind : uint8_t { K_RING = 0, K_STORM = 1, K_PROP = 2, K_DEC = 3, K_LAT = 4, K_BAD = 7 };
static constexpr int kGroupLocal = 2 * kMaxIn;   // groups [0, 64) = in-rings (k*2+vc); 64.. local kinds
static constexpr int kGroups = kGroupLocal + 8;
static constexpr int kMaxVoteEmit = 2 * kMaxCand;

struct Cand {
    uint32_t src;     // K_RING: byte offset of the slot in the forward region; K_PROP: proposal index
    uint32_t w0;      // origin | tag << 16 | vote << 24
    uint32_t id;      // bcast id / pid
    uint32_t w2;      // len | pseq << 24
    uint32_t t0;
    uint32_t need;    // out-ring bits oi = j*2 + vc
    uint32_t kids;    // child bits j
    uint32_t logidx;  // log record of this delivery (payload capture) or ~0u
    int16_t from;     // sender rank (-1: originated here)
    uint8_t group;
    uint8_t kind;
    int32_t judge;    // proposals: judge result
};

struct PendState {      // a proposal held at a non-originator (queue_iar_pending, :1138)
    int32_t pid;
    uint32_t word;      // votes received (low 16 b) | zero votes (high 16 b)
    uint16_t parent_k;  // in-edge the proposal came from (vote goes back on it)
    uint8_t needed;     // fwd_send_cnt (:694)
    uint8_t valid;
    uint32_t pseq;
};

struct VoteEmit {
    uint32_t k, w0, pid, pseq;
};

struct Shared {
    RankTopo t;
    uint64_t in_head[2 * kMaxIn], in_tail[2 * kMaxIn];
    uint64_t out_tail[kMaxOut], out_head[kMaxOut], out_tail0[kMaxOut];
    uint64_t vin_head[kMaxFanout], vin_tail[kMaxFanout];
    uint64_t vout_tail[kMaxIn], vout_head[kMaxIn];
    Cand cand[kMaxCand];
    uint16_t pos[kMaxCand][kMaxFanout];
    uint32_t ring_base[2 * kMaxIn + 1], ring_take[2 * kMaxIn];
    uint32_t vbase[kMaxFanout + 1];
    uint32_t wave_cnt[kWaves][kMaxOut];
    uint32_t first_bad[kGroups];
    uint32_t cum[kMaxCand + 1];
    uint32_t wave_sum[kWaves];
    VoteEmit vemit[kMaxVoteEmit];
    uint32_t nvemit;
    uint32_t ncand, nring, nvote, nlocal_storm;
    // own proposal (my_own_proposal, :241)
    int32_t own_pid;
    uint32_t own_word, own_needed, own_state, own_decision, own_pseq;
    int64_t own_iter, own_n;
    // origination progress
    int64_t sched_next, sched_n;
    uint32_t lat_next;
    // counters
    unsigned long long bcast_delivered, dec_delivered, dec_approved, actions, judge_calls, originated;
    unsigned long long own_decided, own_approved, proposals_recv, log_count, iterations, busy, stalls;
    uint32_t error, error_aux, done, progressed;
    uint64_t last_progress;
    uint32_t hist[kHistBins];
};

// ------------------------------------------------------------------ helpers

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSc1);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSc1);
}
__device__ __forceinline__ uint8_t ld8_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, kAuxSc1);
}
__device__ __forceinline__ uint64_t poll64(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pub64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t poll32(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + kGolden64;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// storm payload word k (DESIGN.md "storm workload"; the oracle's rlo_testvec.h states the same)
__device__ __forceinline__ uint64_t storm_word(uint32_t origin, uint32_t bid, uint32_t k) {
    uint64_t w0 = ((uint64_t)bid << 32) | origin;
    return k == 0 ? w0 : splitmix64(w0 ^ ((uint64_t)k * kGolden64));
}

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ uint32_t chunk_mix(uint32_t q, u32x4 w) {
    return fmix32(w.x ^ fmix32(w.y ^ fmix32(w.z ^ fmix32(w.w ^ (q * kGolden32 + 0x7F4A7C15u)))));
}

__device__ __forceinline__ uint32_t mask_bytes(uint32_t w, int keep) {  // keep low `keep` bytes
    return keep >= 4 ? w : (keep <= 0 ? 0u : (w & ((1u << (8 * keep)) - 1u)));
}

// rootless_ops.c:1534-1556
__device__ __forceinline__ bool passed_origin(int me, int origin, int to) {
    if (to == origin) return true;
    if (me >= origin) {
        if (to > me) return false;
        if (to >= 0 && to < origin) return false;
        return true;
    }
    return !(to > me && to < origin);
}

// child index set j of send_list: originate (:1587) or _bc_forward (:1116-1223)
__device__ __forceinline__ uint32_t children(const RankTopo& t, int me, int origin, int from) {
    if (from < 0) return (1u << t.sll) - 1u;
    if (t.level <= 0) return 0u;
    if (from > t.last_wall) return (1u << (t.scc + 1)) - 1u;
    uint32_t m = 0;
    for (int j = t.scc - 1; j >= 0; j--)
        if (!passed_origin(me, origin, t.send_list[j])) m |= 1u << j;
    return m;
}

__device__ __forceinline__ uint32_t need_bits(const RankTopo& t, uint32_t kids, int origin) {
    uint32_t need = 0;
    while (kids) {
        int j = __builtin_ctz(kids);
        kids &= kids - 1;
        need |= 1u << (2 * j + (t.send_list[j] < origin ? 1 : 0));
    }
    return need;
}

__device__ __forceinline__ uint32_t hist_bin(uint64_t d) {
    if (d < 8) return (uint32_t)d;
    int o = 63 - __builtin_clzll(d);
    uint32_t b = (uint32_t)(o - 2) * 8u + (uint32_t)((d >> (o - 3)) & 7u);
    return b < kHistBins ? b : kHistBins - 1;
}

__device__ __forceinline__ void set_error(Shared& S, const Params& P, uint32_t code, uint32_t aux) {
    if (atomicCAS(&S.error, 0u, code) == 0u) {
        S.error_aux = aux;
        atomicCAS(P.error_flag, 0u, code);
    }
}

__device__ __forceinline__ uint32_t judge_hash(uint64_t seed, uint32_t rank, int32_t pid) {
    return (uint32_t)(splitmix64(seed ^ ((uint64_t)rank << 32) ^ (uint32_t)pid) % 1000000u);
}

// device judge registry; arg_off = byte offset of the proposal data in the forward region
// (data_len bytes, zero-extended: the reference's calloc'd receive buffer).  testcases.c:18-37
// for ISP.  The originator's final call passes NULL (rootless_ops.c:773): every device judge
// approves NULL.
__device__ int judge_eval(const Params& P, __amdgpu_buffer_rsrc_t rf, int me, int32_t pid, uint32_t arg_off,
                          uint32_t data_len) {
    switch (P.judge_kind) {
        case JUDGE_MASK:
            return P.judge_mask[me] ? 0 : 1;
        case JUDGE_HASH:
            return judge_hash(P.judge_seed, me, pid) < P.judge_ppm ? 0 : 1;
        case JUDGE_ISP: {
            const char* mine = P.judge_isp + P.judge_isp_off[me];
            if (mine[0] == 0) return 1;
            for (uint32_t i = 0;; i++) {  // strcmp(mine, arg)
                char a = i < data_len ? (char)ld8_sc1(rf, arg_off + i) : 0;
                if (a != mine[i]) break;
                if (a == 0) return 1;
            }
            char a0 = data_len ? (char)ld8_sc1(rf, arg_off) : 0;
            return ((signed char)a0 < (signed char)mine[0]) ? 0 : 1;
        }
        default:
            return 1;
    }
}

__device__ __forceinline__ uint32_t log_put(Shared& S, const Params& P, int lr, uint32_t kind, int origin, int from,
                                            uint32_t id, uint32_t len, int vote, uint32_t aux) {
    if (!(P.mode & MODE_LOG)) return ~0u;
    uint32_t i = (uint32_t)atomicAdd(&S.log_count, 1ull);
    if (i >= P.log_cap) {
        set_error(S, P, ERR_LOG_FULL, i);
        return ~0u;
    }
    LogRec r;
    r.kind = kind;
    r.origin = origin;
    r.from = from;
    r.id = id;
    r.len = len;
    r.vote = vote;
    r.aux = aux;
    r.payload_idx = (P.log_payload && kind == (LOG_DELIVER | (TAG_BCAST << 8))) ? i : ~0u;
    P.log[(size_t)lr * P.log_cap + i] = r;
    return r.payload_idx;
}

__device__ __forceinline__ void emit_vote(Shared& S, const Params& P, uint32_t k, int origin, int32_t pid, uint32_t pseq,
                                          int vote) {
    uint32_t i = atomicAdd(&S.nvemit, 1u);
    if (i >= kMaxVoteEmit) {
        set_error(S, P, ERR_VOTE_RING, 0xffffffffu);
        return;
    }
    S.vemit[i].k = k;
    S.vemit[i].w0 = (uint32_t)origin | ((uint32_t)(vote & 0xff) << 24);
    S.vemit[i].pid = (uint32_t)pid;
    S.vemit[i].pseq = pseq;
}

__device__ __forceinline__ uint32_t block_excl_scan(Shared& S, uint32_t v, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) S.wave_sum[wave] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        if (w < wave) off += S.wave_sum[w];
        tot += S.wave_sum[w];
    }
    *total = tot;
    return off + x - v;
}

// ------------------------------------------------------------------ the kernel

__global__ __launch_bounds__(kBlock, 1) void rlo_progress_kernel(Params P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    __shared__ Shared S;
    PendState* pend = reinterpret_cast<PendState*>(dyn_lds);  // [2 * n]

    const int lr = blockIdx.x;
    const int me = P.rank_begin + lr;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const __amdgpu_buffer_rsrc_t rf = mk_rsrc(P.fwd_region, P.fwd_region_bytes);
    const __amdgpu_buffer_rsrc_t rv = mk_rsrc(P.vote_region, P.vote_region_bytes);
    const uint32_t fcap_m = P.fwd_cap - 1, vcap_m = P.vote_cap - 1;

    // ---------------- init
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&P.topo[lr]);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&S.t);
        for (int i = tid; i < (int)(sizeof(RankTopo) / 4); i += kBlock) dst[i] = src[i];
        for (int i = tid; i < 2 * P.n; i += kBlock) pend[i] = PendState{0, 0, 0, 0, 0, 0};
        for (int i = tid; i < kHistBins; i += kBlock) S.hist[i] = 0;
        if (tid < 2 * kMaxIn) { S.in_head[tid] = 0; S.in_tail[tid] = 0; }
        if (tid < kMaxOut) { S.out_tail[tid] = 0; S.out_head[tid] = 0; }
        if (tid < kMaxFanout) { S.vin_head[tid] = 0; S.vin_tail[tid] = 0; }
        if (tid < kMaxIn) { S.vout_tail[tid] = 0; S.vout_head[tid] = 0; }
        if (tid == 0) {
            S.nvemit = 0;
            S.own_pid = -1;  // proposal_state_init, :1238
            S.own_word = 0; S.own_needed = 0; S.own_state = 0; S.own_decision = 0; S.own_pseq = 0;
            S.own_iter = 0;
            S.own_n = (P.mode & MODE_IAR) ? (P.prop_off[lr + 1] - P.prop_off[lr]) : 0;
            S.sched_next = 0;
            S.sched_n = (P.mode & MODE_STORM) ? (P.sched_off[lr + 1] - P.sched_off[lr]) : 0;
            S.lat_next = 0;
            S.bcast_delivered = S.dec_delivered = S.dec_approved = S.actions = S.judge_calls = S.originated = 0;
            S.own_decided = S.own_approved = S.proposals_recv = S.log_count = S.iterations = S.busy = S.stalls = 0;
            S.error = 0; S.error_aux = 0; S.done = 0;
            S.last_progress = now_ticks();
        }
    }
    __syncthreads();
    const uint64_t t_start = now_ticks();
    unsigned long long acc_sum = 0;  // checksum of delivered bcast chunks (this thread's share)

    for (;;) {
        const RankTopo& t = S.t;
        const int n_in2 = 2 * t.n_in;
        // ---------------- A: poll
        if (tid < (int)t.n_inbox) {
            uint64_t v = poll64(&P.ctrl[t.inbox_ctrl + tid]);
            if (tid < n_in2) S.in_tail[tid] = v;
            else S.vin_tail[tid - n_in2] = v;
        } else if (tid >= 128 && tid - 128 < (int)t.n_outbox) {
            int i = tid - 128;
            uint64_t v = poll64(&P.ctrl[t.outbox_ctrl + i]);
            if (i < 2 * t.sll) S.out_head[i] = v;
            else S.vout_head[i - 2 * t.sll] = v;
        }
        if (tid == 0) { S.nvemit = 0; S.progressed = 0; }
        __syncthreads();

        // ---------------- B: votes (children -> me)
        if (tid == 0) {
            uint32_t v = 0;
            for (int j = 0; j < t.sll; j++) {
                S.vbase[j] = v;
                uint64_t a = S.vin_tail[j] - S.vin_head[j];
                uint32_t room = kMaxCand - v;
                v += a < room ? (uint32_t)a : room;  // at most 256 votes per iteration
            }
            S.vbase[t.sll] = v;
            S.nvote = v;
        }
        __syncthreads();
        const uint32_t nvote = S.nvote;
        if (nvote) {
            for (uint32_t i = tid; i < nvote; i += kBlock) {
                int j = 0;
                while (i >= S.vbase[j + 1]) j++;
                uint64_t slot = S.vin_head[j] + (i - S.vbase[j]);
                u32x4 v = ld_sc1(rv, t.vin_data[j] + (uint32_t)(slot & vcap_m) * kVoteSlot);
                int origin = (int)(v.x & 0xffffu);
                int vote = (int)(int8_t)(v.x >> 24);
                int32_t pid = (int32_t)v.y;
                uint32_t pseq = v.z;
                if (origin >= P.n) {
                    set_error(S, P, ERR_BAD_SLOT, v.x);
                    continue;
                }
                uint32_t inc = 1u + (vote == 0 ? 0x10000u : 0u);
                if (origin == me) {  // a vote for my own proposal (:756-783)
                    if (S.own_state != 1 || pid != S.own_pid) {
                        set_error(S, P, ERR_VOTE_ORPHAN, (uint32_t)pid);
                        continue;
                    }
                    uint32_t old = atomicAdd(&S.own_word, inc);
                    uint32_t nw = old + inc;
                    if ((nw & 0xffffu) == S.own_needed) {
                        int d = (nw >> 16) == 0 ? 1 : 0;
                        if (d) {  // final judge(NULL) (:770-775)
                            d = 1;
                            atomicAdd(&S.judge_calls, 1ull);
                            log_put(S, P, lr, LOG_JUDGE, me, -1, (uint32_t)pid, 0, d, 1);
                        }
                        S.own_decision = (uint32_t)d;
                        S.own_state = 2;
                    }
                } else {  // _vote_merge (:1056-1070)
                    PendState* ps = &pend[2 * origin + (pseq & 1u)];
                    if (!ps->valid || ps->pid != pid) {
                        set_error(S, P, ERR_VOTE_ORPHAN, (uint32_t)pid);
                        continue;
                    }
                    uint32_t old = atomicAdd(&ps->word, inc);
                    uint32_t nw = old + inc;
                    if ((nw & 0xffffu) == ps->needed) emit_vote(S, P, ps->parent_k, origin, pid, pseq, (nw >> 16) == 0 ? 1 : 0);
                }
            }
        }

        __syncthreads();

        // ---------------- C: select candidates (thread 0)
        if (tid == 0) {
            uint32_t n = 0;
            const uint32_t reserve = (P.mode & MODE_IAR) ? 2u : 0u;
            // fair share: rotate which in-ring may fill the batch first (no ring starves)
            uint32_t* take_g = S.ring_take;
            const int g0 = n_in2 ? (int)(S.iterations % (uint64_t)n_in2) : 0;
            for (int i = 0; i < n_in2; i++) {
                const int g = (g0 + i) % n_in2;
                uint64_t a = S.in_tail[g] - S.in_head[g];
                uint32_t room = kMaxCand - reserve - n;
                uint32_t take = a < room ? (uint32_t)a : room;
                take_g[g] = take;
                n += take;
            }
            n = 0;
            for (int g = 0; g < n_in2; g++) {  // candidates stay grouped by ring, in ring order
                S.ring_base[g] = n;
                n += take_g[g];
            }
            S.ring_base[n_in2] = n;
            S.nring = n;
            // own proposal / decision (RLO_submit_proposal :876, _iar_decision_bcast :908)
            if (P.mode & MODE_IAR) {
                if (S.own_state == 2) {
                    Cand& c = S.cand[n++];
                    c.kind = K_DEC;
                    c.group = kGroupLocal + K_DEC;
                    c.id = (uint32_t)S.own_pid;
                    c.w0 = (uint32_t)me | (TAG_DECISION << 16) | ((S.own_decision & 0xffu) << 24);
                    c.w2 = 23u | (S.own_pseq << 24);
                } else if (S.own_state == 0 && S.own_iter < S.own_n) {
                    int64_t pi = P.prop_off[lr] + S.own_iter;
                    Cand& c = S.cand[n++];
                    c.kind = K_PROP;
                    c.group = kGroupLocal + K_PROP;
                    c.src = (uint32_t)pi;
                    c.id = (uint32_t)P.prop_pid[pi];
                    c.w0 = (uint32_t)me | (TAG_PROPOSAL << 16) | (1u << 24);
                    c.w2 = (16u + P.prop_data_len[pi]) | ((uint32_t)(S.own_iter & 0xff) << 24);
                }
            }
            // storm originations (RLO_msg_new_bc + RLO_bcast_gen)
            S.nlocal_storm = 0;
            if (P.mode & MODE_STORM) {
                int64_t rem = S.sched_n - S.sched_next;
                uint32_t w = rem < (int64_t)P.window ? (uint32_t)rem : P.window;
                if (w > kMaxCand - n) w = kMaxCand - n;
                const uint32_t* ids = P.sched_ids + P.sched_off[lr] + S.sched_next;
                for (uint32_t i = 0; i < w; i++) {
                    Cand& c = S.cand[n++];
                    c.kind = K_STORM;
                    c.group = kGroupLocal + K_STORM;
                    c.id = ids[i];
                }
                S.nlocal_storm = w;
            }
            if ((P.mode & MODE_LAT) && S.lat_next < P.lat_rounds && n < kMaxCand) {
                uint32_t r = poll32(P.lat_round);
                while (S.lat_next < P.lat_rounds && P.lat_origin[S.lat_next] != me) S.lat_next++;
                if (S.lat_next < P.lat_rounds && r == S.lat_next) {
                    Cand& c = S.cand[n++];
                    c.kind = K_LAT;
                    c.group = kGroupLocal + K_LAT;
                    c.id = S.lat_next;
                }
            }
            S.ncand = n;
        }
        __syncthreads();
        const uint32_t ncand = S.ncand, nring = S.nring;

        // ---------------- D: classify
        uint32_t my_need = 0;
        uint8_t my_group = 0;
        if ((uint32_t)tid < ncand) {
            Cand& c = S.cand[tid];
            if ((uint32_t)tid < nring) {
                int g = 0;
                while ((uint32_t)tid >= S.ring_base[g + 1]) g++;
                const int k = g >> 1, vc = g & 1;
                uint64_t slot = S.in_head[g] + (tid - S.ring_base[g]);
                uint32_t off = t.in_data[k][vc] + (uint32_t)(slot & fcap_m) * P.fwd_stride;
                u32x4 h = ld_sc1(rf, off);
                c.src = off;
                c.w0 = h.x;
                c.id = h.y;
                c.w2 = h.z;
                c.t0 = h.w;
                c.from = (int16_t)t.in_src[k];
                c.group = (uint8_t)g;
                c.kind = K_RING;
                const int origin = (int)(h.x & 0xffffu);
                const uint32_t tag = (h.x >> 16) & 0xffu;
                uint32_t kids = 0;
                c.judge = 1;
                if (origin >= P.n || (tag == TAG_BCAST && (P.mode & MODE_LAT) && h.y >= P.lat_rounds)) {
                    set_error(S, P, ERR_BAD_SLOT, h.x);
                    c.kind = K_BAD;  // consumed, never forwarded, no side effects
                } else if (tag == TAG_BCAST || tag == TAG_DECISION) {
                    kids = children(t, me, origin, t.in_src[k]);
                } else if (tag == TAG_PROPOSAL) {
                    // PBuf [pid][vote][data_len u64][data] starts at slot + 16 (rootless_ops.c:1402-1410)
                    u32x4 pb = ld_sc1(rf, off + kHdr);
                    uint32_t dl = pb.z;
                    uint32_t plen = (h.z & 0xffffffu);
                    if (dl > plen - 16u) dl = plen > 16u ? plen - 16u : 0u;
                    c.judge = judge_eval(P, rf, me, (int32_t)h.y, off + kHdr + 16u, dl);
                    kids = c.judge ? children(t, me, origin, t.in_src[k]) : 0u;
                } else {
                    set_error(S, P, ERR_BAD_SLOT, h.x);
                    c.kind = K_BAD;
                }
                c.kids = kids;
                my_need = need_bits(t, kids, origin);
            } else {
                c.from = -1;
                c.t0 = (uint32_t)now_ticks();
                if (c.kind == K_STORM || c.kind == K_LAT) {
                    c.w0 = (uint32_t)me | (TAG_BCAST << 16) | (0xffu << 24);
                    c.w2 = P.len;
                }
                c.kids = (1u << t.sll) - 1u;
                my_need = need_bits(t, c.kids, me);
            }
            c.need = my_need;
            c.logidx = ~0u;
            my_group = c.group;
        }
        if (tid < kGroups) S.first_bad[tid] = 0xffffffffu;
        __syncthreads();

        // ---------------- E: admission
        const int nout = 2 * t.sll;
        for (int oi = 0; oi < nout; oi++) {
            uint64_t b = __ballot((my_need >> oi) & 1u);
            if (lane == 0) S.wave_cnt[wave][oi] = (uint32_t)__popcll(b);
        }
        __syncthreads();
        bool fits = (uint32_t)tid < ncand;
        for (int oi = 0; oi < nout; oi++) {
            uint64_t b = __ballot((my_need >> oi) & 1u);
            if ((my_need >> oi) & 1u) {
                uint32_t pre = (uint32_t)__popcll(b & lt_mask);
                for (int w = 0; w < wave; w++) pre += S.wave_cnt[w][oi];
                uint64_t used = S.out_tail[oi] - S.out_head[oi];
                if ((uint64_t)pre + used >= P.fwd_cap) fits = false;
            }
        }
        __syncthreads();  // wave_cnt reuse below
        if ((uint32_t)tid < ncand && !fits) atomicMin(&S.first_bad[my_group], (uint32_t)tid);
        __syncthreads();
        const bool admitted = (uint32_t)tid < ncand && fits && (uint32_t)tid < S.first_bad[my_group];
        const uint32_t adm_need = admitted ? my_need : 0u;
        for (int oi = 0; oi < nout; oi++) {
            uint64_t b = __ballot((adm_need >> oi) & 1u);
            if (lane == 0) S.wave_cnt[wave][oi] = (uint32_t)__popcll(b);
        }
        __syncthreads();
        // per-oi positions: every lane takes part in each ballot
        for (int oi = 0; oi < nout; oi++) {
            const bool bit = (adm_need >> oi) & 1u;
            uint64_t b = __ballot(bit);
            if (bit) {
                uint32_t pre = (uint32_t)__popcll(b & lt_mask);
                for (int w = 0; w < wave; w++) pre += S.wave_cnt[w][oi];
                const int j = oi >> 1;
                S.pos[tid][j] = (uint16_t)pre;
            }
        }
        __syncthreads();
        if (tid < nout) {
            uint32_t tot = 0;
            for (int w = 0; w < kWaves; w++) tot += S.wave_cnt[w][tid];
            S.out_tail0[tid] = S.out_tail[tid];
            S.out_tail[tid] += tot;
        }
        if (tid < n_in2) {  // consume the admitted prefix of every in-ring
            uint32_t base = S.ring_base[tid], take = S.ring_take[tid];
            uint32_t fb = S.first_bad[tid];
            uint32_t adm = fb == 0xffffffffu ? take : (fb > base ? fb - base : 0u);
            if (adm > take) adm = take;
            S.in_head[tid] += adm;
            if (adm < take) atomicAdd(&S.stalls, 1ull);
        }

        // ---------------- F: side effects of admitted messages
        if (admitted) {
            S.progressed = 1;
            Cand& c = S.cand[tid];
            const int origin = (int)(c.w0 & 0xffffu);
            const uint32_t tag = (c.w0 >> 16) & 0xffu;
            const int vote = (int)(int8_t)(c.w0 >> 24);
            const uint32_t len = c.w2 & 0xffffffu, pseq = c.w2 >> 24;
            if (c.kind == K_RING) {
                if (tag == TAG_BCAST) {  // delivered to this rank's pickup queue (:583-589)
                    atomicAdd(&S.bcast_delivered, 1ull);
                    const uint64_t tn = now_ticks();
                    if (P.mode & MODE_HIST) atomicAdd(&S.hist[hist_bin((uint32_t)tn - c.t0)], 1u);
                    c.logidx = log_put(S, P, lr, LOG_DELIVER | (TAG_BCAST << 8), origin, c.from, c.id, len, -1, 0);
                    if (P.mode & MODE_LAT) {
                        uint32_t old = atomicAdd(&P.lat_count[c.id], 1u);
                        if (old + 1u == (uint32_t)(P.n - 1)) {
                            P.lat_out[c.id] = (uint64_t)((uint32_t)tn - c.t0);
                            __hip_atomic_store(P.lat_round, c.id + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                } else if (tag == TAG_PROPOSAL) {  // _iar_proposal_handler (:668-726)
                    const int32_t pid = (int32_t)c.id;
                    const int k = c.group >> 1;
                    atomicAdd(&S.proposals_recv, 1ull);
                    if (S.own_state != 0 && pid == S.own_pid) {
                        set_error(S, P, ERR_PID_COLLISION, (uint32_t)pid);  // :690-692 (reference never votes)
                    } else {
                        atomicAdd(&S.judge_calls, 1ull);
                        log_put(S, P, lr, LOG_JUDGE, origin, c.from, (uint32_t)pid, len, c.judge, 0);
                        if (!c.judge) {
                            emit_vote(S, P, (uint32_t)k, origin, pid, pseq, 0);
                        } else {
                            PendState* ps = &pend[2 * origin + (pseq & 1u)];
                            uint32_t nk = (uint32_t)__builtin_popcount(c.kids);
                            ps->pid = pid;
                            ps->word = 0;
                            ps->parent_k = (uint16_t)k;
                            ps->needed = (uint8_t)nk;
                            ps->pseq = pseq | ((len - 16u) << 8);  // + proposal data_len (action argument)
                            ps->valid = 1;
                            if (nk == 0) emit_vote(S, P, (uint32_t)k, origin, pid, pseq, 1);
                        }
                    }
                } else if (tag == TAG_DECISION) {  // :603-615, _iar_decision_handler :814-859
                    PendState* ps = &pend[2 * origin + (pseq & 1u)];
                    if (ps->valid && ps->pid == (int32_t)c.id) {
                        if (vote != 0) {
                            atomicAdd(&S.actions, 1ull);
                            log_put(S, P, lr, LOG_ACTION, origin, c.from, c.id, 0, 1, ps->pseq >> 8);
                        }
                        ps->valid = 0;
                    }
                    atomicAdd(&S.dec_delivered, 1ull);
                    if (vote != 0) atomicAdd(&S.dec_approved, 1ull);
                    log_put(S, P, lr, LOG_DELIVER | (TAG_DECISION << 8), origin, c.from, c.id, 7, vote, 0);
                }
            } else if (c.kind == K_PROP) {
                S.own_pid = (int32_t)c.id;
                S.own_word = 0;
                S.own_needed = (uint32_t)t.sll;  // votes_needed = send_list_len (:881)
                S.own_pseq = pseq;
                S.own_state = 1;
            } else if (c.kind == K_DEC) {
                atomicAdd(&S.own_decided, 1ull);
                if (vote) atomicAdd(&S.own_approved, 1ull);
                log_put(S, P, lr, LOG_RESULT, me, -1, c.id, 0, vote, 0);
                S.own_state = 0;
                S.own_pid = -1;  // RLO_proposal_reset via RLO_get_vote_my_proposal (:1649-1673)
                S.own_iter++;
            } else if (c.kind == K_STORM || c.kind == K_LAT) {
                atomicAdd(&S.originated, 1ull);
                if (c.kind == K_LAT) S.lat_next = c.id + 1;
            }
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t fb = S.first_bad[kGroupLocal + K_STORM];
            uint32_t nst = S.nlocal_storm;
            if (nst) {
                uint32_t base = ncand - nst;  // storm candidates are last
                uint32_t adm = fb == 0xffffffffu ? nst : (fb > base ? fb - base : 0u);
                if (adm > nst) adm = nst;
                S.sched_next += adm;
            }
            if (S.nvote) S.progressed = 1;
        }
        // vote placement: one 16-byte write-through slot per vote, towards the parent
        {
            const uint32_t nv = S.nvemit < kMaxVoteEmit ? S.nvemit : kMaxVoteEmit;
            for (uint32_t i = tid; i < nv; i += kBlock) {
                const VoteEmit e = S.vemit[i];
                unsigned long long p = atomicAdd((unsigned long long*)&S.vout_tail[e.k], 1ull);
                if (p - S.vout_head[e.k] >= P.vote_cap) {
                    set_error(S, P, ERR_VOTE_RING, e.k);
                    continue;
                }
                u32x4 v;
                v.x = e.w0;
                v.y = e.pid;
                v.z = e.pseq;
                v.w = (uint32_t)me;
                st_sc1(rv, t.vout_data[e.k] + (uint32_t)(p & vcap_m) * kVoteSlot, v);
            }
        }

        // ---------------- G: copy admitted messages to their children
        {
            uint32_t nch = 0;
            if (admitted) nch = (kHdr + (S.cand[tid].w2 & 0xffffffu) + 15u) >> 4;
            uint32_t total;
            uint32_t ex = block_excl_scan(S, nch, &total);
            S.cum[tid] = ex;
            if (tid == kBlock - 1) S.cum[kBlock] = total;
            __syncthreads();
            for (uint32_t i = tid; i < total; i += kBlock) {
                // candidate owning chunk i: largest c with cum[c] <= i
                int lo = 0, hi = kBlock;
                while (hi - lo > 1) {
                    int mid = (lo + hi) >> 1;
                    if (S.cum[mid] <= i) lo = mid;
                    else hi = mid;
                }
                const Cand& c = S.cand[lo];
                const uint32_t q = i - S.cum[lo];
                const uint32_t len = c.w2 & 0xffffffu;
                const int origin = (int)(c.w0 & 0xffffu);
                u32x4 v;
                if (q == 0) {
                    v.x = c.w0; v.y = c.id; v.z = c.w2; v.w = c.t0;
                } else if (c.kind == K_RING) {
                    v = ld_sc1(rf, c.src + 16u * q);
                } else if (c.kind == K_STORM || c.kind == K_LAT) {
                    const uint32_t k0 = 2u * (q - 1u);
                    const int b0 = (int)len - (int)(8u * k0);
                    uint64_t a = b0 > 0 ? storm_word((uint32_t)me, c.id, k0) : 0ull;
                    uint64_t b = b0 > 8 ? storm_word((uint32_t)me, c.id, k0 + 1u) : 0ull;
                    v.x = mask_bytes((uint32_t)a, b0);
                    v.y = mask_bytes((uint32_t)(a >> 32), b0 - 4);
                    v.z = mask_bytes((uint32_t)b, b0 - 8);
                    v.w = mask_bytes((uint32_t)(b >> 32), b0 - 12);
                } else if (c.kind == K_PROP) {
                    const int64_t pi = (int64_t)c.src;
                    const uint32_t dl = P.prop_data_len[pi];
                    if (q == 1) {
                        v.x = c.id; v.y = 1u; v.z = dl; v.w = 0u;  // PBuf header (:1381-1383)
                    } else {
                        const uint8_t* d = P.prop_data + P.prop_data_off[pi];
                        uint32_t w[4];
                        for (int e = 0; e < 4; e++) {
                            uint32_t x = 0;
                            for (int bb = 0; bb < 4; bb++) {
                                uint32_t idx = 16u * (q - 2u) + 4u * e + bb;
                                if (idx < dl) x |= (uint32_t)d[idx] << (8 * bb);
                            }
                            w[e] = x;
                        }
                        v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
                    }
                } else {  // K_DEC: PBuf(pid, decision, 7, "IAR_DEC") (:908-917)
                    if (q == 1) {
                        v.x = c.id; v.y = (uint32_t)(int32_t)(int8_t)(c.w0 >> 24); v.z = 7u; v.w = 0u;
                    } else {
                        v.x = 0x5F524149u; v.y = 0x00434544u; v.z = 0u; v.w = 0u;
                    }
                }
                uint32_t kids = c.kids;
                while (kids) {
                    const int j = __builtin_ctz(kids);
                    kids &= kids - 1;
                    const int vc = t.send_list[j] < origin ? 1 : 0;
                    const int oi = 2 * j + vc;
                    const uint64_t slot = S.out_tail0[oi] + S.pos[lo][j];
                    st_sc1(rf, t.out_data[j][vc] + (uint32_t)(slot & fcap_m) * P.fwd_stride + 16u * q, v);
                }
                if (c.kind == K_RING && ((c.w0 >> 16) & 0xffu) == TAG_BCAST) {
                    acc_sum += (q == 0) ? chunk_mix(0xFFFFFFFFu, u32x4{(uint32_t)origin, c.id, TAG_BCAST, len})
                                        : chunk_mix(q - 1u, v);
                    if (q > 0 && c.logidx != ~0u && 16u * q <= P.log_stride) {
                        uint8_t* dst = P.log_payload + ((size_t)lr * P.log_cap + c.logidx) * P.log_stride + 16u * (q - 1u);
                        *reinterpret_cast<u32x4*>(dst) = v;
                    }
                }
            }
        }

        // ---------------- H: drain, publish counters, bookkeeping
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid < nout) {
            if (S.out_tail[tid] != S.out_tail0[tid]) pub64(&P.ctrl[t.out_tail[tid >> 1][tid & 1]], S.out_tail[tid]);
        } else if (tid >= 64 && tid - 64 < n_in2) {
            const int g = tid - 64;
            pub64(&P.ctrl[t.in_head[g >> 1][g & 1]], S.in_head[g]);
        } else if (tid >= 128 && tid - 128 < t.sll) {
            const int j = tid - 128;
            const uint64_t nh = S.vin_head[j] + (S.vbase[j + 1] - S.vbase[j]);
            if (nh != S.vin_head[j]) {
                S.vin_head[j] = nh;
                pub64(&P.ctrl[t.vin_head[j]], nh);
            }
        } else if (tid >= 192 && tid - 192 < t.n_in) {
            const int k = tid - 192;
            pub64(&P.ctrl[t.vout_tail[k]], S.vout_tail[k]);
        }
        if (tid == 0) {
            S.iterations++;
            const uint64_t tn = now_ticks();
            if (S.progressed || S.nvote) {
                S.busy++;
                S.last_progress = tn;
            } else if (tn - S.last_progress > P.timeout_ticks) {
                set_error(S, P, ERR_TIMEOUT, 0);
            }
            if (tn - t_start > P.deadline_ticks) set_error(S, P, ERR_TIMEOUT, 1);
            bool done = true;
            if (P.mode & MODE_STORM) done &= S.sched_next == S.sched_n;
            if (P.mode & (MODE_STORM | MODE_LAT)) done &= (int64_t)S.bcast_delivered == P.expect_bcast[lr];
            if (P.mode & MODE_LAT) {
                while (S.lat_next < P.lat_rounds && P.lat_origin[S.lat_next] != me) S.lat_next++;
                done &= S.lat_next >= P.lat_rounds;
            }
            if (P.mode & MODE_IAR)
                done &= S.own_iter == S.own_n && S.own_state == 0 && (int64_t)S.dec_delivered == P.expect_dec[lr];
            if (S.error == ERR_TIMEOUT) done = true;
            if (poll32(P.error_flag) != 0) done = true;  // another rank failed: stop everyone
            S.done = done;
        }
        __syncthreads();
        if (S.done) break;
    }

    // ---------------- flush statistics
    atomicAdd((unsigned long long*)&P.stats[lr].bcast_sum, acc_sum);
    __syncthreads();
    if (tid < kHistBins) P.stats[lr].hist[tid] = S.hist[tid];
    if (tid == 0) {
        RankStats& st = P.stats[lr];
        st.bcast_delivered = S.bcast_delivered;
        st.originated = S.originated;
        st.dec_delivered = S.dec_delivered;
        st.dec_approved = S.dec_approved;
        st.actions = S.actions;
        st.judge_calls = S.judge_calls;
        st.own_decided = S.own_decided;
        st.own_approved = S.own_approved;
        st.proposals_recv = S.proposals_recv;
        st.iterations = S.iterations;
        st.busy_iterations = S.busy;
        st.stalls = S.stalls;
        st.log_count = S.log_count;
        st.t_start = t_start;
        st.t_end = now_ticks();
        st.error = S.error;
        st.error_aux = S.error_aux;
    }
}

}  // namespace rlo

// C-ABI launch shim used by rlo_world.cpp
extern "C" hipError_t rlo_launch_progress(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream) {
    hipLaunchKernelGGL(rlo::rlo_progress_kernel, dim3(blocks), dim3(rlo::kBlock), dyn_lds, stream, *p);
    return hipGetLastError();
}

extern "C" size_t rlo_kernel_static_lds(void) { return sizeof(rlo::Shared); }

extern "C" hipError_t rlo_occupancy(int* blocks, size_t dyn_lds) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, rlo::rlo_progress_kernel, rlo::kBlock, dyn_lds);
}
