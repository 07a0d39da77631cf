// rlo_hop.hip -- the hop kernel (gfx950 / CDNA4): the latency and iar programs on ONE wave per rank.
//
// The programs that move one message at a time -- the latency program (one bcast in flight, rootless_ops.c
// testcases.c:59-108 at scale) and the iar program (proposal / vote / decision rounds with device judges,
// rootless_ops.c:668-917) -- spend their time on the HOP: a message's arrival, its checks, its forwards.  The
// progress kernel (rlo_kernel.hip) serves them with its doorbell pass, but that pass lives inside a 4 / 8-wave
// kernel built for batched storms: 200-256 VGPRs and 240-360 SGPRs spilled to VGPR lanes, so a hop's checks were
// ~800 instructions.  This kernel restates only what these programs need, in one wave, and
// handles every message the way the reference does -- one received message at a time, in per-edge FIFO order
// (make_progress_gen :551-641 surfaces one per call) -- with no batched iteration at all:
//
//   poll   : one round trip for every counter of the rank (in-ring tails, vote-in tails, out-ring heads, vote-out
//            heads), its forward and vote DOORBELLS (rlo_device.hpp), the part's error word and the latency round
//            word; an idle rank repeats it until a polled word moves
//   bells  : a whole doorbell is its ring's head message: staged in LDS, taken and forwarded first (children's
//            out-rings from a table of (in-edge, origin) pairs built at launch)
//   load   : the ring messages and votes the counters show beyond what the bells carried, one round trip
//   votes  : _iar_vote_handler :743-812 / _vote_merge :1056-1070, a completed merge votes up (_vote_back :728-741)
//   rings  : per in-ring, its messages in order: _bc_forward :1104-1225 (children relative to the dynamic origin,
//            forwarded into every child's ring and doorbell), then the delivery / proposal / decision effects
//            (:583-615, :668-726, :814-859); a message whose out-rings are full waits (the ring stops there)
//   own    : the pool's decisions (_iar_decision_bcast :908-917), then its next proposals (RLO_submit_proposal
//            :876-906), or this rank's next latency round (RLO_bcast_gen :1581-1604)
//   publish: one drain of the round's stores, then its counters (vmcnt counts loads and stores in issue order)
//
// Rings, doorbells, counters, pending tables, logs and statistics are the world's own (rlo_world.cpp builds them
// for both kernels): parts of one world may run either kernel, and every test of these programs runs this one.
// Memory ordering as in rlo_kernel.hip: every handed-off byte stored sc1 (system scope across GPUs) and loaded
// sc1 behind the counter that covers it; a counter is stored after its stores drained.  A world created with
// RLO_PART_ONE_XCD runs the LOC instantiation instead: every rank-wave on one XCD, cached rings, plain stores that
// stay in that XCD's L2 (still loaded sc1, past the CU's L1), the placement checked at launch.
#include "rlo_kernel_common.hpp"

namespace rlo {

constexpr uint32_t kHopScratch = 64u * 16u;  // one batch of 16-B chunks (64 lanes x 16 B)
constexpr uint32_t kHopLoads = 4;            // ring-message loads per lane per round trip (256 chunks)
constexpr uint32_t kPmHop = ~(uint32_t)MODE_HOST;  // log_put: no host-mode code here
constexpr uint32_t kHopSpin = 64;            // re-polls of an idle rank before a whole round runs again
constexpr uint32_t kHopNeedLds = 2048;       // (in-edge, origin) pairs of the LDS out-ring table (8 KiB)
// the diagnostics build's section profile (tools/hop_anatomy.py): shader clocks per section of a round into
// stats.prof[0..7] and event counts into stats.dbg[0..7]; the product kernel carries none of it
#ifdef RLO_DIAG
constexpr bool kHopProf = true;
#else
constexpr bool kHopProf = false;
#endif

// Per-rank state lives in registers, not LDS: every counter, the own-proposal pool, the vote-ring tails and heads
// and the topology's remote addresses are lane-distributed VGPRs (lane i holds entry i), read with v_readlane by a
// wave-uniform index and written by the one lane that owns the entry.  A round's effects run on the whole wave in
// uniform control flow (no lane-0 sections of dependent LDS read-modify-writes: DESIGN.md 4.0.2).  LDS keeps only the
// pending-proposal table (n x pend_slots entries), the slot / vote staging of a round and the rare error / log words.
struct HopShared {
    RankTopo t;
    uint32_t error, error_aux;
    unsigned long long log_count;
    uint64_t pk_tail;  // (log_put's host-mode fields: this kernel runs no host mode)
    uint32_t ev_n;
    uint32_t hist[kHistBins];
    alignas(16) uint8_t msg[kHopLoads * kHopScratch];  // loaded ring messages, message m chunk q at 16 (m mch + q)
    alignas(16) uint8_t bell[kHopScratch];   // a round's forward bells, in-edge k's chunk q at 16 (8 k + q)
    uint32_t need_lds[kHopNeedLds];          // worlds of <= kHopNeedLds (in-edge, origin) pairs: out-rings by pair
    alignas(16) uint8_t vote[kHopScratch];   // loaded votes, one 16-B slot per lane; a judged proposal's copy
};

// the counters of RankStats, one per lane of a single VGPR pair (cnt_r)
enum HopCnt : int {
    HC_BCAST = 0, HC_DEC, HC_DEC_APPR, HC_ACTIONS, HC_JUDGE, HC_ORIG, HC_OWN_DEC, HC_OWN_APPR, HC_PROP_RECV, HC_STALE,
    HC_ITER, HC_BUSY
};

// SYS: the world spans GPUs (Params.sys_scope): every hand-off store and counter at system scope -- a template
// parameter, so no store of the hop path branches on the scope at run time.  LOC (MODE_XCD1, worlds created with
// RLO_PART_ONE_XCD): the grid is 8 workgroups per rank and only every eighth runs a rank (workgroups 8 apart share an
// XCD; checked at launch), the rings are in cached memory and the hand-off stores are plain, so a line stays in that
// XCD's L2 and the consumer's sc1 load hits it (tools/xcd_probe.hip: one hop 0.51 us vs 1.11 us)
template <bool PH, bool SYS, bool LOC>
__global__ __launch_bounds__(64) void rlo_hop_kernel(Params P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    __shared__ HopShared S;
    if constexpr (LOC)
        if (blockIdx.x & 7u) return;
    const int lr = LOC ? (int)(blockIdx.x >> 3) : (int)blockIdx.x, me = P.rank_begin + lr;
    const int lane = (int)threadIdx.x;
    PendState* pend;  // [n][pend_slots]: dynamic LDS, or (PH) this rank's table in HBM
    if constexpr (PH)
        pend = (PendState*)(__attribute__((address_space(1))) PendState*)(P.pend_hbm + (size_t)lr * (uint32_t)P.n * P.pend_slots);
    else
        pend = reinterpret_cast<PendState*>(dyn_lds);
#define PEND(o, q) pend[(uint32_t)(o) * P.pend_slots + ((uint32_t)(q) & (P.pend_slots - 1u))]
    const bool lat = (P.mode & MODE_LAT) != 0, iar = (P.mode & MODE_IAR) != 0;
    const uint32_t mch = P.hop_chunks;  // 16-B chunks of the program's longest message (<= 64)

    // ---------------- init
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&P.topo[lr]);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&S.t);
        for (int i = lane; i < (int)(sizeof(RankTopo) / 4); i += 64) dst[i] = src[i];
        // (the latency program never touches the table, and is launched without one: rlo_world.cpp hop_lds)
        if (iar)
            for (int i = lane; i < P.n * (int)P.pend_slots; i += 64) pend[i] = PendState{0, 0, 0, 0, 0, 0};
        for (int i = lane; i < kHistBins; i += 64) S.hist[i] = 0;
        if (lane == 0) {
            S.error = 0; S.error_aux = 0;
            S.log_count = 0; S.pk_tail = 0; S.ev_n = 0;
        }
    }
    if constexpr (PH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the table's zeros land before any read
    __syncthreads();
    const uint64_t t_start = now_ticks();
    unsigned long long acc_sum = 0;  // checksum of delivered bcast chunks (this lane's share)
    const int64_t expect_bcast = lat ? P.expect_bcast[lr] : 0;
    const int64_t expect_dec = iar ? P.expect_dec[lr] : 0;
    const uint32_t my_mask = (iar && P.judge_kind == JUDGE_MASK) ? P.judge_mask[me] : 0u;

    // topology: wave-uniform scalars + lane-distributed lists and remote addresses
    const RankTopo& t = S.t;
    const int level = uni(t.level), last_wall = uni(t.last_wall), scc = uni(t.scc), sll = uni(t.sll);
    const int n_in = uni(t.n_in), n_in2 = 2 * n_in, nout = 2 * sll;
    const uint32_t inbox = (uint32_t)uni((int)t.inbox_ctrl), outbox = (uint32_t)uni((int)t.outbox_ctrl);
    const uint32_t in_bell = (uint32_t)uni((int)t.in_bell), vin_bell = (uint32_t)uni((int)t.vin_bell);
    const uint32_t sl_r = lane < sll ? (uint32_t)t.send_list[lane] : 0u;
    constexpr bool sys = SYS;
    // hand-off stores: system scope (SYS), plain (LOC), else agent scope (sc1)
    auto st16 = [&](__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
        if constexpr (SYS) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSc1 | 1);
        else if constexpr (LOC) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSc1);
    };
    auto st64 = [&](uint64_t addr, uint64_t v) {
        if constexpr (SYS) __hip_atomic_store(gptr64(addr), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else if constexpr (LOC) __hip_atomic_store(gptr64(addr), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else __hip_atomic_store(gptr64(addr), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    const __amdgpu_buffer_rsrc_t rf = mk_rsrc(P.fwd_region, P.fwd_region_bytes);
    const __amdgpu_buffer_rsrc_t rv = mk_rsrc(P.vote_region, P.vote_region_bytes);
    const __amdgpu_buffer_rsrc_t rc = mk_rsrc(P.ctrl, P.ctrl_bytes);
    const uint32_t fcap_m = P.fwd_cap - 1, vcap_m = P.vote_cap - 1, oring_bytes = P.fwd_cap * P.fwd_stride;
    // lane g = in-ring g (k*2 + vc), lane oi = out-ring oi (j*2 + vc), lane j = vote ring from child j, lane k = in-edge k
    // (its sender, the vote ring to it and that ring's bell)
    const uint32_t in_src_r = lane < n_in ? (uint32_t)t.in_src[lane] : 0u;
    const uint32_t in_data_r = lane < n_in2 ? t.in_data[lane >> 1][lane & 1] : 0u;
    const uint32_t vin_data_r = lane < sll ? t.vin_data[lane] : 0u;
    const uint64_t obase_r = lane < nout ? t.out_ring[lane >> 1][lane & 1] : 0ull;  // out-ring oi in the child's part
    const uint64_t bbase_r = lane < nout ? t.out_bell[lane >> 1] : 0ull;            // the child's doorbell for the edge
    const uint64_t otail_a = lane < nout ? t.out_tail[lane >> 1][lane & 1] : 0ull;   // counter words I publish
    const uint64_t ihead_a = lane < n_in2 ? t.in_head[lane >> 1][lane & 1] : 0ull;
    const uint64_t vinh_a = lane < sll ? t.vin_head[lane] : 0ull;
    const uint64_t vtail_a = lane < n_in ? t.vout_tail[lane] : 0ull;
    const uint64_t vring_r = lane < n_in ? t.vout_ring[lane] : 0ull;  // vote ring to the parent of in-edge k
    const uint64_t vbell_r = lane < n_in ? t.vout_bell[lane] : 0ull;  // and its vote bell
    // ring state and the values last published
    uint64_t in_head_r = 0, out_tail_r = 0, vin_head_r = 0, vout_tail_r = 0, vout_hd_r = 0;
    uint64_t pub_in = 0, pub_out = 0, pub_vin = 0, pub_vout = 0;
    // counters (HopCnt: lane i holds counter i)
    uint64_t cnt_r = 0;
#define CNT_ADD(i, v) (cnt_r += (lane == (i)) ? (uint64_t)(v) : 0ull)
    // own proposals, the pool (rootless_ops.c:30, :159-165, :1251-1366): lane k = slot k, named by the pseq byte
    int32_t own_pid_r = -1;
    uint32_t own_word_r = 0, own_state_r = 0, own_dec_r = 0;
    const uint32_t own_needed = (uint32_t)sll;  // votes_needed = send_list_len (:881)
    uint32_t own_rr = 0;
    int64_t own_iter = 0;
    const int64_t poff = iar ? P.prop_off[lr] : 0;
    const int64_t own_n = iar ? P.prop_off[lr + 1] - poff : 0;
    // the next own proposal, fetched while the current one is in flight (RLO_submit_proposal's arguments): stage 1 its
    // pid / data_len / data offset, stage 2 its PBuf chunks (lane q = chunk q, q >= 1), so an origination loads nothing
    // (vector loads into VGPRs, read with v_readfirstlane once landed: a scalar load would count in lgkmcnt, which
    // every LDS wait of the round also waits for -- a memory round trip inside the next LDS access)
    int64_t nx_i = -1;
    uint32_t nx_stage = 0, nx_pid_v = 0, nx_dl_v = 0, nx_doff_v = 0;
    u32x4 nx_v = {0u, 0u, 0u, 0u};
    auto vld32 = [&](const void* base, uint32_t idx) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(mk_rsrc(const_cast<void*>(base), 0xFFFFFFFFu), 4u * idx, 0, 0);
    };
    auto prefetch_meta = [&](int64_t i) {
        nx_stage = 0;
        nx_i = i;
        if (i >= own_n) return;
        nx_pid_v = vld32(P.prop_pid, (uint32_t)(poff + i));
        nx_dl_v = vld32(P.prop_data_len, (uint32_t)(poff + i));
        nx_doff_v = vld32(P.prop_data_off, (uint32_t)(poff + i));
        nx_stage = 1;
    };
    // the latency program: my originations
    uint32_t lat_pos = 0, lat_seen = 0;
    const uint32_t lat_pos_n = lat ? P.lat_own_off[lr + 1] - P.lat_own_off[lr] : 0u;
    uint32_t lat_own_next = lat_pos_n ? P.lat_own[P.lat_own_off[lr]] : 0xffffffffu;
    if (iar) prefetch_meta(0);
    // MODE_TL (diagnostics build): this round's poll issued / returned, counters published, ring loop entered
    uint32_t tl_iss = 0, tl_back = 0, tl_pub = 0, tl_loop = 0;
    uint64_t idle_since = 0;
    uint32_t idle_n = 0;
    bool done = false;
    const bool logon = (P.mode & MODE_LOG) != 0u;  // (uniform: no lane-0 section is entered for a log that is off)
    auto err = [&](uint32_t code, uint32_t aux) {
        if (lane == 0) set_error(S, P, code, aux);
    };

    // a message (lane q holds slot chunk q, q < nch) into out-rings `need` at their tails, and into each child's
    // doorbell for the edge when it fits one (tag bell_tag(ring sequence) | vc << 31).  The caller advances out_tail_r
    auto forward = [&](u32x4 v, uint32_t nch, uint32_t need) {
        const uint32_t q = (uint32_t)lane;
        for (uint32_t m = need; m; m &= m - 1) {
            const int oi = __builtin_ctz(m);
            const uint64_t slot = rdl64(out_tail_r, oi);
            const __amdgpu_buffer_rsrc_t ro = mk_rsrc(reinterpret_cast<void*>(rdl64(obase_r, oi)), oring_bytes);
            if (q < nch) st16(ro, (uint32_t)(slot & fcap_m) * P.fwd_stride + 16u * q, v);
            if (nch <= kBellChunks && q < nch) {
                const uint32_t T = bell_tag(slot) | ((uint32_t)(oi & 1) << 31);
                const __amdgpu_buffer_rsrc_t rb = mk_rsrc(reinterpret_cast<void*>(rdl64(bbase_r, oi)), kBellWords * 8u);
                st16(rb, 32u * q, u32x4{v.x, T, v.y, T});
                st16(rb, 32u * q + 16u, u32x4{v.z, T, v.w, T});
            }
        }
    };
    // out-rings of `need` that have no free slot (uniform)
    auto full_of = [&](uint32_t need, uint64_t out_head_r) -> bool {
        return __ballot(lane < nout && ((need >> lane) & 1u) && out_tail_r - out_head_r >= P.fwd_cap) != 0ull;
    };
    // a pending entry, read by every lane (one LDS / HBM broadcast) as {pid, word, parent_k | needed << 16 | valid << 24,
    // pseq}; lane 0's copy is the one used (it wrote the entry last, so program order covers its own stores)
    auto pend_rd = [&](int origin, uint32_t pseq) -> u32x4 {
        const u32x4 x = *reinterpret_cast<const u32x4*>(&PEND(origin, pseq));
        return u32x4{rdl32(x.x, 0), rdl32(x.y, 0), rdl32(x.z, 0), rdl32(x.w, 0)};
    };
    auto pend_wr = [&](int origin, uint32_t pseq, u32x4 x) {
        if (lane == 0) *reinterpret_cast<u32x4*>(&PEND(origin, pseq)) = x;
    };

    // vote up towards the parent over in-edge k (_vote_back :728-741): its vote bell {origin | pseq << 16 | vote << 24,
    // T, pid, T} (lanes 0, 1) and the 16-B slot {origin | vote << 24, pid, pseq, me} (lanes 2, 3), T = bell_tag(vote
    // sequence); global stores, agent scope (system scope when the world spans GPUs)
    auto vote_up = [&](uint32_t k, int origin, int32_t pid, uint32_t pseq, int vote) {
        const uint64_t p = rdl64(vout_tail_r, (int)k);
        if (p - rdl64(vout_hd_r, (int)k) >= P.vote_cap) {
            err(ERR_VOTE_RING, k);
            return;
        }
        if (lane == (int)k) vout_tail_r = p + 1u;
        const uint32_t T = bell_tag(p);
        uint64_t addr = 0, val = 0;
        if (lane < 2) {
            addr = rdl64(vbell_r, (int)k) + 8u * (uint32_t)lane;
            val = lane == 0 ? ((uint64_t)(((uint32_t)origin & 0xffffu) | ((pseq & 0xffu) << 16) | ((uint32_t)(vote & 0xff) << 24)) |
                               ((uint64_t)T << 32))
                            : ((uint64_t)(uint32_t)pid | ((uint64_t)T << 32));
        } else if (lane < 4) {
            addr = rdl64(vring_r, (int)k) + (uint64_t)(p & vcap_m) * kVoteSlot + 8u * (uint32_t)(lane - 2);
            val = lane == 2 ? ((uint64_t)((uint32_t)origin | ((uint32_t)(vote & 0xff) << 24)) | ((uint64_t)(uint32_t)pid << 32))
                            : ((uint64_t)(pseq & 0xffu) | ((uint64_t)(uint32_t)me << 32));
        }
        if (lane < 4) st64(addr, val);
    };

    // one vote from child j: _iar_vote_handler :743-812, _vote_merge :1056-1070 (uniform)
    auto merge_vote = [&](int origin, int32_t pid, uint32_t pseq, int vote, uint32_t vw) {
        const uint32_t inc = 1u + (vote == 0 ? 0x10000u : 0u);
        if (origin >= P.n) {
            err(ERR_BAD_SLOT, vw);
        } else if (origin == me) {  // a vote for my own proposal (:756-783)
            const uint32_t k = pseq & (P.pend_slots - 1u);
            if (rdl32(own_state_r, (int)k) != 1u || pid != (int32_t)rdl32((uint32_t)own_pid_r, (int)k)) {
                err(ERR_VOTE_ORPHAN, (uint32_t)pid);
            } else {
                const uint32_t nw = rdl32(own_word_r, (int)k) + inc;
                if (lane == (int)k) own_word_r = nw;
                if ((nw & 0xffffu) == own_needed) {
                    const uint32_t d = (nw >> 16) == 0 ? 1u : 0u;
                    if (d) {  // final judge(NULL) (:770-775): every device judge approves NULL
                        CNT_ADD(HC_JUDGE, 1);
                        if (logon && lane == 0) log_put<kPmHop>(S, P, lr, LOG_JUDGE, me, -1, (uint32_t)pid, 0, 1, 1);
                    }
                    if (lane == (int)k) { own_dec_r = d; own_state_r = 2; }
                }
            }
        } else {
            const u32x4 pe = pend_rd(origin, pseq);
            if ((pe.z >> 24) != PS_ACTIVE || (int32_t)pe.x != pid) {
                err(ERR_VOTE_ORPHAN, (uint32_t)pid);
            } else {
                const uint32_t nw = pe.y + inc;
                pend_wr(origin, pseq, u32x4{pe.x, nw, pe.z, pe.w});
                if ((nw & 0xffffu) == ((pe.z >> 16) & 0xffu))
                    vote_up(pe.z & 0xffffu, origin, pid, pseq, (nw >> 16) == 0 ? 1 : 0);
            }
        }
    };

    // one ring message from in-ring g, lane q holding slot chunk q (q < nch): checks, forwards, effects.  Returns
    // false when it cannot go now (an out-ring it needs is full, or its pending entry still holds the previous
    // proposal of that pool slot): nothing changed, the ring waits
    // worlds of <= 16 ranks with <= 4 in-edges (every one-proposal iar world this kernel runs): a forwarded message's
    // out-rings by (in-edge k, origin o) in lane 16 k + o, computed once (_bc_forward :1116-1223, fwd_send_cnt :1559-1579)
    const bool ntab = P.n <= 16 && n_in <= 4;
    uint32_t need_t = 0;
    if (ntab) {
        for (int k = 0; k < n_in; k++)
            for (int o = 0; o < P.n; o++) {
                const uint32_t nd = need_of_u(kids_of_u(me, o, (int)rdl32(in_src_r, k), level, last_wall, scc, sll, sl_r, lane), o,
                                              sll, sl_r, lane);
                if (lane == 16 * k + o) need_t = nd;
            }
    }
    // larger worlds up to kHopNeedLds pairs (256 ranks x 8 in-edges): the same table in LDS, entry n k + o, each lane
    // computing its own origins' entries (kids_of / need_of: the per-lane forms)
    const bool ltab = !ntab && (uint32_t)P.n * (uint32_t)n_in <= kHopNeedLds;
    if (ltab) {
        for (int k = 0; k < n_in; k++) {
            const int from = (int)rdl32(in_src_r, k);
            for (int o = lane; o < P.n; o += 64)
                S.need_lds[(uint32_t)k * (uint32_t)P.n + (uint32_t)o] =
                    need_of(kids_of(me, o, from, level, last_wall, scc, sll, sl_r), o, sll, sl_r);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // kHopProf: a take's clocks -- lane 0 checks (to the forward), 1 forward, 2 effects; lane 3 takes (stats.hist[124..127])
    uint64_t tk_r = 0;
    auto take = [&](u32x4 v, int g, uint64_t out_head_r) -> bool {
        const uint32_t tl_take = TL_ON(P) ? (uint32_t)now_ticks() : 0u;
        const uint64_t tk0 = kHopProf ? __builtin_amdgcn_s_memtime() : 0ull;
        uint64_t tk1 = 0, tk2 = 0;
        const uint32_t q = (uint32_t)lane;
        const int from = (int)rdl32(in_src_r, g >> 1);
        const uint32_t w0 = rdl32(v.x, 0), id = rdl32(v.y, 0), w2 = rdl32(v.z, 0), t0 = rdl32(v.w, 0);
        const int origin = (int)(w0 & 0xffffu);
        const uint32_t tag = (w0 >> 16) & 0xffu, len = w2 & 0xffffu, nch = (kHdr + len + 15u) >> 4, pseq = w2 >> 24;
        const int vote = (int)(int8_t)(w0 >> 24);
        if (((w2 >> 16) & 0xffu) != kSlotMark) {  // bytes not visible behind the published tail: a protocol violation
            CNT_ADD(HC_STALE, 1);
            err(ERR_BAD_SLOT, 0x57A1Eu);
            return true;  // consumed, never forwarded
        }
        if (origin >= P.n || nch > mch || !(tag == TAG_BCAST || tag == TAG_DECISION || tag == TAG_PROPOSAL) ||
            (tag == TAG_BCAST && lat && id >= P.lat_rounds)) {
            err(ERR_BAD_SLOT, w0);
            return true;
        }
        int judge = 1;
        u32x4 pe = {0u, 0u, 0u, 0u};
        if (tag != TAG_BCAST) pe = pend_rd(origin, pseq);
        if (tag == TAG_PROPOSAL) {
            if ((pe.z >> 24) != PS_NONE) return false;  // the decision ahead of it first
            // device judge on the PBuf data [pid][vote][data_len u64][data] at slot + 16 (:1402-1410): chunk 1's
            // word 2 is data_len, the data from chunk 2 on (LDS copy of this lane's chunk)
            uint32_t dl = rdl32(v.z, 1);
            if (dl > len - 16u) dl = len > 16u ? len - 16u : 0u;
            if (P.judge_kind == JUDGE_ISP) {
                if (q < nch) *reinterpret_cast<u32x4*>(S.vote + 16u * q) = v;  // (scratch: no vote staged now)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const uint8_t* d = S.vote + kHdr + 16u;
                judge = judge_eval_f(P, me, my_mask, (int32_t)id, [&](uint32_t i) { return d[i]; }, dl);
            } else {
                judge = judge_eval_f(P, me, my_mask, (int32_t)id, [&](uint32_t) { return (uint8_t)0; }, dl);
            }
            judge = uni(judge);
        }
        const uint64_t tka = kHopProf ? __builtin_amdgcn_s_memtime() : 0ull;
        // the out-rings of the message's children (one per child: 2 j + vc): from the table of (in-edge, origin) pairs
        // where the world is small enough to have one, else computed
        const uint32_t need = judge != 1 ? 0u
                              : ntab ? rdl32(need_t, (int)(((uint32_t)g >> 1) * 16u + (uint32_t)origin))
                              : ltab ? (uint32_t)uni((int)S.need_lds[((uint32_t)g >> 1) * (uint32_t)P.n + (uint32_t)origin])
                                     : need_of_u(kids_of_u(me, origin, from, level, last_wall, scc, sll, sl_r, lane), origin, sll,
                                                 sl_r, lane);
        if (full_of(need, out_head_r)) return false;
        if (TL_ON(P) && tag == TAG_BCAST && lane == 0) {  // the hop's clocks (tools/round_timeline.py)
            tl_put(P, id, TLC_ARRIVE, lr, tl_take);
            tl_put(P, id, TLC_ISSUE, lr, tl_iss);
            tl_put(P, id, TLC_PASS, lr, tl_back);
            tl_put(P, id, TLC_FWD, lr, tl_pub);
            tl_put(P, id, TLC_NEXT, lr, tl_loop);
            tl_put(P, id, TLC_P1, lr, (uint32_t)now_ticks());
            tl_parent(P, id, lr, from);
        }
        if constexpr (kHopProf) tk1 = __builtin_amdgcn_s_memtime();
        forward(v, nch, need);  // before the effects, as the reference forwards before queueing the pickup (:583-589)
        if constexpr (kHopProf) tk2 = __builtin_amdgcn_s_memtime();
        if (TL_ON(P) && tag == TAG_BCAST && lane == 0) tl_put(P, id, TLC_P2, lr, (uint32_t)now_ticks());
        if (lane < nout && ((need >> lane) & 1u)) out_tail_r++;
        if (tag == TAG_BCAST) {  // delivered to this rank's pickup queue (:583-589)
            CNT_ADD(HC_BCAST, 1);
            const uint32_t tn = (uint32_t)now_ticks();  // this rank's pickup
            uint32_t li = ~0u;
            if (lane == 0) {
                if (P.mode & MODE_HIST) atomicAdd(&S.hist[hist_bin(tn - t0)], 1u);
                if (P.mode & MODE_LOG) li = log_put<kPmHop>(S, P, lr, LOG_DELIVER | (TAG_BCAST << 8), origin, from, id, len, -1, tn - t0);
            }
            if (q < nch) acc_sum += q == 0 ? chunk_mix(0xFFFFFFFFu, u32x4{(uint32_t)origin, id, TAG_BCAST, len}) : chunk_mix(q - 1u, v);
            if (P.mode & MODE_LOG) {
                li = rdl32(li, 0);
                if (li != ~0u && q >= 1u && q < nch && 16u * q <= P.log_stride)
                    st_sys16(P.log_payload + ((size_t)lr * P.log_cap + li) * P.log_stride + 16u * (q - 1u), v);
            }
            if (lat && lane == 0) {  // the round's last pickup completes it
                // the round's one-way latency: origination -> the LAST receiver's pickup, each receiver's own pickup
                // clock (the reference harness's t_recv, ref_harness.c mode_lat), so the completion count's round
                // trip below is not part of it (non-returning max; lat_out is zeroed at every launch)
                __hip_atomic_fetch_max(&P.lat_out[id], (uint64_t)(tn - t0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t old = sys ? __hip_atomic_fetch_add(&P.lat_count[id], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                         : atomicAdd(&P.lat_count[id], 1u);
                if (old + 1u == (uint32_t)(P.n - 1)) {
                    tl_mark(P, id, TL_ROUND);
                    if (sys) __hip_atomic_store(P.lat_round, id + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    else __hip_atomic_store(P.lat_round, id + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (TL_ON(P) && lane == 0) tl_mark(P, id, kTlGlobal + P.n_local + (uint32_t)lr);
        } else if (tag == TAG_PROPOSAL) {  // _iar_proposal_handler :668-726
            CNT_ADD(HC_PROP_RECV, 1);
            // a received proposal carrying one of my own in-flight pids (:690-692; here every slot of the pool)
            if (__ballot((uint32_t)lane < P.pend_slots && own_state_r != 0u && own_pid_r == (int32_t)id)) {
                err(ERR_PID_COLLISION, id);
            } else {
                const uint32_t k = (uint32_t)g >> 1;
                CNT_ADD(HC_JUDGE, 1);
                if (logon && lane == 0) log_put<kPmHop>(S, P, lr, LOG_JUDGE, origin, from, id, len, judge, 0);
                if (!judge) {  // declined: vote 0, not forwarded, not pending (:700-706)
                    vote_up(k, origin, (int32_t)id, pseq, 0);
                } else {
                    const uint32_t nk = (uint32_t)__builtin_popcount(need);  // (one out-ring per child)
                    pend_wr(origin, pseq, u32x4{id, 0u, k | (nk << 16) | ((uint32_t)PS_ACTIVE << 24), pseq | ((len - 16u) << 8)});
                    if (nk == 0) vote_up(k, origin, (int32_t)id, pseq, 1);
                }
            }
        } else {  // decision: _iar_decision_handler :814-859
            if ((pe.z >> 24) == PS_ACTIVE && (int32_t)pe.x == (int32_t)id) {
                if (vote != 0) {
                    CNT_ADD(HC_ACTIONS, 1);
                    if (logon && lane == 0) log_put<kPmHop>(S, P, lr, LOG_ACTION, origin, from, id, 0, 1, pe.w >> 8);
                }
                pend_wr(origin, pseq, u32x4{pe.x, pe.y, pe.z & 0x00ffffffu, pe.w});  // valid = PS_NONE
            }
            CNT_ADD(HC_DEC, 1);
            if (vote != 0) CNT_ADD(HC_DEC_APPR, 1);
            if (logon && lane == 0) log_put<kPmHop>(S, P, lr, LOG_DELIVER | (TAG_DECISION << 8), origin, from, id, 7, vote, 0);
        }
        if constexpr (kHopProf) {
            const uint64_t tk3 = __builtin_amdgcn_s_memtime();
            tk_r += lane == 0 ? tk1 - tk0 : lane == 1 ? tk2 - tk1 : lane == 2 ? tk3 - tk2 : lane == 3 ? 1ull : lane == 4 ? tka - tk0 : 0ull;
        }
        return true;
    };

    // a local origination to the whole send list (:1587): header + chunks (v: lane q's chunk q >= 1, generated or
    // prefetched); false (nothing changed) when an out-ring is full
    const uint32_t need_all = need_of_u((1u << sll) - 1u, me, sll, sl_r, lane);  // an origination's out-rings (:1587)
    auto originate = [&](uint32_t w0, uint32_t id, uint32_t w2, u32x4 v, uint64_t out_head_r) -> bool {
        const uint32_t len = w2 & 0xffffu, nch = (kHdr + len + 15u) >> 4;
        const uint32_t need = need_all;
        if (full_of(need, out_head_r)) return false;
        if (lane == 0) v = u32x4{w0, id, (w2 & 0xff00ffffu) | (kSlotMark << 16), (uint32_t)now_ticks()};
        forward(v, nch, need);
        if (lane < nout && ((need >> lane) & 1u)) out_tail_r++;
        return true;
    };

    // what the last poll saw (lane-distributed, as the counters): an idle rank re-polls until one of them moves
    uint64_t snap_in = 0, snap_vin = 0, snap_out = 0;
    uint32_t snap_lat = 0;
    bool idle_prev = false, room_wait = false;
    // kHopProf: clocks per section (0 poll + spin, 1 bells, 2 publish, 3 loads, 4 votes, 5 loaded messages,
    // 6 originations, 7 bookkeeping) and counts (0 rounds, 1 re-polls, 2 bell takes, 3 slot takes, 4 votes merged,
    // 5 refusals, 6 originations, 7 busy rounds)
    // (lane i: clocks of section i, lane 8 + i: count i -- one VGPR pair, as cnt_r)
    uint64_t hp_r = 0;
    uint64_t hpt = kHopProf ? __builtin_amdgcn_s_memtime() : 0;
#define HP_MARK(i)                                            \
    do {                                                      \
        if constexpr (kHopProf) {                             \
            const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
            hp_r += lane == (i) ? t_ - hpt : 0ull;            \
            hpt = t_;                                         \
        }                                                     \
    } while (0)
#define HP_CNT(i, v)                                                       \
    do {                                                                   \
        if constexpr (kHopProf) hp_r += lane == 8 + (i) ? (uint64_t)(v) : 0ull; \
    } while (0)
    // RLO_PART_ONE_XCD (LOC): every rank-wave must sit on the first one's XCD (HIP does not promise the round-robin
    // placement the grid relies on).  A rendezvous on uncached words before any hand-off -- [0] the first XCC id + 1,
    // [1] arrivals | a misplaced wave's 1 << 16, one atomic each -- and a wave elsewhere stops the whole launch with
    // RLO_DERR_XCD instead of handing messages through another XCD's L2
    bool xcd_ok = true;
    if constexpr (LOC) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const uint32_t mine = (xcc & 0xFu) + 1u;
        uint32_t first = 0, bad = 0;
        if (lane == 0) {
            first = atomicCAS(P.xcd_word, 0u, mine);
            const uint32_t off = first != 0u && first != mine ? 0x10001u : 1u;
            atomicAdd(P.xcd_word + 1, off);
            uint32_t v = 0;
            for (uint32_t s = 0; s < (1u << 22); s++) {  // bounded: every rank-wave is co-resident (hop_eligible)
                v = __hip_atomic_load(P.xcd_word + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((v & 0xFFFFu) >= P.n_local) break;
            }
            bad = (v >> 16) != 0u || (v & 0xFFFFu) < P.n_local;
        }
        if (rdl32(bad, 0) != 0u) {
            err(ERR_XCD, (rdl32(first, 0) << 8) | mine);
            xcd_ok = false;
        }
    }
    while (xcd_ok) {
        // ---------------- poll: counters, doorbells, error word, round word -- one round trip
        // (branch-free: rlo_kernel_common.hpp kOob).  After a round that did nothing the poll repeats right away, with
        // no round around it, until a polled word moves: a message landing at an idle rank waits for at most one poll
        // period of one round trip, not of a whole round (bounded, so the idle clock and the deadline still tick)
        const uint32_t bk = (uint32_t)lane >> 3, bq = (uint32_t)lane & 7u;
        const bool inb = (int)bk < n_in;
        const uint32_t bo = inb ? (in_bell + bk * kBellWords) * 8u + 32u * bq : kOob;
        uint64_t in_tail_r, vin_tail_r, out_head_r, vout_head_r;
        uint32_t errf, latr;
        u32x4 ba, bb, vb;
        // the tags that make in-edge k's bell whole for its ring heads (vc 0 / vc 1), and child j's vote bell
        const uint32_t e0 = bell_tag((uint32_t)__shfl((int)(uint32_t)in_head_r, (int)(2u * bk)));
        const uint32_t e1 = bell_tag((uint32_t)__shfl((int)(uint32_t)in_head_r, (int)(2u * bk + 1u))) | 0x80000000u;
        const uint32_t ve = bell_tag(vin_head_r);
        for (uint32_t sp = 0;; sp++) {
            if (TL_ON(P)) tl_iss = (uint32_t)now_ticks();
            in_tail_r = ld64_sc1(rc, lane < n_in2 ? (inbox + (uint32_t)lane) * 8u : kOob);
            vin_tail_r = ld64_sc1(rc, lane < sll ? (inbox + (uint32_t)(n_in2 + lane)) * 8u : kOob);
            out_head_r = ld64_sc1(rc, lane < nout ? (outbox + (uint32_t)lane) * 8u : kOob);
            vout_head_r = ld64_sc1(rc, lane < n_in ? (outbox + (uint32_t)(nout + lane)) * 8u : kOob);
            errf = ld32_sc1(rc, 0u);  // (the part's error word is its ctrl word 0)
            ba = ld_sc1(rc, bo);
            bb = ld_sc1(rc, bo == kOob ? kOob : bo + 16u);
            vb = ld_sc1(rc, lane < sll ? (vin_bell + 2u * (uint32_t)lane) * 8u : kOob);
            // the latency round word (part 0's when sharded; system scope covers both)
            latr = __hip_atomic_load(lat ? P.lat_round : P.error_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler (also the previous round's stores)
            if (TL_ON(P)) tl_back = (uint32_t)now_ticks();
            if (!idle_prev || sp >= kHopSpin) break;
            HP_CNT(1, 1);
            // new work: a bell's first half tagged for a ring head or a vote head (the round checks it is whole), a
            // counter beyond what was taken that moved since the last round, freed out-ring slots when something waits
            // for room, the round word when it concerns this rank, an error
            const bool moved = (inb && bq == 0u && (ba.y == e0 || ba.y == e1)) || (lane < sll && vb.y == ve) ||
                               (lane < n_in2 && in_tail_r > in_head_r && in_tail_r != snap_in) ||
                               (lane < sll && vin_tail_r > vin_head_r && vin_tail_r != snap_vin) ||
                               (room_wait && lane < nout && out_head_r != snap_out) ||
                               (latr != snap_lat && (me == 0 || latr == lat_own_next)) || errf != 0u;
            if (__ballot(moved)) break;
        }
        snap_in = in_tail_r; snap_vin = vin_tail_r; snap_out = out_head_r; snap_lat = latr;
        CNT_ADD(HC_ITER, 1);
        HP_MARK(0);
        HP_CNT(0, 1);
        vout_hd_r = vout_head_r;
        bool progressed = false;
        room_wait = false;
        const bool go = !done && __builtin_amdgcn_readfirstlane(errf) == 0;

        // ---------------- whole doorbells first (forward-first): in-edge k's bell holds ring (k, vc)'s head when every
        // 8-byte half of its header's chunks carries bell_tag(in-ring head) | vc << 31.  That message is taken from the
        // bells (one 16-B LDS read per lane after one write of the round's bells), forwarded before this rank merges or
        // loads anything -- the reference forwards on receipt too (_bc_forward from make_progress_gen :583-589)
        uint64_t blocked = 0;  // rings whose head cannot go this round (full out-ring, pending entry busy): they wait
        // lane (k, q): its chunk's tag when all four halves agree; the header lanes (q = 0) that carry a head's tag
        const uint32_t tg = ba.y == ba.w && ba.y == bb.y && ba.y == bb.w ? ba.y : 0u;
        const uint64_t hc = __ballot(inb && bq == 0u && tg != 0u && (tg == e0 || tg == e1));
        if (go && hc) {
            if (TL_ON(P)) tl_pub = tl_loop = (uint32_t)now_ticks();
            *reinterpret_cast<u32x4*>(S.bell + 16u * (uint32_t)lane) = u32x4{ba.x, ba.z, bb.x, bb.z};
            for (uint64_t cs = hc; cs; cs &= cs - 1) {  // (uniform; in-edge order)
                const int hl = __builtin_ctzll(cs);
                const uint32_t th = rdl32(tg, hl);
                const int g = 2 * (hl >> 3) + (int)(th >> 31);  // (vc 1 tags carry bit 31)
                const uint32_t nch = (kHdr + (rdl32(bb.x, hl) & 0xffffu) + 15u) >> 4;
                if (nch > kBellChunks) continue;
                const uint64_t m = ((1ull << nch) - 1ull) << hl;
                if ((__ballot(tg == th) & m) != m) continue;  // not whole yet: the counter path takes it
                u32x4 v = {0u, 0u, 0u, 0u};
                if ((uint32_t)lane < nch) v = *reinterpret_cast<const u32x4*>(S.bell + 16u * ((uint32_t)hl + (uint32_t)lane));
                if (take(v, g, out_head_r)) {
                    if (lane == g) in_head_r++;
                    progressed = true;
                    HP_CNT(2, 1);
                } else {
                    blocked |= 1ull << g;
                    room_wait = true;
                    HP_CNT(5, 1);
                }
            }
        }
        HP_MARK(1);

        // (every counter of the previous rounds is out: each round publishes its own at its end)
        if (done) break;
        if (!go) break;   // another rank failed: stop everyone
        if (lat && me == 0 && latr > lat_seen) {  // world rank 0 observes round completions on its own clock
            const uint64_t tn = now_ticks();
            for (uint32_t k = lat_seen + (uint32_t)lane; k < latr && k < P.lat_rounds; k += 64u) P.lat_obs[k] = tn;
            lat_seen = latr;
        }
        // the next own proposal's chunks, now that its pid / length / offset are in (stage 1 -> 2)
        if (nx_stage == 1u) {
            const uint32_t nx_dl = (uint32_t)uni((int)nx_dl_v), nx_doff = (uint32_t)uni((int)nx_doff_v);
            const uint32_t nch = (kHdr + 16u + nx_dl + 15u) >> 4;
            nx_v = u32x4{0u, 0u, 0u, 0u};
            if (lane == 1) nx_v = u32x4{(uint32_t)uni((int)nx_pid_v), 1u, nx_dl, 0u};  // PBuf [pid][vote=1][data_len u64] (:1369-1396)
            if ((nx_doff & 3u) == 0u) {
                // dword-aligned data (the usual packing): 16-B loads, left in flight -- the bytes past data_len are
                // masked off at the origination (the range of the resource ends at the data's end, rounded up)
                const __amdgpu_buffer_rsrc_t rd = mk_rsrc(const_cast<uint8_t*>(P.prop_data) + nx_doff, (nx_dl + 3u) & ~3u);
                if (lane >= 2 && (uint32_t)lane < nch) nx_v = __builtin_amdgcn_raw_buffer_load_b128(rd, 16u * ((uint32_t)lane - 2u), 0, 0);
            } else if (lane >= 2 && (uint32_t)lane < nch) {
                const __attribute__((address_space(1))) uint8_t* d =
                    (const __attribute__((address_space(1))) uint8_t*)(P.prop_data + nx_doff);
                uint32_t w[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    uint32_t x = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        const uint32_t idx = 16u * ((uint32_t)lane - 2u) + 4u * e + b;
                        if (idx < nx_dl) x |= (uint32_t)d[idx] << (8 * b);
                    }
                    w[e] = x;
                }
                nx_v = u32x4{w[0], w[1], w[2], w[3]};
            }
            nx_stage = 2;
        }
        HP_MARK(2);

        // ---- the messages the counters show beyond what was taken (ring g: from its head, unless the head waits),
        // and the vote slots beyond child j's vote bell
        const uint64_t ip = lane < n_in2 && !((blocked >> lane) & 1ull) && in_tail_r > in_head_r ? in_tail_r - in_head_r : 0ull;
        const uint32_t vbh = lane < sll && vb.y == ve && vb.w == ve ? 1u : 0u;
        const uint64_t vp = lane < sll && vin_tail_r > vin_head_r ? vin_tail_r - vin_head_r : 0ull;

        // ---- load them: ring messages (lane (m, q): chunk q of the m-th message to load) and votes (one slot per
        // lane), one round trip
        const uint32_t mmax = min(kHopLoads * 64u / mch, 64u);
        uint32_t mtot = 0;
        const uint32_t want = (uint32_t)min(ip, (uint64_t)mmax);
        const uint32_t mb = wave_excl_scan(want, &mtot);
        const uint32_t mtake = mb >= mmax ? 0u : min(want, mmax - mb);  // lane g: slot messages loaded this round
        const uint32_t mload = min(mtot, mmax);
        uint32_t vtot = 0;
        const uint32_t vwant = (uint32_t)min(vp > vbh ? vp - vbh : 0ull, (uint64_t)64);
        const uint32_t vbase = wave_excl_scan(vwant, &vtot);
        const uint32_t vtake = vbase >= 64u ? 0u : min(vwant, 64u - vbase);  // lane j: vote slots loaded
        if (mtot | vtot) {
            u32x4 lm[kHopLoads], lw;
#pragma unroll
            for (uint32_t u = 0; u < kHopLoads; u++) {  // item u 64 + lane = (message m, chunk qq)
                lm[u] = u32x4{0u, 0u, 0u, 0u};
                if (u * 64u >= mload * mch) continue;  // (uniform)
                const uint32_t i = u * 64u + (uint32_t)lane, m = i / mch, qq = i - m * mch;
                uint32_t src = 0;
                bool any = false;
                for (uint64_t gs = __ballot(mtake > 0u); gs; gs &= gs - 1) {  // uniform loop over rings with loads
                    const int g = __builtin_ctzll(gs);
                    const uint32_t b0 = rdl32(mb, g), n0 = rdl32(mtake, g);
                    if (m >= b0 && m < b0 + n0) {
                        const uint64_t seq = rdl64(in_head_r, g) + (m - b0);
                        src = rdl32(in_data_r, g) + (uint32_t)(seq & fcap_m) * P.fwd_stride + 16u * qq;
                        any = true;
                    }
                }
                lm[u] = ld_sc1(rf, any ? src : kOob);  // (branch-free: rlo_kernel_common.hpp kOob)
            }
            {
                bool any = false;
                uint32_t src = 0;
                for (uint64_t js = __ballot(vtake > 0u); js; js &= js - 1) {
                    const int j = __builtin_ctzll(js);
                    const uint32_t b0 = rdl32(vbase, j), n0 = rdl32(vtake, j);
                    if ((uint32_t)lane >= b0 && (uint32_t)lane < b0 + n0) {
                        const uint64_t seq = rdl64(vin_head_r, j) + rdl32(vbh, j) + ((uint32_t)lane - b0);
                        src = rdl32(vin_data_r, j) + (uint32_t)(seq & vcap_m) * kVoteSlot;
                        any = true;
                    }
                }
                lw = ld_sc1(rv, any ? src : kOob);
            }
#pragma unroll
            for (uint32_t u = 0; u < kHopLoads; u++)
                if (u * 64u < mload * mch) *reinterpret_cast<u32x4*>(S.msg + 16u * (u * 64u + (uint32_t)lane)) = lm[u];
            *reinterpret_cast<u32x4*>(S.vote + 16u * (uint32_t)lane) = lw;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        HP_MARK(3);

        // ---------------- votes: child j's head from its bell, then its loaded slots, in order (uniform)
        for (uint64_t js = __ballot(vbh || vtake); js; js &= js - 1) {
            const int j = __builtin_ctzll(js);
            const uint32_t hb = rdl32(vbh, j), nv = rdl32(vtake, j), b0 = rdl32(vbase, j);
            if (hb) {  // vote bell {origin | pseq << 16 | vote << 24, pid}
                const uint32_t x = rdl32(vb.x, j), pid = rdl32(vb.z, j);
                merge_vote((int)(x & 0xffffu), (int32_t)pid, (x >> 16) & 0xffu, (int)(int8_t)(x >> 24), x);
            }
            for (uint32_t i = 0; i < nv; i++) {  // vote slot {origin | vote << 24, pid, pseq, voter}
                const u32x4 vs = *reinterpret_cast<const u32x4*>(S.vote + 16u * (b0 + i));
                const uint32_t x = uni((int)vs.x), pid = uni((int)vs.y), ps = uni((int)vs.z);
                merge_vote((int)(x & 0xffffu), (int32_t)pid, ps & 0xffu, (int)(int8_t)(x >> 24), x);
            }
            if (lane == j) vin_head_r += hb + nv;
            progressed = true;
            HP_CNT(4, hb + nv);
        }
        HP_MARK(4);

        // ---------------- loaded ring messages: per in-ring, in order from its head
        for (uint64_t gs = __ballot(mtake > 0u); gs; gs &= gs - 1) {
            const int g = __builtin_ctzll(gs);
            const uint32_t nm = rdl32(mtake, g), b0 = rdl32(mb, g);
            uint32_t taken = 0;
            for (uint32_t i = 0; i < nm; i++) {  // uniform
                u32x4 v = {0u, 0u, 0u, 0u};
                if ((uint32_t)lane < mch) v = *reinterpret_cast<const u32x4*>(S.msg + 16u * ((b0 + i) * mch) + 16u * (uint32_t)lane);
                if (!take(v, g, out_head_r)) {
                    room_wait = true;
                    HP_CNT(5, 1);
                    break;
                }
                taken++;
            }
            if (lane == g) in_head_r += taken;
            if (taken) progressed = true;
            HP_CNT(3, taken);
        }
        HP_MARK(5);

        // ---------------- my own originations
        if (iar) {
            for (;;) {  // the pool's decided slots (_iar_decision_bcast :908-917)
                const uint64_t dm = __ballot((uint32_t)lane < P.pend_slots && own_state_r == 2u);
                if (!dm) break;
                const int k = __builtin_ctzll(dm);
                const uint32_t id = rdl32((uint32_t)own_pid_r, k), dec = rdl32(own_dec_r, k);
                u32x4 v = {0u, 0u, 0u, 0u};  // PBuf(pid, decision, 7, "IAR_DEC") (:908-917)
                if (lane == 1) v = u32x4{id, dec, 7u, 0u};
                if (lane == 2) v = u32x4{0x5F524149u, 0x00434544u, 0u, 0u};
                if (!originate((uint32_t)me | (TAG_DECISION << 16) | ((dec & 0xffu) << 24), id, 23u | ((uint32_t)k << 24), v,
                               out_head_r)) {
                    room_wait = true;
                    break;
                }
                HP_CNT(6, 1);
                CNT_ADD(HC_OWN_DEC, 1);
                if (dec) CNT_ADD(HC_OWN_APPR, 1);
                if (logon && lane == 0) log_put<kPmHop>(S, P, lr, LOG_RESULT, me, -1, id, 0, (int)dec, (uint32_t)k);
                if (lane == k) { own_state_r = 0; own_pid_r = -1; }  // proposalPool_rm (:1334-1347) / RLO_proposal_reset (:1649-1673)
                progressed = true;
            }
            for (;;) {  // RLO_submit_proposal :876-906, up to own_pool in flight
                const uint64_t busy = __ballot((uint32_t)lane < P.pend_slots && own_state_r != 0u);
                if (own_iter >= own_n || (uint32_t)__popcll(busy) >= P.own_pool) break;
                uint32_t k = own_rr;
                while ((busy >> k) & 1ull) k = (k + 1u) & (P.pend_slots - 1u);
                uint32_t id, dl;
                u32x4 pv = {0u, 0u, 0u, 0u};
                if (nx_i != own_iter || nx_stage != 2u) {  // (not prefetched yet: fetch it now, one wait)
                    const int64_t pi = poff + own_iter;
                    id = (uint32_t)P.prop_pid[pi];
                    dl = P.prop_data_len[pi];
                    const uint32_t nch = (kHdr + 16u + dl + 15u) >> 4;
                    if (lane == 1) pv = u32x4{id, 1u, dl, 0u};
                    else if (lane >= 2 && (uint32_t)lane < nch)
                        pv = gen_chunk(P, K_PROP, me, id, 16u + dl, (uint32_t)pi, 1, (uint32_t)lane);
                } else {
                    id = (uint32_t)uni((int)nx_pid_v);
                    dl = (uint32_t)uni((int)nx_dl_v);
                    pv = nx_v;
                    if (lane >= 2) {  // the data's zero-padded tail (loaded whole dwords)
                        const int b0 = (int)dl - (int)(16u * ((uint32_t)lane - 2u));
                        pv = u32x4{mask_bytes(pv.x, b0), mask_bytes(pv.y, b0 - 4), mask_bytes(pv.z, b0 - 8), mask_bytes(pv.w, b0 - 12)};
                    }
                }
                if (!originate((uint32_t)me | (TAG_PROPOSAL << 16) | (1u << 24), id, (16u + dl) | (k << 24), pv,
                               out_head_r)) {
                    room_wait = true;
                    break;
                }
                HP_CNT(6, 1);
                // proposalPool_proposal_add (:1253-1279)
                if (lane == (int)k) { own_pid_r = (int32_t)id; own_word_r = 0; own_state_r = 1; }
                own_iter++;
                own_rr = (k + 1u) & (P.pend_slots - 1u);
                prefetch_meta(own_iter);  // the next one's arguments, in flight until the next round
                progressed = true;
            }
        }
        if (lat && lat_own_next != 0xffffffffu && latr == lat_own_next) {
            u32x4 v = {0u, 0u, 0u, 0u};
            if (lane >= 1 && (uint32_t)lane < ((kHdr + P.len + 15u) >> 4))
                v = gen_chunk(P, K_LAT, me, lat_own_next, P.len, 0u, -1, (uint32_t)lane);
            if (!originate((uint32_t)me | (TAG_BCAST << 16) | (0xffu << 24), lat_own_next, P.len, v, out_head_r)) {
                room_wait = true;
            } else {
                HP_CNT(6, 1);
                if (lane == 0) tl_mark(P, lat_own_next, TL_ORIGIN);
                CNT_ADD(HC_ORIG, 1);
                lat_pos++;
                lat_own_next = lat_pos < lat_pos_n ? P.lat_own[P.lat_own_off[lr] + lat_pos] : 0xffffffffu;
                progressed = true;
            }
        }
        // ---------------- this round's counters, published now behind one drain of its stores -- not after the next
        // poll: a message the bells did not carry is visible to its consumer a round earlier (C4 at 8 ranks 168 K -> 175 K
        // decisions/s, profiles/r6_hop_eager_ab.txt); the poll's wait then covers its loads only
        if (__ballot((lane < nout && out_tail_r != pub_out) || (lane < n_in2 && in_head_r != pub_in) ||
                     (lane < sll && vin_head_r != pub_vin) || (lane < n_in && vout_tail_r != pub_vout))) {
            VM_DRAIN();
            if (lane < nout && out_tail_r != pub_out) { pub_out = out_tail_r; st64(otail_a, out_tail_r); }
            if (lane < n_in2 && in_head_r != pub_in) { pub_in = in_head_r; st64(ihead_a, in_head_r); }
            if (lane < sll && vin_head_r != pub_vin) { pub_vin = vin_head_r; st64(vinh_a, vin_head_r); }
            if (lane < n_in && vout_tail_r != pub_vout) { pub_vout = vout_tail_r; st64(vtail_a, vout_tail_r); }
        }
        HP_MARK(6);

        // ---------------- bookkeeping (uniform)
        if (progressed) {
            CNT_ADD(HC_BUSY, 1);
            idle_n = 0;
        } else if ((++idle_n & 63u) == 1u) {  // the clock on the 1st and every 64th idle round only
            const uint64_t tn = now_ticks();
            if (idle_n == 1) idle_since = tn;
            else if (tn - idle_since > P.timeout_ticks) err(ERR_TIMEOUT, 0);
        }
        const uint64_t n_iter = rdl64(cnt_r, HC_ITER);
        if ((n_iter & 1023u) == 0 && now_ticks() - t_start > P.deadline_ticks) err(ERR_TIMEOUT, 1);
        bool d = true;
        if (lat) d &= lat_pos >= lat_pos_n && (int64_t)rdl64(cnt_r, HC_BCAST) == expect_bcast;
        if (iar)
            d &= own_iter == own_n && __ballot((uint32_t)lane < P.pend_slots && own_state_r != 0u) == 0ull &&
                 (int64_t)rdl64(cnt_r, HC_DEC) == expect_dec;
        if (uni((int)S.error) == (int)ERR_TIMEOUT) d = true;
        done = d;
        idle_prev = !progressed && !done;
        HP_CNT(7, progressed ? 1 : 0);
        HP_MARK(7);
        // (done: one more poll round publishes this round's counters behind its drain, then the loop ends)
    }
#undef PEND

    // ---------------- statistics
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    atomicAdd((unsigned long long*)&P.stats[lr].bcast_sum, acc_sum);
    for (int i = lane; i < kHistBins; i += 64) P.stats[lr].hist[i] = S.hist[i];
    if (kHopProf && lane < 5) P.stats[lr].hist[lane < 4 ? kHistBins - 4 + lane : kHistBins - 5] = (uint32_t)min(tk_r, (uint64_t)0xffffffffu);
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (lane == i) { P.stats[lr].prof[i] = hp_r; P.stats[lr].dbg[i] = rdl64(hp_r, 8 + i); }
#undef HP_MARK
#undef HP_CNT
    uint64_t cv[12];
#pragma unroll
    for (int i = 0; i < 12; i++) cv[i] = rdl64(cnt_r, i);
    if (lane == 0) {
        RankStats& st = P.stats[lr];
        st.bcast_delivered = cv[HC_BCAST];
        st.originated = cv[HC_ORIG];
        st.dec_delivered = cv[HC_DEC];
        st.dec_approved = cv[HC_DEC_APPR];
        st.actions = cv[HC_ACTIONS];
        st.judge_calls = cv[HC_JUDGE];
        st.own_decided = cv[HC_OWN_DEC];
        st.own_approved = cv[HC_OWN_APPR];
        st.proposals_recv = cv[HC_PROP_RECV];
        st.iterations = cv[HC_ITER];
        st.busy_iterations = cv[HC_BUSY];
        st.stalls = 0;
        st.unmarked_slots = cv[HC_STALE];
        st.log_count = S.log_count;
        st.t_start = t_start;
        st.t_end = now_ticks();
        st.error = S.error;
        st.error_aux = S.error_aux;
    }
#undef CNT_ADD
}

}  // namespace rlo

// C-ABI launch shims (rlo_world.cpp): one 64-thread workgroup per local rank, the pending table in dynamic LDS
// (dyn_lds bytes) or, with Params.pend_hbm, in HBM (the PH instantiation); system-scope worlds run the SYS one
template <bool PH, bool SYS, bool LOC = false>
static hipError_t hop_grant(size_t dyn_lds) {
    static size_t granted = 0;
    if (dyn_lds > granted) {
        hipError_t e = hipFuncSetAttribute((const void*)rlo::rlo_hop_kernel<PH, SYS, LOC>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn_lds);
        if (e != hipSuccess) return e;
        granted = dyn_lds;
    }
    return hipSuccess;
}
template <bool PH, bool SYS, bool LOC = false>
static hipError_t hop_launch(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream) {
    hipError_t e = hop_grant<PH, SYS, LOC>(dyn_lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((rlo::rlo_hop_kernel<PH, SYS, LOC>), dim3(LOC ? 8 * blocks : blocks), dim3(64), dyn_lds, stream, *p);
    return hipGetLastError();
}
template <bool PH, bool SYS>
static hipError_t hop_occ(int* blocks, size_t dyn_lds) {
    hipError_t e = hop_grant<PH, SYS>(dyn_lds);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, rlo::rlo_hop_kernel<PH, SYS, false>, 64, dyn_lds);
}

extern "C" hipError_t rlo_launch_hop(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream) {
    const bool ph = p->pend_hbm != nullptr, sys = p->sys_scope != 0;
    if ((p->mode & rlo::MODE_XCD1) && (sys || !p->xcd_word)) return hipErrorInvalidValue;  // (the rendezvous word)
    if (p->mode & rlo::MODE_XCD1)  // RLO_PART_ONE_XCD
        return ph ? hop_launch<true, false, true>(p, blocks, dyn_lds, stream) : hop_launch<false, false, true>(p, blocks, dyn_lds, stream);
    return ph ? (sys ? hop_launch<true, true>(p, blocks, dyn_lds, stream) : hop_launch<true, false>(p, blocks, dyn_lds, stream))
              : (sys ? hop_launch<false, true>(p, blocks, dyn_lds, stream) : hop_launch<false, false>(p, blocks, dyn_lds, stream));
}

// the smaller of the two scope instantiations' answers (the world's scope is known only at launch)
extern "C" hipError_t rlo_occupancy_hop(int* blocks, size_t dyn_lds, int ph) {
    int a = 0, b = 0;
    hipError_t e = ph ? hop_occ<true, false>(&a, dyn_lds) : hop_occ<false, false>(&a, dyn_lds);
    if (e != hipSuccess) return e;
    e = ph ? hop_occ<true, true>(&b, dyn_lds) : hop_occ<false, true>(&b, dyn_lds);
    if (e != hipSuccess) return e;
    *blocks = a < b ? a : b;
    return hipSuccess;
}
