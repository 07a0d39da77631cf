// rlo_kernel.hip -- the persistent progress kernel (gfx950 / CDNA4).
//
// One 4-wave (256-thread) workgroup = one virtual rank.  A progress iteration is the
// device restatement of make_progress_gen (rootless_ops.c:551-641), batched: up to 256
// messages, wave w owning messages [64w, 64w + 64):
//
//   A  poll     : wave 0 loads the packed inbox tails / outbox heads (replaces MPI_Test of the
//                 single ANY_SOURCE irecv, :643-650); every wave drains its own stores
//   C  select   : wave 0 publishes the previous iteration's counters, then takes fair per-ring
//                 quotas of the in-ring backlog (FIFO per ring) and the local originations
//                 (RLO_bcast_gen :1581, own proposal :876, decision :908)
//   B  votes    : wave 1 loads every vote slot that arrived and AND-merges them with LDS
//                 atomics (_iar_vote_handler :743-812); completed merges vote up (:728-741)
//   D  stage    : each wave pulls its messages' slots into LDS with LDS-DMA, coalesced
//                 (consecutive messages of an in-ring are consecutive slots), ONE round trip;
//                 skip-ring children relative to the dynamic origin (_bc_forward :1104-1225),
//                 device judge for proposals (:698)
//   E  admit    : per out-ring positions from wave ballots + cross-wave prefixes in LDS; credit
//                 check; FIFO prefix per source (head-of-line order of a ring); every admitted
//                 message gets its slot index in each out-ring it goes to (olist)
//   F  effects  : deliveries (pickup), proposal state, decisions + actions (:814-859)
//   G  copy     : per out-ring, the admitted messages occupy consecutive slots: lanes take
//                 (message, chunk) items so every store writes contiguous slot bytes; large
//                 messages are staged first (loads before stores: vmcnt is in-order on CDNA)
//
// Inside the workgroup synchronisation is s_barrier + LDS waits (BAR), never a vmcnt drain:
// payload stores stay in flight until the next iteration's poll has been issued.
// Memory ordering across ranks (MI355X_MICROARCH.md "Valid forms", row 1): every handed-off
// byte is stored sc1 and loaded sc1; each storing wave drains vmcnt(0) before the barrier
// that precedes the counter store.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rlo_kernel_common.hpp"

namespace rlo {

struct CandL {          // one message of this iteration, kept for the copy phase
    uint32_t w0, id, w2, t0;  // slot header (forwarded unchanged)
    uint32_t src;       // K_RING: slot byte offset in the forward region; K_PROP: proposal index
    uint32_t need;      // admitted out-ring bits (2j + vc); 0 when not admitted
    uint32_t logidx;    // log record of this delivery (payload capture) or ~0u
    uint32_t kind, group;
    uint32_t relay;     // pull worlds: byte offset of this message's slot in my relay ring, ~0u = none
};

// bulk-message state (the BULK instantiation only)
// a job post decided by one lane (phase C / F), queued in LDS and written out by all of wave 0 at a
// converged point (flush_posts): one lane writing a 4-MiB message's 256 sub-job records alone took
// ~60 us -- longer than moving the bytes
struct PostReq {
    uint32_t cls, kind, origin, lr, slot, bid, len, ntiles, from, logidx, q, gen;
    uint64_t j0;
};
constexpr uint32_t kPostQ = 16;
struct BulkSh {
    PostReq pq[kPostQ];         // progress: queued job posts
    uint32_t npost;
    BulkJob mv_job;             // mover: the job of the claimed tile
    uint32_t mv_ti, mv_stop;
    unsigned long long mv_sum;
    uint32_t bq[kPass];         // progress: storm candidate i -> bulk sequence, ~0u = a ring message
    uint32_t blen[kPass];       // storm candidate i -> payload length
    uint32_t bact[kMaxPend];    // pending receptions (o * B + s), compact
    uint32_t nbact, ncomp;
    uint64_t fbase, dbase;      // progress: my flag lines (o, s) at fbase + (o B + s) kBulkLine, my done words
                                // (s) at dbase + s kBulkLine -- no part-table loads on the poll path
    // pending entries [0, nstable): the ones the last evaluation (bulk_eval, wave 0) covered, the range phase
    // C may deliver from.  Other waves append only in phase F; wave 0 evaluates after the consume phase's
    // barrier (every append of the iteration landed) and before the next phase F, so it sees whole entries
    uint32_t nstable;
    uint64_t cmask[kMaxPend / 64];  // completion bits by position in bact (phase A poll)
    uint32_t bonw[kMaxPend / 32];   // live receptions by (o * B + s): a guard (register twice / complete
                                    // one that is not live = a device error, never a lost reception)
    uint64_t sdone[8];          // done(me, s), s < B
    uint32_t bulk_q;            // my bulk originations so far
};
struct NoBulkSh {};
struct BulkPend {               // dynamic LDS [N * B]: a pending bulk reception of (o, s)
    uint32_t bid, len, ntiles;
    int32_t from;
    uint32_t t0, q, pad0, pad1;
};

// W waves per rank-workgroup (rlo_device.hpp kBlock documents the 4-wave form): 64 W candidate
// messages per iteration.  8 waves (512 candidates, two waves per SIMD) when every rank has a CU
// of its own; 4 waves when two rank-workgroups share a CU (worlds larger than the GPU)
template <int W, bool BULK>
struct Shared {
    typename std::conditional<BULK, BulkSh, NoBulkSh>::type b;
    static constexpr int kWaves = W, kMaxCand = 64 * W;
    RankTopo t;
    // selection of this iteration (wave 0)
    uint64_t ring_head[2 * kMaxIn];  // consumer count of in-ring g at iteration start
    uint32_t ring_base[2 * kMaxIn], ring_take[2 * kMaxIn];
    uint64_t ract;                   // in-rings with candidates
    uint64_t out_tail0[kMaxOut];     // producer count of out-ring oi at iteration start
    uint32_t ofree[kMaxOut];         // free slots of out-ring oi at iteration start
    uint32_t n_oi[kMaxOut];          // slots admitted into out-ring oi this iteration
    uint32_t R, C, nstorm, storm_base, loc_kind, lat_id, exit_now;
    // host-service mode: command run selected this iteration, pickup ring position
    uint32_t hbase, nh, ev_n, quit, gap_lo, gap_hi, nchmax;
    uint64_t hhead, hin_head, pk_tail;
    int64_t prop_idx;
    uint32_t storm_ids[kPass];
    uint64_t vhead[kMaxFanout];
    uint32_t vbase[kMaxFanout], va[kMaxFanout], vtot;
    // admission
    uint32_t wcnt[kWaves][kMaxOut];
    uint32_t first_bad[kGroups];
    CandL cand[kMaxCand];
    alignas(16) uint16_t pos[kMaxCand][kMaxFanout];  // admitted message c: its slot in out-ring (j, vc) - out_tail0
    uint16_t big[kMaxCand];              // admitted messages too large for the stage path
    uint32_t nbig, bm, bq0, nblk;
    uint32_t blk_c[128], blk_q0[128];    // large-message blocks staged in stage2 (two halves when pipelined)
    uint32_t nblk2[2];                   // blocks planned into each half
    // vote rings towards my parents (LDS atomics from every wave)
    uint64_t vout_tail[kMaxIn], vout_head[kMaxIn];
    // wave 0: last published counter per lane (in-ring heads, out-ring tails, vote-in heads, vote-out
    // tails) and the last poll per lane (in tails, vote-in tails, out heads, vote-out heads)
    uint64_t pubw[4][64], snap[4][64];
    // own proposals: the proposal pool (PROPOSAL_POOL_SIZE 16, rootless_ops.c:30, :159-165,
    // :1251-1366; my_own_proposal :241 when the pool depth is 1).  Slot k is named by the pseq byte
    // of the proposal, its votes and its decision; state 0 free, 1 voting, 2 decided (decision to
    // originate), 3 waiting for the host's final judge(NULL)
    int32_t own_pid[kPoolMax];
    uint32_t own_word[kPoolMax], own_state[kPoolMax], own_decision[kPoolMax];
    uint32_t own_needed, own_rr;
    unsigned long long own_iter;
    int64_t own_n;
    // local IAR originations of this iteration: candidates [R, R + loc_nd) decisions, then
    // [R + loc_nd, R + loc_n) proposals (prop_idx + i), each with its pool slot
    uint32_t loc_nd, loc_n;
    uint8_t loc_slot[2 * kPoolMax];
    // origination progress
    uint32_t lat_pos, lat_pos_n, lat_own_next, lat_seen, error, error_aux, progressed;
    uint32_t hwait;  // host mode: judge verdicts the host owes this rank (its command ring is polled every spin then)
    // host mode with command doorbells: wave 1 polls the host (PCIe) while wave 0 spins on the rings --
    // the command tail / pickup head it saw last, and the phase-A round wave 0 finished (wave 1 stops)
    uint64_t hp[2];
    uint32_t a_done, cseq;
    uint64_t hd[8], hd_t0;  // MODE_HDIAG counters (host mode)
    // pull worlds: my relay ring (slots taken / released), this iteration's allocations, and the release
    // records: relay count rq_relay[e] is released once every out-ring's consumer passed rq_out[e][oi]
    uint64_t relay_tail, relay_rel;
    uint32_t relay_n, ref_any, rq_n, rq_h, relay_free;
    uint64_t rq_relay[kRelQ];
    uint64_t rq_out[kRelQ][kMaxOut];
    // counters
    unsigned long long bcast_delivered, dec_delivered, dec_approved, actions, judge_calls, originated;
    unsigned long long own_decided, own_approved, proposals_recv, log_count, stalls, stale;
    uint64_t prof[8], prof_t, dbg[8];
    uint64_t hpt[9];     // MODE_HOPPROF: shader clocks at the points of the current doorbell hop
    uint32_t tl_clk[4];  // MODE_TL: when wave 0's spin issued its polls, when the doorbell pass began, its probes
    uint32_t tl_bfid;    // MODE_TL: a bulk announcement the doorbell pass took (+1), for its TLC_NEXT clock
    int64_t expect_dec;
    uint32_t hist[kHistBins];
};


// ------------------------------------------------------------------ bulk messages (rlo_device.hpp)

// a bulk index out of range: report (device error ERR_BULK, aux = site << 24 | value) and stop,
// instead of touching memory that is not the heap's.  Always on in the bulk instantiation: a wild
// peer-memory store can take down every GPU of the node, a report costs a few compares
__device__ __forceinline__ void bulk_fault(const Params& P, uint32_t site, uint32_t v) {
    // this part stops (its workgroups poll the word); the other parts of a sharded world then stop at
    // their no-progress timeout
    uint32_t* pe = P.error_flag;
    if (atomicCAS(pe, 0u, (uint32_t)ERR_BULK) == 0u) pe[1] = (site << 24) | (v & 0xffffffu);  // ctrl word 0, high half
}
#define BULK_GUARD(cond, site, v)                       \
    do {                                                \
        if (__builtin_expect(!(cond), 0)) bulk_fault(P, (site), (uint32_t)(v)); \
    } while (0)
// (r, o, s) in range: else a report and the sink line (jctl's spare words), never a wild address
__device__ __forceinline__ bool bulk_ok(const Params& P, int r, int o, uint32_t s, uint32_t site) {
    const bool ok = (uint32_t)r < (uint32_t)P.n && (uint32_t)o < (uint32_t)P.n && s < P.bulk_slots;
    if (!ok) bulk_fault(P, site, ((uint32_t)r << 12) | ((uint32_t)o & 0xfffu));
    return ok;
}

// the part tables (written by the host before launch, read-only in the kernel) through the constant address
// space: uniform indices then load with s_load (lgkmcnt), not with vector loads, whose vmcnt wait would also
// wait for every store in flight -- inside the movers' copy loops that was a full drain per destination
template <class T>
__device__ __forceinline__ T ldc(const T* p, int i) {
    return ((const __attribute__((address_space(4))) T*)(uintptr_t)p)[i];
}
// heap slot (r, o, s), its flag line and the origin's done word, in whichever part holds r / o
__device__ __forceinline__ uint8_t* bulk_heap(const Params& P, int r, int o, uint32_t s) {
    if (!bulk_ok(P, r, o, s, 1)) return nullptr;  // a null rsrc base: every access is dropped
    const int p = ldc(P.part_of, r);
    const uint64_t lr = (uint64_t)(r - ldc(P.part_begin, p));
    return reinterpret_cast<uint8_t*>(ldc(P.bheap, p)) + ((lr * (uint64_t)P.n + (uint64_t)o) * P.bulk_slots + s) * P.bulk_cap;
}
// heap slot (r, o, s) as a buffer resource in SGPRs -- the address is uniform, but it is computed from
// loaded table words, and a VGPR resource makes the compiler wrap every access in a waterfall loop --
// cut to bytes [off, off + bytes) of that slot: accesses past the end are dropped by the hardware's
// range check (loads return zeros), which is what lets the copy loops below run without per-granule guards
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bulk_rsrc_at(const Params& P, int r, int o, uint32_t s, uint32_t off,
                                                              uint32_t bytes) {
    return mk_rsrc(reinterpret_cast<void*>(uni64(reinterpret_cast<uint64_t>(bulk_heap(P, r, o, s)) + off)),
                   (uint32_t)uni((int)bytes));
}
__device__ __forceinline__ uint32_t* bulk_flags(const Params& P, int r, int o, uint32_t s) {
    if (!bulk_ok(P, r, o, s, 2)) return reinterpret_cast<uint32_t*>(P.jctl + kJctlSink);
    const int p = P.part_of[r];
    const uint64_t lr = (uint64_t)(r - P.part_begin[p]);
    return reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(P.bflag[p]) +
                                       ((lr * (uint64_t)P.n + (uint64_t)o) * P.bulk_slots + s) * kBulkLine);
}
__device__ __forceinline__ uint64_t* bulk_done(const Params& P, int o, uint32_t s) {
    if (!bulk_ok(P, o, o, s, 3)) return P.jctl + kJctlSink;
    const int p = P.part_of[o];
    const uint64_t lr = (uint64_t)(o - P.part_begin[p]), nlp = (uint64_t)(P.part_begin[p + 1] - P.part_begin[p]);
    return reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(P.bflag[p]) +
                                       (nlp * (uint64_t)P.n * P.bulk_slots + lr * P.bulk_slots + s) * kBulkLine);
}
// (flag words through global pointers: a generic access counts in lgkmcnt too, so the next LDS wait of the wave
// waited for it to reach memory)
__device__ __forceinline__ uint32_t bflag_ld(uint32_t* p, bool sys) {
    gu32* g = (gu32*)p;
    return sys ? __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
               : __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void bflag_add(uint32_t* p, uint32_t v, bool sys) {
    gu32* g = (gu32*)p;
    if (sys) __hip_atomic_fetch_add(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_fetch_add(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a receiver's completion count (tiles landed in its copy).  Direct plans (one GPU) keep it in 16 shards
// -- the line's words 0..15, which only the scatter -> gather hand-off of chunked plans uses -- each mover
// adding to shard (mover & 15): hundreds of movers adding to ONE word of uncached memory serialise on it
// (a 4-MiB message's 256 tiles x 7 receivers); chunked plans count in word kBulkTflag
__device__ __forceinline__ uint32_t bulk_tcount(const Params& P, uint32_t* f, bool sys) {
    if (P.bulk_cross) return bflag_ld(f + kBulkTflag, sys);
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = bflag_ld(f + i, sys);
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) t += v[i];
    return t;
}
// release / acquire around the bulk flags (the proven form of the first bulk kernel: a fence on
// both sides, MI355X_MICROARCH.md "Valid forms" first bullet; explicit vmcnt after the release,
// "Compiler hazard")
__device__ __forceinline__ void bulk_release(bool sys) {
    if (sys) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void bulk_acquire(bool sys) {
    if (sys) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// clear the flags of (r, o, s) and count r's completion at the origin (slot s may be reused once
// every receiver did this): RLO_user_msg_recycle of a bulk delivery (rootless_ops.c:981-992)
__device__ __forceinline__ void bulk_slot_release(const Params& P, int r, int o, uint32_t s, bool sys,
                                                  uint32_t want = 0u, uint32_t bid = 0u) {
    atomicAdd((unsigned long long*)&P.jctl[kJctlReleases], 1ull);  // diagnostics: releases
    uint32_t* f = bulk_flags(P, r, o, s);
    if (want) {  // the reception must be complete here: a release mid-reception would lose it
        const uint32_t tf = bulk_tcount(P, f, sys);
        if (tf < want && atomicCAS((unsigned long long*)&P.jctl[kJctlFault], 0ull,
                                   (0xEEull << 56) | ((uint64_t)(r & 0xff) << 48) | ((uint64_t)(o & 0xff) << 40) |
                                       ((uint64_t)(s & 0xf) << 36) | ((uint64_t)(bid & 0xfff) << 24) | ((tf & 0xfffu) << 12) |
                                       (want & 0xfffu)) == 0ull)
            bulk_fault(P, 13, ((uint32_t)r << 12) | ((uint32_t)o & 0xfffu));
    }
    for (int i = 0; i <= (int)kBulkTflag; i++) __hip_atomic_store((gu32*)f + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bulk_release(sys);
    gu64* d = gptr64(reinterpret_cast<uint64_t>(bulk_done(P, o, s)));
    if (sys) __hip_atomic_fetch_add(d, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_fetch_add(d, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// post a job (one lane) as nsub <= kMaxSub sub-jobs of consecutive tiles: their indices j0 .. j0 +
// nsub - 1 in one fetch-add; a slot takes sub-job j once its generation word reads j / J (the ring
// holds every sub-job that can be unfinished at once -- rlo_world.cpp sizes it -- so that is at once;
// the wait is a guard).  The bodies land first, then, after one drain, the words with the sequence,
// which a mover's ticket waits for.  BulkJob's words are passed as scalars (a struct whose address
// is taken would live in scratch).
__device__ __forceinline__ void post_job(const Params& P, uint32_t cls, uint32_t kind, int origin, int lr, uint32_t slot_s,
                                         uint32_t bid, uint32_t len, uint32_t ntiles, int from, uint32_t logidx,
                                         uint32_t q, uint32_t gen) {
    if (!(kind >= JOB_SCATTER && kind <= JOB_VERIFY && (uint32_t)origin < (uint32_t)P.n && (uint32_t)lr < P.n_local &&
          slot_s < P.bulk_slots && len > 0 && len <= P.bulk_cap && ntiles > 0)) {
        bulk_fault(P, 6, (kind << 20) | (len & 0xfffffu));
        return;
    }
    const uint32_t per = (ntiles + max_sub(kind) - 1u) / max_sub(kind), nsub = (ntiles + per - 1u) / per;
    const uint64_t j0 = atomicAdd((unsigned long long*)&P.jctl[cls * 16 + kJctlPost], (unsigned long long)nsub);
    atomicAdd((unsigned long long*)&P.jctl[kJctlPostsByKind + kind], 1ull);  // diagnostics: posts by kind (41..43)
    const uint32_t jm = P.jslots - 1u, lg = (uint32_t)__builtin_ctz(P.jslots);
    const uint64_t t0 = now_ticks();
    // the slots' generation words 16 at a time, loads issued together (one round trip per 16 sub-jobs;
    // a dependent load per sub-job made a 1-MiB scatter's 70 sub-jobs cost ~70 round trips)
    uint64_t* const jf = P.jfree + (size_t)cls * P.jslots;
    for (uint32_t u0 = 0; u0 < nsub; u0 += 16u) {
        uint64_t g[16];
#pragma unroll
        for (uint32_t i = 0; i < 16u; i++) {
            const uint64_t j = j0 + min(u0 + i, nsub - 1u);  // (past the end: the last one again)
            g[i] = __hip_atomic_load(&jf[(uint32_t)(j & jm)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (uint32_t i = 0; i < 16u; i++) {
            const uint64_t j = j0 + min(u0 + i, nsub - 1u);
            while (g[i] != (j >> lg)) {
                __builtin_amdgcn_s_sleep(1);
                if (now_ticks() - t0 > P.timeout_ticks) {  // cannot happen unless a mover died: stop loudly
                    atomicCAS(P.error_flag, 0u, (uint32_t)ERR_TIMEOUT);
                    return;
                }
                g[i] = __hip_atomic_load(&jf[(uint32_t)(j & jm)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    const uint32_t parent = (uint32_t)(j0 & jm);
    for (uint32_t u = 0; u < nsub; u++) {
        u32x4* dst = reinterpret_cast<u32x4*>(P.jobs + (size_t)cls * P.jslots + (uint32_t)((j0 + u) & jm));
        const uint32_t a = u * per, nt = min(per, ntiles - a);
        // everything but the 8 bytes holding the sequence (st_sys16 is two 8-B stores, which may
        // land in either order: the sequence half goes last, after the drain)
        __hip_atomic_store(reinterpret_cast<uint64_t*>(dst) + 1, (uint64_t)(uint32_t)origin | ((uint64_t)(uint32_t)lr << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st_sys16(dst + 1, u32x4{slot_s, bid, len, nt});
        st_sys16(dst + 2, u32x4{a, parent, (uint32_t)from, logidx});
        st_sys16(dst + 3, u32x4{q, gen, ntiles, (uint32_t)j0});
    }
    VM_DRAIN();
    for (uint32_t u = 0; u < nsub; u++) {
        uint64_t* dst = reinterpret_cast<uint64_t*>(P.jobs + (size_t)cls * P.jslots + (uint32_t)((j0 + u) & jm));
        __hip_atomic_store(dst, (uint64_t)(uint32_t)(j0 + u + 1u) | ((uint64_t)kind << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// queue a post (any lane, divergent); a full queue posts it from this lane alone
__device__ __forceinline__ void queue_job(BulkSh& B, const Params& P, uint32_t cls, uint32_t kind, int origin, int lr,
                                          uint32_t slot_s, uint32_t bid, uint32_t len, uint32_t ntiles, int from,
                                          uint32_t logidx, uint32_t q, uint32_t gen) {
    const uint32_t i = atomicAdd(&B.npost, 1u);
    if (i >= kPostQ) {
        post_job(P, cls, kind, origin, lr, slot_s, bid, len, ntiles, from, logidx, q, gen);
        return;
    }
    PostReq& r = B.pq[i];
    r.cls = cls; r.kind = kind; r.origin = (uint32_t)origin; r.lr = (uint32_t)lr; r.slot = slot_s; r.bid = bid;
    r.len = len; r.ntiles = ntiles; r.from = (uint32_t)from; r.logidx = logidx; r.q = q; r.gen = gen;
}
__device__ __forceinline__ void queue_job(NoBulkSh&, const Params&, uint32_t, uint32_t, int, int, uint32_t, uint32_t,
                                          uint32_t, uint32_t, int, uint32_t, uint32_t, uint32_t) {}  // (no bulk messages)
// registered bulk receptions (wave-uniform)
__device__ __forceinline__ uint32_t nact_of(const BulkSh& B) { return (uint32_t)uni((int)B.nbact); }
__device__ __forceinline__ uint32_t nact_of(const NoBulkSh&) { return 0u; }
// write out the queued posts (wave 0, all lanes): post_job's protocol with sub-job u on lane u mod 64 --
// the slots' generation checks, the record bodies, one drain, then the sequence words
__device__ __forceinline__ void flush_posts(BulkSh& B, const Params& P, int lane) {
    const uint32_t np = min((uint32_t)uni((int)B.npost), kPostQ);
    if (!np) return;
    const uint32_t jm = P.jslots - 1u, lg = (uint32_t)__builtin_ctz(P.jslots);
    const uint64_t t0 = now_ticks();
    for (uint32_t i = 0; i < np; i++) {
        const PostReq& r = B.pq[i];
        const uint32_t cls = (uint32_t)uni((int)r.cls), kind = (uint32_t)uni((int)r.kind), lr = (uint32_t)uni((int)r.lr);
        const uint32_t origin = (uint32_t)uni((int)r.origin), slot_s = (uint32_t)uni((int)r.slot), len = (uint32_t)uni((int)r.len);
        const uint32_t ntiles = (uint32_t)uni((int)r.ntiles);
        if (!(kind >= JOB_SCATTER && kind <= JOB_VERIFY && cls <= JCLS_B && origin < (uint32_t)P.n && lr < P.n_local &&
              slot_s < P.bulk_slots && len > 0 && len <= P.bulk_cap && ntiles > 0)) {
            if (lane == 0) {
                bulk_fault(P, 6, (kind << 20) | (len & 0xfffffu));
                B.pq[i].ntiles = 0u;  // skipped below
            }
            continue;
        }
        const uint32_t per = (ntiles + max_sub(kind) - 1u) / max_sub(kind), nsub = (ntiles + per - 1u) / per;
        uint64_t j0 = 0;
        if (lane == 0) {
            j0 = atomicAdd((unsigned long long*)&P.jctl[cls * 16 + kJctlPost], (unsigned long long)nsub);
            atomicAdd((unsigned long long*)&P.jctl[kJctlPostsByKind + kind], 1ull);  // diagnostics: posts by kind
            B.pq[i].j0 = j0;
        }
        j0 = rdl64(j0, 0);
        uint64_t* const jf = P.jfree + (size_t)cls * P.jslots;
        const __amdgpu_buffer_rsrc_t rj = mk_rsrc(reinterpret_cast<void*>(P.jobs + (size_t)cls * P.jslots), P.jslots * (uint32_t)sizeof(BulkJob));
        const uint32_t parent = (uint32_t)(j0 & jm);
        for (uint32_t u = (uint32_t)lane; u < nsub; u += 64u) {
            const uint64_t j = j0 + u;
            bool ok = true;
            while (__hip_atomic_load(&jf[(uint32_t)(j & jm)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (j >> lg)) {
                __builtin_amdgcn_s_sleep(1);
                if (now_ticks() - t0 > P.timeout_ticks) {  // cannot happen unless a mover died: stop loudly
                    atomicCAS(P.error_flag, 0u, (uint32_t)ERR_TIMEOUT);
                    ok = false;
                    break;
                }
            }
            if (!ok) break;
            u32x4* dst = reinterpret_cast<u32x4*>(P.jobs + (size_t)cls * P.jslots + (uint32_t)(j & jm));
            const uint32_t a = u * per, nt = min(per, ntiles - a);
            // the body: one 8-B store and three 16-B sc1 stores (the job ring is part-local uncached memory,
            // read by this part's movers only); the 8 bytes holding the sequence go last, after the drain
            __hip_atomic_store(reinterpret_cast<uint64_t*>(dst) + 1, (uint64_t)origin | ((uint64_t)lr << 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t jo = (uint32_t)(j & jm) * (uint32_t)sizeof(BulkJob);
            st_sc1(rj, jo + 16u, u32x4{slot_s, (uint32_t)uni((int)r.bid), len, nt});
            st_sc1(rj, jo + 32u, u32x4{a, parent, (uint32_t)uni((int)r.from), (uint32_t)uni((int)r.logidx)});
            st_sc1(rj, jo + 48u, u32x4{(uint32_t)uni((int)r.q), (uint32_t)uni((int)r.gen), ntiles, (uint32_t)j0});
        }
    }
    VM_DRAIN();
    for (uint32_t i = 0; i < np; i++) {
        const PostReq& r = B.pq[i];
        const uint32_t ntiles = (uint32_t)uni((int)r.ntiles);
        if (!ntiles) continue;
        const uint32_t cls = (uint32_t)uni((int)r.cls), kind = (uint32_t)uni((int)r.kind);
        const uint32_t per = (ntiles + max_sub(kind) - 1u) / max_sub(kind), nsub = (ntiles + per - 1u) / per;
        const uint64_t j0 = uni64(r.j0);
        for (uint32_t u = (uint32_t)lane; u < nsub; u += 64u) {
            uint64_t* dst = reinterpret_cast<uint64_t*>(P.jobs + (size_t)cls * P.jslots + (uint32_t)((j0 + u) & jm));
            __hip_atomic_store(dst, (uint64_t)(uint32_t)(j0 + u + 1u) | ((uint64_t)kind << 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (kind == JOB_SCATTER && lane == 0) tl_mark(P, (uint32_t)uni((int)r.bid), TL_POSTED);
    }
    if (lane == 0) B.npost = 0u;
}

// One tile of the movers' copy: granules [0, ngr) of src into ndst destinations (dst(j): the j-th one's
// resource, cut to the tile like src).  No branch per granule: with one, the compiler could not count the
// stores in flight and put a vmcnt(0) before EVERY store, so each 16-B-per-lane store waited for the
// previous one's write acknowledgement (a mover moved ~5 GB/s).  The next batch's loads are issued before
// this batch's stores: vmcnt retires in issue order, so waiting for those loads never waits for the stores.
template <bool SYS, int W, class F>
__device__ __forceinline__ void tile_copy(__amdgpu_buffer_rsrc_t rs, uint32_t ngr, int tid, int ndst, F dst) {
    constexpr int kT = 64 * W, D = kMoveDepth;
    constexpr uint32_t step = (uint32_t)D * kT;
    u32x4 a[D], b[D];
    auto load = [&](u32x4 (&v)[D], uint32_t g0) {
#pragma unroll
        for (int u = 0; u < D; u++) {
            const uint32_t off = 16u * (g0 + (uint32_t)(u * kT + tid));
            v[u] = SYS ? ld_sys(rs, off) : ld_sc1(rs, off);
        }
    };
    auto store = [&](const u32x4 (&v)[D], uint32_t g0) {
        for (int j = 0; j < ndst; j++) {
            const __amdgpu_buffer_rsrc_t rd = dst(j);
#pragma unroll
            for (int u = 0; u < D; u++) st_ring(rd, 16u * (g0 + (uint32_t)(u * kT + tid)), v[u], SYS);
        }
    };
    // ping-pong, no register copies; a prefetch past the tile reads zeros (range check) and is not stored
    load(a, 0u);
    for (uint32_t g0 = 0; g0 < ngr; g0 += 2u * step) {
        load(b, g0 + step);
        store(a, g0);
        if (g0 + step >= ngr) break;
        load(a, g0 + 2u * step);
        store(b, g0 + step);
    }
}

// storm payload bytes [off, off + 16) of bcast (origin, bid, len) (off a multiple of 16)
__device__ __forceinline__ u32x4 storm_granule(uint32_t origin, uint32_t bid, uint32_t len, uint32_t off) {
    const int b0 = (int)len - (int)off;
    const uint32_t k0 = off >> 3;
    const uint64_t a = b0 > 0 ? storm_word(origin, bid, k0) : 0ull;
    const uint64_t b = b0 > 8 ? storm_word(origin, bid, k0 + 1u) : 0ull;
    return u32x4{mask_bytes((uint32_t)a, b0), mask_bytes((uint32_t)(a >> 32), b0 - 4), mask_bytes((uint32_t)b, b0 - 8),
                 mask_bytes((uint32_t)(b >> 32), b0 - 12)};
}

// A mover workgroup: draws sub-jobs of its class by ticket (one fetch-add, never retried: the
// claim rate no longer serialises on one word), waits for the ticket's record, and moves every tile
// of it.  A slot is freed as soon as its record is read, except a VERIFY job's first slot, whose
// jdone / jsum accumulate the job until its last sub-job finished.  Exits once every progress
// workgroup of the part has exited and no sub-job was posted for its ticket.
template <int W, class SH>
__device__ __forceinline__ void mover_run(const Params& P, SH& SS, int tid) {
    BulkSh& S = SS.b;
    constexpr int kT = 64 * W;
    const uint32_t mi = blockIdx.x - P.n_local;
    // chunked plans: class A the SCATTER and VERIFY jobs, class B the GATHERs (which wait), half the movers each.
    // Direct plans (one GPU) post no GATHERs: every mover serves class A, VERIFYs in FIFO order with the scatters.
    // (VERIFYs on a dedicated share of the movers -- 4, 7, 10 sixteenths -- cut a 64-MiB round to 160-214 us but
    // left the verifications behind: 278-609 us of kernel per round against 267 us all in one class)
    const uint32_t na = (P.nmov + 1u) / 2u;
    const uint32_t cls = (P.bulk_cross == 0u || mi < na) ? JCLS_A : JCLS_B;
    const bool sys = P.sys_scope != 0;
    const int n = P.n;
    const uint32_t jm = P.jslots - 1u, lg = (uint32_t)__builtin_ctz(P.jslots);
    uint64_t* posted = &P.jctl[cls * 16 + kJctlPost];
    uint64_t* ticket = &P.jctl[cls * 16 + kJctlClaim];
    BulkJob* ring = P.jobs + (size_t)cls * P.jslots;
    uint64_t acq_key = ~0ull;  // (job, chunk) the last acquire covered
    const uint64_t t_launch = now_ticks();
    for (;;) {
        // ---- draw a sub-job
        if (tid == 0) {
            uint32_t stop = 0, spins = 0;
            const uint64_t j = atomicAdd((unsigned long long*)ticket, 1ull);
            const uint32_t slot = (uint32_t)(j & jm);
            const u32x4* js = reinterpret_cast<const u32x4*>(&ring[slot]);
            u32x4 v0 = __builtin_nontemporal_load(js);
            while (v0.x != (uint32_t)(j + 1u)) {
                // not posted (yet): every progress workgroup exited after its last post and the posts
                // stop short of this ticket -> nothing more will come
                if (__hip_atomic_load(&P.jctl[kJctlExited], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= P.n_local &&
                    __hip_atomic_load(posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= j) {
                    stop = 1;
                    break;
                }
                if (poll32(P.error_flag)) { stop = 1; break; }
                __builtin_amdgcn_s_sleep(2);
                if ((++spins & 1023u) == 0 && now_ticks() - t_launch > P.deadline_ticks) {
                    atomicCAS(P.error_flag, 0u, (uint32_t)ERR_TIMEOUT);
                    stop = 1;
                    break;
                }
                v0 = __builtin_nontemporal_load(js);
            }
            if (!stop) {
                u32x4 jv[4];
#pragma unroll
                for (int q = 0; q < 4; q++) jv[q] = __builtin_nontemporal_load(js + q);  // re-read behind the sequence
                if (jv[0].x != (uint32_t)(j + 1u)) bulk_fault(P, 5, (uint32_t)j);
                u32x4* jd = reinterpret_cast<u32x4*>(&S.mv_job);
#pragma unroll
                for (int q = 0; q < 4; q++) jd[q] = jv[q];
                S.mv_ti = slot;
                if (!(jv[0].y == JOB_VERIFY && jv[2].y == slot)) {  // read: the slot takes sub-job j + J
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&P.jfree[cls * P.jslots + slot], (j >> lg) + 1ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            S.mv_stop = stop;
        }
        BAR();
        if (S.mv_stop) return;
        // the sub-job, made wave-uniform explicitly: read from LDS it lives in VGPRs, and every heap
        // address derived from it would be a VGPR buffer resource -- the compiler then wraps EACH load and
        // store of the copy loops in a readfirstlane waterfall loop (the movers ran at ~5 GB/s each)
        BulkJob jb;
        {
            const u32x4* js = reinterpret_cast<const u32x4*>(&S.mv_job);
            u32x4 q[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const u32x4 v = js[i];
                q[i] = u32x4{(uint32_t)uni((int)v.x), (uint32_t)uni((int)v.y), (uint32_t)uni((int)v.z), (uint32_t)uni((int)v.w)};
            }
            __builtin_memcpy(&jb, q, sizeof jb);
        }
        if (!(jb.kind >= JOB_SCATTER && jb.kind <= JOB_VERIFY && (uint32_t)jb.origin < (uint32_t)n &&
              (uint32_t)jb.lr < P.n_local && jb.slot < P.bulk_slots && jb.len > 0 && jb.len <= P.bulk_cap &&
              jb.ntiles > 0 && jb.ti0 + jb.ntiles <= jb.total && jb.parent <= jm)) {
            if (tid == 0) bulk_fault(P, 4, (jb.kind << 20) | (jb.seq & 0xfffffu));
            return;
        }
        const uint32_t len = jb.len, s = jb.slot;
        const int o = jb.origin;
        const int me = P.rank_begin + jb.lr;
        if (tid == 0 && jb.kind == JOB_SCATTER && jb.ti0 == 0u) tl_mark(P, jb.bid, TL_CLAIMED);
        const BulkPlan pl = bulk_plan(n, len, P.bulk_cross != 0);
        if (jb.kind == JOB_SCATTER && pl.direct) {
            // one GPU (direct plan): the sub-job's tiles are one contiguous range of the message -- moved as
            // one (a fan-out from the origin's copy into every receiver's), then ONE add of its tile count to
            // this mover's shard of every receiver's completion count
            const uint32_t off0 = jb.ti0 * pl.tile;
            const uint32_t ngr = (min(jb.ntiles * pl.tile, len - off0) + 15u) >> 4;
            const __amdgpu_buffer_rsrc_t rs = bulk_rsrc_at(P, o, o, s, off0, 16u * ngr);
            if (!jb.gen) {  // a device program's origination: its bytes into the origin's copy first (see below)
                for (uint32_t g0 = 0; g0 < ngr; g0 += (uint32_t)kMoveDepth * kT) {
#pragma unroll
                    for (int uu = 0; uu < kMoveDepth; uu++) {
                        const uint32_t g = g0 + (uint32_t)uu * kT + (uint32_t)tid;
                        st_ring(rs, 16u * g, storm_granule((uint32_t)o, jb.bid, len, off0 + 16u * g), sys);
                    }
                }
            }
            if (tid == 0 && jb.ti0 == 0u) tl_mark(P, jb.bid, TL_GEN);
            auto recv = [&](int jj) { return bulk_rsrc_at(P, (o + 1 + jj) % n, o, s, off0, 16u * ngr); };
            if (sys) tile_copy<true, W>(rs, ngr, tid, n - 1, recv);
            else tile_copy<false, W>(rs, ngr, tid, n - 1, recv);
#ifdef RLO_DIAG
            if ((P.mode & MODE_CORRUPT) && jb.ti0 == 0u && tid == 0) {  // (the test that VERIFY's check fires)
                VM_DRAIN();
                st_ring(recv(0), 16u, u32x4{0u, 0u, 0u, 0u}, sys);
            }
#endif
            VM_DRAIN();
            __syncthreads();
            if (tid == 0 && jb.ti0 == 0u) tl_mark(P, jb.bid, TL_DRAINED);
            if (tid < 64) {
                if (sys) bulk_release(true);
                for (int d = 1 + tid; d < n; d += 64) bflag_add(bulk_flags(P, (o + d) % n, o, s) + (mi & 15u), jb.ntiles, sys);
                if (tid == 0) tl_mark(P, jb.bid, TL_MOVED);
            }
        } else
        for (uint32_t ti = jb.ti0; ti < jb.ti0 + jb.ntiles; ti++) {
            if (jb.kind == JOB_SCATTER || jb.kind == JOB_GATHER) {
                // tile -> (chunk c, stripe k, tile i of that stripe-chunk)
                uint32_t u = ti, c = 0, k = 0, i = 0;
                if (jb.kind == JOB_SCATTER) {
                    for (c = 0; c + 1 < pl.nchunks; c++) {
                        const uint32_t ct = bulk_chunk_tiles(pl, len, c);
                        if (u < ct) break;
                        u -= ct;
                    }
                    const uint64_t c0 = (uint64_t)c * pl.chunk;
                    const uint32_t clen = (uint32_t)min((uint64_t)pl.chunk, (uint64_t)len - c0);
                    const uint32_t full = clen / pl.stripe, tf = bulk_tiles_of(pl, pl.stripe);
                    if (u < full * tf) { k = u / tf; i = u - k * tf; }
                    else { k = full; i = u - full * tf; }
                } else {
                    k = (uint32_t)((me - o - 1 + n) % n);
                    for (c = 0; c + 1 < pl.nchunks; c++) {
                        const uint32_t ct = bulk_tiles_of(pl, bulk_stripe_len(pl, len, c, k));
                        if (u < ct) break;
                        u -= ct;
                    }
                    i = u;
                }
                const uint32_t slen = bulk_stripe_len(pl, len, c, k);
                const uint32_t off0 = c * pl.chunk + k * pl.stripe + i * pl.tile;
                const uint32_t tlen = min(pl.tile, slen - i * pl.tile);
                const uint32_t ngr = (tlen + 15u) >> 4;
                if (jb.kind == JOB_SCATTER) {
                    const int owner = (o + 1 + (int)k) % n;
                    const __amdgpu_buffer_rsrc_t rs = bulk_rsrc_at(P, o, o, s, off0, 16u * ngr);
                    if (!jb.gen) {
                        // a device program's origination: its bytes are first written into the origin's own
                        // heap slot (the copy an application would have staged, rlo_host_bulk_stage), then
                        // read back from there like the host's -- the scatter always moves the origin's copy.
                        // (Each thread reads back only granules it wrote: same-thread order, no drain.)
                        for (uint32_t g0 = 0; g0 < ngr; g0 += (uint32_t)kMoveDepth * kT) {
#pragma unroll
                            for (int uu = 0; uu < kMoveDepth; uu++) {
                                const uint32_t g = g0 + (uint32_t)uu * kT + (uint32_t)tid;
                                st_ring(rs, 16u * g, storm_granule((uint32_t)o, jb.bid, len, off0 + 16u * g), sys);
                            }
                        }
                    }
                    const __amdgpu_buffer_rsrc_t rd = bulk_rsrc_at(P, owner, o, s, off0, 16u * ngr);
                    auto one = [&](int) { return rd; };
                    if (sys) tile_copy<true, W>(rs, ngr, tid, 1, one);
                    else tile_copy<false, W>(rs, ngr, tid, 1, one);
                    VM_DRAIN();
                    __syncthreads();
                    if (tid == 0) {
                        // one GPU: the drain of every storing wave + barrier + one agent-scope add is the
                        // proven hand-off for sc1 stores (MI355X_MICROARCH.md "Valid forms" row 1), no L2
                        // write-back; across GPUs the system-scope release stays
                        if (sys) bulk_release(true);
                        uint32_t* f = bulk_flags(P, owner, o, s);
                        bflag_add(f + c, 1u, sys);
                        bflag_add(f + kBulkTflag, 1u, sys);
                    }
                } else {
                    // GATHER: my stripe of chunk c must have landed (class-A scatter tiles only)
                    if (tid == 0) {
                        uint32_t* f = bulk_flags(P, me, o, s);
                        const uint32_t want = bulk_tiles_of(pl, slen);
                        uint32_t spins = 0;
                        if (bflag_ld(f + c, sys) < want) {  // diagnostics: gather tiles waiting now / last wait
                            atomicAdd((unsigned long long*)&P.jctl[kJctlGatherWaited], 1ull);
                            P.jctl[kJctlLastGather] = ((uint64_t)(uint32_t)o << 48) | ((uint64_t)me << 32) | ((uint64_t)s << 24) | want;
                        }
                        while (bflag_ld(f + c, sys) < want) {
                            __builtin_amdgcn_s_sleep(1);
                            if ((++spins & 1023u) == 0 && (poll32(P.error_flag) || now_ticks() - t_launch > P.deadline_ticks)) {
                                atomicCAS(P.error_flag, 0u, (uint32_t)ERR_TIMEOUT);
                                break;
                            }
                        }
                        const uint64_t key = ((uint64_t)jb.seq << 8) | c;
                        if (key != acq_key) { bulk_acquire(sys); acq_key = key; }
                        atomicAdd((unsigned long long*)&P.jctl[kJctlGatherPassed], 1ull);  // diagnostics: gather waits passed
                    }
                    __syncthreads();
                    const __amdgpu_buffer_rsrc_t rs = bulk_rsrc_at(P, me, o, s, off0, 16u * ngr);
                    // every other non-originator: (o + d) mod n for d = 1 .. n - 1 but my own d
                    const int dme = (me - o + n) % n;
                    auto other = [&](int jj) {
                        const int d = jj + 1 + (jj + 1 >= dme ? 1 : 0);
                        return bulk_rsrc_at(P, (o + d) % n, o, s, off0, 16u * ngr);
                    };
                    if (sys) tile_copy<true, W>(rs, ngr, tid, n - 2, other);
                    else tile_copy<false, W>(rs, ngr, tid, n - 2, other);
                    VM_DRAIN();
                    __syncthreads();
                    if (tid < 64) {
                        if (sys) bulk_release(true);  // (one GPU: drain + barrier + agent add, as the scatter)
                        // every other receiver got this tile; and so did my own count: my copy may not be
                        // released (the origin may not reuse it) before my pushes out of it are done
                        for (int d = 1 + tid; d < n; d += 64) {
                            const int dst = (o + d) % n;
                            bflag_add(bulk_flags(P, dst, o, s) + kBulkTflag, 1u, sys);
                        }
                    }
                }
            } else {  // JOB_VERIFY: checksum my complete copy (the pickup read of every byte)
                if (tid == 0) {
                    const uint64_t key = (uint64_t)jb.seq << 8;
                    if (key != acq_key) { bulk_acquire(sys); acq_key = key; }
                }
                __syncthreads();
                const uint32_t off0 = ti * kVerifyTile;
                const uint32_t tlen = min(kVerifyTile, len - off0);
                const uint32_t ngr = (tlen + 15u) >> 4;
                // cut to the tile: the loads carry no branch (past the end they read zeros), only the sum does
                const __amdgpu_buffer_rsrc_t rs = bulk_rsrc_at(P, me, o, s, off0, 16u * ngr);
                unsigned long long acc = 0;
                {
                    // two batches in flight: the next one's loads are issued before this one is summed
                    constexpr uint32_t step = (uint32_t)kMoveDepth * kT;
                    u32x4 va[kMoveDepth], vb[kMoveDepth];
                    auto load = [&](u32x4 (&v)[kMoveDepth], uint32_t g0) {
#pragma unroll
                        for (int uu = 0; uu < kMoveDepth; uu++) {
                            const uint32_t g = g0 + (uint32_t)uu * kT + (uint32_t)tid;
                            v[uu] = sys ? ld_sys(rs, 16u * g) : ld_sc1(rs, 16u * g);
                        }
                    };
                    auto sum = [&](const u32x4 (&v)[kMoveDepth], uint32_t g0) {
#pragma unroll
                        for (int uu = 0; uu < kMoveDepth; uu++) {
                            const uint32_t g = g0 + (uint32_t)uu * kT + (uint32_t)tid;
#ifdef RLO_AB_VERIFY_READ_ONLY  // A/B probe (fails verification by design): the read-back without its arithmetic
                            if (g < ngr) acc += v[uu].x ^ v[uu].y ^ v[uu].z ^ v[uu].w;
                            continue;
#endif
                            if (g < ngr) {
                                const uint32_t off = off0 + 16u * g;
                                const int b0 = (int)len - (int)off;  // the reference's zero-padded tail
                                const u32x4 w = {mask_bytes(v[uu].x, b0), mask_bytes(v[uu].y, b0 - 4),
                                                 mask_bytes(v[uu].z, b0 - 8), mask_bytes(v[uu].w, b0 - 12)};
                                acc += chunk_mix(off >> 4, w);
                                // the engine's own check of every delivered byte: a device program's bulk
                                // message is the storm payload of (origin, bid), so a granule that is not
                                // what the origin wrote -- a tile whose stores never became visible behind a
                                // complete count -- is a device error, not a wrong sum
#ifndef RLO_AB_VERIFY_NO_CMP  // A/B probe: the checksum without the per-granule comparison with the generator
                                const u32x4 x = storm_granule((uint32_t)o, jb.bid, len, off);
                                if (w.x != x.x || w.y != x.y || w.z != x.z || w.w != x.w)
                                    bulk_fault(P, 14, (uint32_t)(me & 0xff) << 16 | ((off >> 14) & 0xffffu));
#endif
                            }
                        }
                    };
                    load(va, 0u);
                    for (uint32_t g0 = 0; g0 < ngr; g0 += 2u * step) {
                        load(vb, g0 + step);
                        sum(va, g0);
                        if (g0 + step >= ngr) break;
                        load(va, g0 + 2u * step);
                        sum(vb, g0 + step);
                    }
                }
                // workgroup sum of this tile -> the sub-job's sum (LDS; added to the job's once, below)
                for (int sh = 32; sh >= 1; sh >>= 1) acc += __shfl_xor(acc, sh);
                if ((tid & 63) == 0) atomicAdd((unsigned long long*)&S.mv_sum, acc);
            }
        }
        // ---- sub-job finished
        if (tid == 0) atomicAdd((unsigned long long*)&P.jctl[kJctlTilesDone + cls], (unsigned long long)jb.ntiles);  // diagnostics
        if (jb.kind == JOB_VERIFY) {
            __syncthreads();  // every wave's tile sums are in S.mv_sum
            if (tid == 0) {
                const uint32_t ps = jb.parent;
                (void)__hip_atomic_fetch_add(&P.jsum[cls * P.jslots + ps], (uint64_t)S.mv_sum, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                S.mv_sum = 0;
                // this sub-job's sum before its count: the finisher reads them
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t old = atomicAdd(&P.jdone[cls * P.jslots + ps], jb.ntiles);
                if (old + jb.ntiles == jb.total) {  // the job's last tiles: deliver the checksum, release
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    const uint64_t part = __hip_atomic_load(&P.jsum[cls * P.jslots + ps], __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t tot = part + chunk_mix(0xFFFFFFFFu, u32x4{(uint32_t)o, jb.bid, TAG_BCAST, len});
                    atomicAdd((unsigned long long*)&P.stats[jb.lr].bcast_sum, (unsigned long long)tot);
                    if (jb.logidx != ~0u)  // the delivery record gets the message checksum
                        st_sys16(reinterpret_cast<u32x4*>(&P.log[(size_t)jb.lr * P.log_cap + jb.logidx]) + 1,
                                 u32x4{len, 0xffffffffu, (uint32_t)tot, (uint32_t)(tot >> 32)});
                    const uint32_t nt = n > 2 ? bulk_stripe_tiles(pl, len, (uint32_t)((me - o - 1 + n) % n)) : 0u;
                    bulk_slot_release(P, me, o, s, sys, bulk_total_tiles(pl, len) + nt, jb.bid);
                    tl_mark(P, jb.bid, TL_VERIFIED);
                    __hip_atomic_store(&P.jdone[cls * P.jslots + ps], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&P.jsum[cls * P.jslots + ps], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&P.jfree[cls * P.jslots + ps], (uint64_t)(jb.pjob >> lg) + 1ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        BAR();  // S.mv_* is rewritten by the next draw
    }
}

// ------------------------------------------------------------------ the kernel

// program masks of the kernel instantiations (rlo_progress_kernel's PM): every mode bit but the program classes
// it cannot run
constexpr uint32_t kPmAll = 0xFFFFFFFFu;
constexpr uint32_t kPmLat = ~(uint32_t)(MODE_STORM | MODE_IAR | MODE_HOST);
constexpr uint32_t kPmIar = ~(uint32_t)(MODE_STORM | MODE_LAT | MODE_HOST);
constexpr uint32_t kPmStorm = ~(uint32_t)(MODE_LAT | MODE_IAR | MODE_HOST);
constexpr uint32_t kPmHost = ~(uint32_t)(MODE_STORM | MODE_LAT);  // the drop-in's host service (MODE_HOST | MODE_IAR)

// PH: the pending-proposal tables live in HBM (Params.pend_hbm; worlds whose N x pool entries would crowd
// the small copy path's stage out of LDS: the 8-GPU worlds), instantiated for the programs that hold
// proposals (iar, host service).  Every other launch of such a world runs PH = false and never touches
// the table.  All PendState traffic is the rank's own workgroup's, and every iteration that changed an
// entry ends with a drain + barrier (the eager scheme) before any wave reads it again
template <int W, bool BULK, bool LL, bool PH = false, uint32_t PM = kPmAll>
__global__ __launch_bounds__(64 * W) void rlo_progress_kernel(Params P) {
    // PM: the programs this instantiation can run (kPm*): a mode bit PM lacks is a compile-time 0, so the code of
    // the other programs drops out of it (the latency and iar programs' doorbell kernels: fewer live values on the
    // hop path).  rlo_launch_progress picks the instantiation by Params.mode
#define PMODE(x) ((PM & (uint32_t)(x)) ? (P.mode & (uint32_t)(x)) : 0u)
    // pulled payloads (Params.pull) exist only in the 4-wave kernel without bulk messages (slots beyond
    // the small copy path); compiled out of the others
#define PULL_ON (W == 4 && !BULK && P.pull != 0u)
    constexpr int kWaves = W, kBlock = 64 * W, kMaxCand = 64 * W;
    constexpr uint32_t kHostBase = kMaxCand - kPass;  // host mode: command run staged at the last 64 candidates
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    __shared__ Shared<W, BULK> S;
    if constexpr (BULK) {
        if (blockIdx.x >= P.n_local) {  // a mover workgroup of the same launch
            if (threadIdx.x == 0) S.b.mv_sum = 0;
            __syncthreads();
            mover_run<W>(P, S, (int)threadIdx.x);
            return;
        }
    }
    const uint32_t nsmall = P.nsmall;  // chunks per staged message
    const uint32_t nmagic = nsmall > 1 ? 0xFFFFFFFFu / nsmall + 1u : 0u;
    const uint32_t pend_bytes = P.pend_hbm ? 0u : 16u * (uint32_t)P.n * P.pend_slots;
    PendState* pend;  // [n][pend_slots]: dynamic LDS, or (PH) this rank's table in HBM (global-address typed:
                      // no flat instructions, no extra registers on the LDS instantiations)
    if constexpr (PH)
        pend = (PendState*)(__attribute__((address_space(1))) PendState*)(P.pend_hbm + (size_t)blockIdx.x * (uint32_t)P.n * P.pend_slots);
    else
        pend = reinterpret_cast<PendState*>(dyn_lds);
    uint16_t* olist = reinterpret_cast<uint16_t*>(dyn_lds + pend_bytes);       // [oi][256]
    uint8_t* stage = dyn_lds + pend_bytes + P.nout_max * (2u * kMaxCand);      // [message][q] x 16 B
    uint8_t* stage2 = stage + (uint32_t)kMaxCand * nsmall * 16u;                    // [block][lane] x 16 B
    // large messages move in groups of up to kSubMax 1-KiB units (64 payload chunks, one per lane) of
    // one message, packed into stage2: a 4-KiB payload is one group of four units, a 1-KiB payload one
    // group of one unit.  The per-group work (LDS metadata, out-ring walk) is what a staging round
    // costs, so the fewer groups per byte the better; one unit where registers are short (8 waves)
    constexpr uint32_t kSubMax = W == 4 ? 4u : 1u;
    constexpr uint32_t kPair = W == 4 ? 2u : 1u;  // units in registers at once

    const uint32_t s2_units = P.stage2_bytes >> 10;
#define STG(c, q) (stage + (((uint32_t)(c) * nsmall + (uint32_t)(q)) << 4))
#define OL(oi, r) olist[(uint32_t)(oi) * (uint32_t)kMaxCand + (uint32_t)(r)]
    // the pending entry of (origin, pool slot) (rlo_device.hpp Params.pend_slots)
#define PEND(o, q) pend[(uint32_t)(o) * P.pend_slots + ((uint32_t)(q) & (P.pend_slots - 1u))]

    const int lr = blockIdx.x;
    const int me = P.rank_begin + lr;
    const int tid = threadIdx.x, w = tid >> 6;
    // the lane is re-derived every iteration (opaque to the compiler), so lane-derived values cannot be
    // hoisted out of the main loop and held in registers for the whole launch: that took 246 / 254
    // VGPRs (8 / 4 waves) down to 179 / 201, the bulk instantiation from 1 to 2 waves per SIMD, made
    // room for the doorbell pass, and left the storm's speed as it was (profiles/r3_storm_ab.txt)
    int lane = tid & 63;
    uint64_t lt_mask = (1ull << lane) - 1ull;
    const __amdgpu_buffer_rsrc_t rf = mk_rsrc(P.fwd_region, P.fwd_region_bytes);
    const __amdgpu_buffer_rsrc_t rv = mk_rsrc(P.vote_region, P.vote_region_bytes);
    const uint32_t fcap_m = P.fwd_cap - 1, vcap_m = P.vote_cap - 1;
    const bool host = PM == kPmHost || (PMODE(MODE_HOST)) != 0;  // (kPmHost: launched for host mode only)
    // counters are published at the end of the iteration whose stores they cover (all waves
    // drained), not after the next poll: one poll round trip less per hop (p50 -8%, decisions/s
    // +11%).  Not in the storm program: there the drain overlaps wave 0's bookkeeping and poll
    // instead (bcasts/s +4%)
    const bool eager = host || !(PMODE(MODE_LAZYPUB | MODE_STORM));
    const bool hjudge = host && P.host_judge != 0;  // host mode: the host's callbacks judge
    const uint32_t my_mask = ((PMODE(MODE_IAR)) && !hjudge && P.judge_kind == JUDGE_MASK) ? P.judge_mask[me] : 0u;
    // host-service mode: this rank's command ring (pinned host memory) and its counters
    const __amdgpu_buffer_rsrc_t rh =
        mk_rsrc(host ? P.hin + (size_t)lr * P.hin_cap * P.fwd_stride : P.fwd_region, host ? P.hin_cap * P.fwd_stride : 16u);
    uint64_t* const hctl = host ? P.hctl + (size_t)lr * kHctlWords : nullptr;
    uint64_t* const hctl_dev = host ? P.hctl_dev + (size_t)lr * kHctlWords : nullptr;
    const uint32_t hcap_m = host ? P.hin_cap - 1u : 0u;
    // host mode: the command doorbells of this rank (rlo_shm.hpp), and whether the doorbell pass may take
    // commands (its scratch at kLLCmd .. kLLCmdBell + 256 must fit the stage area)
    constexpr uint32_t kLLCmdSlotB = kBellChunks * 32u;
    const __amdgpu_buffer_rsrc_t rll = mk_rsrc(host && P.hll ? P.hll + (size_t)lr * P.hin_cap * kLLCmdSlotB : P.fwd_region,
                                               host && P.hll ? P.hin_cap * kLLCmdSlotB : 16u);
    const bool ll_cmds = host && (uint32_t)kMaxCand * nsmall * 16u >= kLLCmdBell + 256u;
    // bulk messages: pending receptions (o, s) in dynamic LDS [N * B] (BULK instantiation only)
    [[maybe_unused]] BulkPend* const bpend = reinterpret_cast<BulkPend*>(dyn_lds + (BULK ? P.bpend_off : 0u));
    [[maybe_unused]] const uint32_t bsl = BULK ? P.bulk_slots : 1u;

    // ---------------- init
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&P.topo[lr]);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&S.t);
        for (int i = tid; i < (int)(sizeof(RankTopo) / 4); i += kBlock) dst[i] = src[i];
        if (PH || !P.pend_hbm)  // (a PH world's other programs: no table in LDS at all)
            for (int i = tid; i < P.n * (int)P.pend_slots; i += kBlock) pend[i] = PendState{0, 0, 0, 0, 0, 0};
        if constexpr (BULK) {
            for (int i = tid; i < P.n * (int)P.bulk_slots; i += kBlock) bpend[i] = BulkPend{0u, 0u, 0u, -1, 0u, 0u, 0u, 0u};
        }
        for (int i = tid; i < kHistBins; i += kBlock) S.hist[i] = 0;
        for (int i = tid; i < 4 * 64; i += kBlock) { (&S.pubw[0][0])[i] = 0; (&S.snap[0][0])[i] = 0; }
        if (tid < kMaxIn) { S.vout_tail[tid] = 0; S.vout_head[tid] = 0; }
        if (tid < 8) { S.prof[tid] = 0; S.dbg[tid] = 0; S.hd[tid] = 0; }
        if (tid == 0) S.tl_bfid = 0;
        if (tid == 0) {
            S.prof_t = __builtin_amdgcn_s_memtime();
            for (int k = 0; k < kPoolMax; k++) {  // proposalPools_reset, :1351-1362
                S.own_pid[k] = -1;
                S.own_word[k] = 0; S.own_state[k] = 0; S.own_decision[k] = 0;
            }
            S.own_needed = 0; S.own_rr = 0; S.loc_nd = 0; S.loc_n = 0;
            S.own_iter = 0;
            S.own_n = ((PMODE(MODE_IAR)) && !host) ? (P.prop_off[lr + 1] - P.prop_off[lr]) : 0;
            S.lat_pos = 0;
            S.lat_seen = 0;
            S.lat_pos_n = (PMODE(MODE_LAT)) ? P.lat_own_off[lr + 1] - P.lat_own_off[lr] : 0u;
            S.lat_own_next = S.lat_pos_n ? P.lat_own[P.lat_own_off[lr]] : 0xffffffffu;
            S.expect_dec = ((PMODE(MODE_IAR)) && !host) ? P.expect_dec[lr] : 0;
            S.hbase = 0; S.nh = 0; S.ev_n = 0; S.quit = 0; S.hhead = 0; S.hin_head = 0; S.pk_tail = 0;
            S.bcast_delivered = S.dec_delivered = S.dec_approved = S.actions = S.judge_calls = S.originated = 0;
            S.own_decided = S.own_approved = S.proposals_recv = S.log_count = S.stalls = S.stale = 0;
            S.error = 0; S.error_aux = 0; S.exit_now = 0; S.progressed = 0; S.hd_t0 = 0; S.hwait = 0;
            S.hp[0] = 0; S.hp[1] = 0; S.a_done = 0; S.cseq = 0;
            S.relay_tail = 0; S.relay_rel = 0; S.relay_n = 0; S.ref_any = 0; S.rq_n = 0; S.rq_h = 0; S.relay_free = 0;
            if constexpr (BULK) {
                S.b.nbact = 0; S.b.ncomp = 0; S.b.bulk_q = 0; S.b.nstable = 0; S.b.npost = 0;
                S.b.fbase = reinterpret_cast<uint64_t>(bulk_flags(P, me, 0, 0));
                S.b.dbase = reinterpret_cast<uint64_t>(bulk_done(P, me, 0u));
                for (int i = 0; i < kMaxPend / 64; i++) S.b.cmask[i] = 0;
                for (int i = 0; i < kMaxPend / 32; i++) S.b.bonw[i] = 0;
            }
        }
    }
    if constexpr (PH) VM_DRAIN();  // the table's zeros land before any wave (the doorbell pass) reads them
    BAR();
    if (host && tid == 0) pub64_sys(&hctl[kHctlState], 1ull);  // serving (rlo_host_wait_started)
    // a program that holds proposals in a PH world runs the PH instantiation (rlo_launch_progress)
    if (!PH && P.pend_hbm && (PMODE(MODE_IAR | MODE_HOST)) && tid == 0) set_error(S, P, ERR_HOST_CMD, 0x9E4Du);
    const uint64_t t_start = now_ticks();
    unsigned long long acc_sum = 0;  // checksum of delivered bcast chunks (this thread's share)

    // topology: wave-uniform scalars + lane-distributed tables (constant for the launch)
    const RankTopo& t = S.t;
    const int level = uni(t.level), last_wall = uni(t.last_wall), scc = uni(t.scc), sll = uni(t.sll);
    const int n_in = uni(t.n_in), n_in2 = 2 * n_in, nout = 2 * sll;
    const uint32_t inbox = (uint32_t)uni((int)t.inbox_ctrl), outbox = (uint32_t)uni((int)t.outbox_ctrl);
    const uint32_t sl_r = lane < sll ? (uint32_t)t.send_list[lane] : 0u;
    const bool sys = P.sys_scope != 0;
    const uint32_t oring_bytes = P.fwd_cap * P.fwd_stride;
    // wave 0 owns the ring counters: lane g = in-ring g, lane oi = out-ring oi, lane j = vote ring j;
    // each counter is published by a store into the part that polls it
    // remote counter / ring addresses are read from the LDS copy of the topology where they are
    // used (lane = out-ring / in-ring / vote ring), not kept in registers: the kernel sits at the
    // VGPR limit of two waves per SIMD
#define OTPTR t.out_tail[lane >> 1][lane & 1]
#define IHPTR t.in_head[lane >> 1][lane & 1]
#define VHPTR t.vin_head[lane]
#define VTPTR t.vout_tail[lane]
#define ORING(oi) uni64(t.out_ring[(oi) >> 1][(oi) & 1])
    uint64_t in_head_r = 0, out_tail_r = 0, vin_head_r = 0;
    // wave 0's last published counters and last poll, lane-indexed, in LDS (not registers: the
    // kernel sits at the VGPR limit of two waves per SIMD)
#define PUB_IN S.pubw[0][lane]
#define PUB_OUT S.pubw[1][lane]
#define PUB_VIN S.pubw[2][lane]
#define PUB_VOUT S.pubw[3][lane]
    // per in-ring window: messages worth staging next iteration.  A ring whose prefix was cut by
    // out-ring credits is re-staged only a little past what fitted, so a hot rank does not pull
    // (and classify) hundreds of messages per iteration that cannot leave anyway
    uint32_t win_r = kMaxCand;
    uint64_t hpoll = 0;  // host mode, wave 0: lane 0 = command-ring tail, lane 1 = pickup-ring head
    bool peer_failed = false;
    uint64_t idle_since = 0;
    uint32_t idle_n = 0;
    bool idle_prev = false;  // wave 0: the last iteration selected nothing
    uint64_t p_h = 0;  // wave 0: the last poll (host counters; the ring counters are in S.snap)
    uint32_t p_lat = 0;
    // wave 0's own bookkeeping, kept in registers (LDS read-modify-writes by one lane are a serial
    // chain of LDS round trips on the critical path of every iteration)
    const int64_t sched_base = (PMODE(MODE_STORM)) ? P.sched_off[lr] : 0;
    const int64_t sched_n = (PMODE(MODE_STORM)) ? P.sched_off[lr + 1] - sched_base : 0;
    const int64_t expect_bcast = (PMODE(MODE_STORM | MODE_LAT)) ? P.expect_bcast[lr] : 0;
    int64_t sched_next = 0;
    uint64_t n_iter = 0, n_busy = 0, n_stalls = 0;
    bool done_w0 = false;
    uint32_t rbase_r = 0, rtake_r = 0, noi_r = 0;  // lane g / oi: this iteration's selection, admitted counts
    // doorbells (rlo_device.hpp, MODE_LL): on in this launch unless it profiles phases or A/Bs the fast path
    const bool llm = LL && (PMODE(MODE_LL)) && !(PMODE(MODE_PROF | MODE_NOFAST));
    // host mode with doorbells and command doorbells: the host's words (command tail, pickup head, the next
    // command's doorbell) are polled by wave 1 during phase A, so wave 0's spin is one VRAM round trip, not
    // a PCIe one (a host-service hop took twice the device program's: tools/host_latency.py)
    // (4-wave kernels only -- the drop-in's large-slot worlds: the 8-wave doorbell kernel has no registers for it)
    const bool hpw = W == 4 && host && llm && ll_cmds && P.hll != nullptr && !(P.mode & MODE_NOHPW);
    uint32_t a_it = 0;  // phase-A rounds (every wave counts them alike)
    const __amdgpu_buffer_rsrc_t rc = mk_rsrc(P.ctrl, P.ctrl_bytes);  // my part's ctrl region (my bells)
    const uint32_t in_bell = (uint32_t)uni((int)t.in_bell), vin_bell = (uint32_t)uni((int)t.vin_bell);
    bool ll_prog = false;  // the doorbell pass handled something since the last bookkeeping (progress)

    // the lone path's child set: lane-parallel in the program-specialised kernels (the general ones keep the serial
    // form, which needs no extra registers)
#define KIDS_U(o, f) (PM != kPmAll ? kids_of_u(me, (o), (f), level, last_wall, scc, sll, sl_r, lane) \
                               : kids_of(me, (o), (f), level, last_wall, scc, sll, sl_r))
#define NEED_U(k, o) (PM != kPmAll ? need_of_u((k), (o), sll, sl_r, lane) : need_of((k), (o), sll, sl_r))
    // a small message (lane q: slot chunk q, q < nch) into out-rings `need` at their tails: the ring slot,
    // and with bells the child's doorbell for the edge, tagged bell_tag(ring sequence) | vc << 31.  The
    // caller advances out_tail_r
    auto fwd_small = [&](u32x4 v, uint32_t nch, uint32_t need) {
        const uint32_t q = (uint32_t)lane;
        // every out-ring's base (and its child's bell) read from LDS at once, lane oi holding ring oi's: one LDS
        // round trip per forward, not two dependent ones per out-ring (program-specialised kernels: the general
        // ones have no registers for it)
        uint64_t obase = 0, bbase = 0;
        if constexpr (PM != kPmAll) {
            if (lane < nout) {
                obase = t.out_ring[lane >> 1][lane & 1];
                if (LL && llm) bbase = t.out_bell[lane >> 1];
            }
        }
        for (uint32_t m = need; m; m &= m - 1) {
            const int oi = __builtin_ctz(m);
            const uint64_t slot = rdl64(out_tail_r, oi);
            const __amdgpu_buffer_rsrc_t ro =
                mk_rsrc(reinterpret_cast<void*>(PM != kPmAll ? rdl64(obase, oi) : ORING(oi)), oring_bytes);
            if (q < nch) st_ring(ro, (uint32_t)(slot & fcap_m) * P.fwd_stride + 16u * q, v, sys);
            if (LL && llm && nch <= kBellChunks && q < nch) {
                const uint32_t T = bell_tag(slot) | ((uint32_t)(oi & 1) << 31);
                const __amdgpu_buffer_rsrc_t rb = mk_rsrc(
                    reinterpret_cast<void*>(PM != kPmAll ? rdl64(bbase, oi) : uni64(t.out_bell[oi >> 1])), kBellWords * 8u);
                st_ring(rb, 32u * q, u32x4{v.x, T, v.y, T}, sys);
                st_ring(rb, 32u * q + 16u, u32x4{v.z, T, v.w, T}, sys);
            }
        }
    };

    // ---- one lone small message by wave 0 alone: the fast path of phase C (loaded from its ring slot)
    // and the doorbell pass of phase A (from a bell).  Lane q holds slot chunk q (q < nsmall); it came
    // on in-ring fg.  Its effects restate phase F line for line, its forward is phase G's (fwd_small),
    // when every out-ring it needs has room and it is no held proposal.  Returns the out-rings it went to
    // (bit oi), or ~0u: then nothing changed and the full path takes it.  A proposal's data is judged from
    // the ring slot (fsrc) or, for a bell's message, from its LDS copy (from_bell).  The doorbell pass
    // borrows the stage area while the other waves wait at the barrier: bells' data at [0, 1 KiB), votes'
    // at [1 KiB, 1.125 KiB), a bell message's judge copy at kBellJudge (the area is >= 4 KiB: 256 x 16 B)
    // Host judges (hjudge): a proposal without a verdict is held -- its judge request (phase D's LOG_JREQ,
    // with the PBuf) is written the first time (kAsked), later calls find it asked (kHeld); nothing is
    // consumed either way.  With the verdict in (PS_JYES / PS_JNO, a CMD_JUDGE applied) it goes on as judged.
    auto lone = [&](u32x4 v, int fg, uint32_t fsrc, bool from_bell, uint64_t out_head_r) -> uint32_t {
        const uint32_t q = (uint32_t)lane;
        const int ffrom = uni(t.in_src[fg >> 1]);
        const uint32_t fw0 = rdl32(v.x, 0), fid = rdl32(v.y, 0), fw2 = rdl32(v.z, 0), ft0 = rdl32(v.w, 0);
        const int forg = (int)(fw0 & 0xffffu);
        const uint32_t ftag = (fw0 >> 16) & 0xffu, flen = fw2 & 0xffffu, fnch = (kHdr + flen + 15u) >> 4;
        const uint32_t fpseq = fw2 >> 24;
        // this event's payload in the pickup ring's tagged form (host-service kernels, when it fits the slot's
        // stride at 2x); else plain, read by the host once the published tail covers it
        const bool tagp = PM == kPmHost && 32u * (fnch - 1u) <= P.log_stride;
        if (TL_ON(P) && ftag == TAG_BCAST && lane == 0) {
            tl_mark(P, fid, kTlGlobal + (uint32_t)lr);
            tl_put(P, fid, TLC_ISSUE, lr, S.tl_clk[0]);
            tl_put(P, fid, TLC_PASS, lr, S.tl_clk[1]);
            tl_put(P, fid, TLC_FWD, lr, S.tl_clk[2]);
            tl_put(P, fid, TLC_NEXT, lr, S.tl_clk[3]);
        }
        const int fvote = (int)(int8_t)(fw0 >> 24);
        bool ok = ((fw2 >> 16) & 0xffu) == kSlotMark && forg < P.n && fnch <= nsmall &&
                  (ftag == TAG_BCAST || ftag == TAG_DECISION || ftag == TAG_PROPOSAL || (BULK && ftag == TAG_BULK)) &&
                  !(ftag == TAG_BCAST && (PMODE(MODE_LAT)) && fid >= P.lat_rounds);
        int fjudge = 1;
        uint32_t fkids = 0, fneed = 0;
        uint32_t flog = ~0u;
        if (ok && ftag == TAG_PROPOSAL && hjudge) {
            const uint8_t pv = PEND(forg, fpseq).valid;
            const bool same = PEND(forg, fpseq).pid == (int32_t)fid;
            if ((pv == PS_JYES || pv == PS_JNO) && same) {
                fjudge = pv == PS_JYES ? 1 : 0;
            } else if (pv == PS_JREQ && same) {
                return kHeld;  // asked already: the verdict is on its way
            } else if (pv != PS_NONE) {
                return ~0u;    // the entry still holds an earlier proposal of that pool slot: the full path
            } else if (own_has(S, P, (int32_t)fid)) {
                if (lane == 0) set_error(S, P, ERR_PID_COLLISION, fid);  // :690-692
                return kHeld;
            } else {  // judge(data) request with the PBuf (the phase-D hold)
                if (lane == 0) {
                    PendState* pw = &PEND(forg, fpseq);
                    pw->pid = (int32_t)fid;
                    pw->valid = PS_JREQ;
                    flog = log_put<PM>(S, P, lr, LOG_JREQ, forg, ffrom, fid, flen, -1, fpseq, false, tagp);
                    atomicAdd(&S.hwait, 1u);
                }
                flog = rdl32(flog, 0);
                if (q >= 1u && q < fnch) {
                    if (tagp) {
                        pk_payload_tagged(S, P, lr, flog, q, v);
                    } else if (16u * q <= P.log_stride) {  // (plain: the host reads it once the tail covers it)
                        st_sys16(P.log_payload + ((size_t)lr * P.log_cap + flog) * P.log_stride + 16u * (q - 1u), v);
                    }
                }
                return kAsked;
            }
        }
        if (ok) {
            if (ftag == TAG_PROPOSAL) {
                if (!hjudge) {  // device judge on the PBuf data (phase D)
                    uint32_t dl = nsmall > 1 ? rdl32(v.z, 1) : 0u;
                    if (dl > flen - 16u) dl = flen > 16u ? flen - 16u : 0u;
                    if (from_bell) {
                        if (q < kBellChunks) *reinterpret_cast<u32x4*>(stage + kBellJudge + 16u * q) = v;
                        const uint8_t* d = stage + kBellJudge + kHdr + 16u;
                        fjudge = judge_eval_f(P, me, my_mask, (int32_t)fid, [&](uint32_t i) { return d[i]; }, dl);
                    } else {
                        fjudge = judge_eval(P, rf, me, my_mask, (int32_t)fid, fsrc + kHdr + 16u, dl);
                    }
                }
                fkids = fjudge == 1 ? KIDS_U(forg, ffrom) : 0u;
            } else {
                fkids = KIDS_U(forg, ffrom);
            }
            fneed = NEED_U(fkids, forg);
            const bool full = lane < nout && ((fneed >> lane) & 1u) && out_tail_r - out_head_r >= P.fwd_cap;
            // a proposal whose pending entry still holds an earlier proposal of that pool slot
            // goes the full path (held there until that one's decision was applied); with host judges the
            // entry holds this proposal's verdict (checked above)
            const bool held = ftag == TAG_PROPOSAL && !hjudge && PEND(forg, fpseq).valid != PS_NONE;
            ok = __ballot(full) == 0 && !held;
        }
        if (!ok) return ~0u;
        HP(4);
        // the forwards first: a child's copy does not wait for this rank's own effects (its pickup record and
        // payload -- PCIe writes in host mode --, counters, pending state), as the reference forwards before it
        // queues the pickup (rootless_ops.c:583-589)
        fwd_small(v, fnch, fneed);  // the same slot bytes into every needed out-ring (phase G)
        HP(5);
        if (TL_ON(P) && ftag == TAG_BCAST && lane == 0) tl_put(P, fid, TLC_P1, lr, (uint32_t)now_ticks());
        if (ftag == TAG_BCAST) {
            if (lane == 0) {
                tl_parent(P, fid, lr, ffrom);
                atomicAdd(&S.bcast_delivered, 1ull);
                if (PMODE(MODE_HIST)) atomicAdd(&S.hist[hist_bin((uint32_t)now_ticks() - ft0)], 1u);
                flog = log_put<PM>(S, P, lr, LOG_DELIVER | (TAG_BCAST << 8), forg, ffrom, fid, flen, -1,
                               (uint32_t)now_ticks() - ft0, false, tagp);
            }
            flog = rdl32(flog, 0);
            if (q < fnch)
                acc_sum += q == 0 ? chunk_mix(0xFFFFFFFFu, u32x4{(uint32_t)forg, fid, TAG_BCAST, flen})
                                  : chunk_mix(q - 1u, v);
        } else if (ftag == TAG_PROPOSAL) {  // _iar_proposal_handler :668-726
            if (lane == 0) {
                atomicAdd(&S.proposals_recv, 1ull);
                if (own_has(S, P, (int32_t)fid)) {
                    set_error(S, P, ERR_PID_COLLISION, fid);  // :690-692
                } else {
                    const uint32_t k = (uint32_t)fg >> 1;
                    atomicAdd(&S.judge_calls, 1ull);
                    if (!host) log_put<PM>(S, P, lr, LOG_JUDGE, forg, ffrom, fid, flen, fjudge, 0);
                    else if (!hjudge)  // device judge in host mode: the verdict + PBuf for action() (phase F)
                        flog = log_put<PM>(S, P, lr, LOG_JUDGED, forg, ffrom, fid, flen, fjudge, fpseq, false, tagp);
                    PendState* ps = &PEND(forg, fpseq);
                    if (!fjudge) {  // declined: vote 0, not forwarded, not pending (:700-706)
                        ps->valid = PS_NONE;
                        emit_vote<LL>(S, P, me, k, forg, (int32_t)fid, fpseq, 0);
                    } else {
                        const uint32_t nk = (uint32_t)__builtin_popcount(fkids);
                        ps->pid = (int32_t)fid;
                        ps->word = 0;
                        ps->parent_k = (uint16_t)k;
                        ps->needed = (uint8_t)nk;
                        ps->pseq = fpseq | ((flen - 16u) << 8);
                        ps->valid = PS_ACTIVE;
                        if (nk == 0) emit_vote<LL>(S, P, me, k, forg, (int32_t)fid, fpseq, 1);
                    }
                }
            }
            flog = rdl32(flog, 0);
        } else if (BULK && ftag == TAG_BULK) {
            // a bulk announcement (phase F's registration, restated): pending until my copy is complete;
            // its payload is the descriptor {len, bulk sequence} (chunk 1).  On the fast path a hop of the
            // announcement costs what a lone bcast's does, not a full iteration per tree level
            if constexpr (BULK) {
                const uint32_t dlen = rdl32(v.x, 1), dq = rdl32(v.y, 1);
                const uint32_t sl = dq & (bsl - 1u);
                const BulkPlan pl = bulk_plan(P.n, dlen, P.bulk_cross != 0);
                const uint32_t e = (uint32_t)forg * bsl + sl;
                const uint32_t nt = P.n > 2 ? bulk_stripe_tiles(pl, dlen, (uint32_t)((me - forg - 1 + P.n) % P.n)) : 0u;
                if (lane == 0) {
                    tl_mark(P, fid, kTlGlobal + (uint32_t)lr);
                    tl_parent(P, fid, lr, ffrom);
                    const uint32_t ob = atomicOr(&S.b.bonw[e >> 5], 1u << (e & 31u));
                    if ((ob >> (e & 31u)) & 1u) bulk_fault(P, 10, (e << 12) | (fid & 0xfffu));  // still live: announced twice
                    bpend[e] = BulkPend{fid, dlen, bulk_total_tiles(pl, dlen) + nt, ffrom, ft0, dq,
                                        0x5A000000u | ((uint32_t)forg << 8) | sl, 0u};
                    S.b.bact[atomicAdd(&S.b.nbact, 1u)] = e;
                    if (nt) queue_job(S.b, P, JCLS_B, JOB_GATHER, forg, lr, sl, fid, dlen, nt, ffrom, ~0u, dq, 0u);
                }
            }
        } else if (lane == 0) {  // decision: _iar_decision_handler :814-859
            PendState* ps = &PEND(forg, fpseq);
            if (ps->valid == PS_ACTIVE && ps->pid == (int32_t)fid) {
                if (fvote != 0) {
                    atomicAdd(&S.actions, 1ull);
                    log_put<PM>(S, P, lr, LOG_ACTION, forg, ffrom, fid, 0, 1, ps->pseq >> 8);
                }
                ps->valid = PS_NONE;
            }
            atomicAdd(&S.dec_delivered, 1ull);
            if (fvote != 0) atomicAdd(&S.dec_approved, 1ull);
            log_put<PM>(S, P, lr, LOG_DELIVER | (TAG_DECISION << 8), forg, ffrom, fid, 7, fvote, 0);
        }
        if (TL_ON(P) && ftag == TAG_BCAST && lane == 0) tl_put(P, fid, TLC_P2, lr, (uint32_t)now_ticks());
        HP(6);
        if constexpr (BULK) {
            if (TL_ON(P) && ftag == TAG_BULK && lane == 0) {
                tl_put(P, fid, TLC_FWD, lr, (uint32_t)now_ticks());
                S.tl_bfid = fid + 1u;
            }
        }
        if (TL_ON(P) && ftag == TAG_BCAST && lane == 0) tl_mark(P, fid, kTlGlobal + P.n_local + (uint32_t)lr);
        if (flog != ~0u && q >= 1u && q < fnch) {
            if (tagp) {  // the pickup ring's tagged form (no drain and no tail publish stand before the host)
                pk_payload_tagged(S, P, lr, flog, q, v);
            } else if (16u * q <= P.log_stride) {  // (the parity log, a host-mode general kernel, a long payload: plain)
                st_sys16(P.log_payload + ((size_t)lr * P.log_cap + flog) * P.log_stride + 16u * (q - 1u), v);
            }
        }
        if (ftag == TAG_BCAST && (PMODE(MODE_LAT)) && lane == 0) {  // the round's last pickup
            const uint32_t old = sys ? __hip_atomic_fetch_add(&P.lat_count[fid], 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_SYSTEM)
                                     : atomicAdd(&P.lat_count[fid], 1u);
            if (old + 1u == (uint32_t)(P.n - 1)) {
                tl_mark(P, fid, TL_ROUND);
                P.lat_out[fid] = (uint64_t)((uint32_t)now_ticks() - ft0);
                if (sys) __hip_atomic_store(P.lat_round, fid + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else __hip_atomic_store(P.lat_round, fid + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return fneed;
    };

    // ---- a local origination by wave 0 alone (doorbell pass): header + chunks generated in registers,
    // stored to every child when all out-rings have room.  Returns false (nothing changed) otherwise
    // (kind K_HOST: the payload chunks are a host command's, loaded to LDS at src by the doorbell pass)
    auto originate = [&](uint32_t kind, uint32_t w0, uint32_t id, uint32_t w2, uint32_t src, uint64_t out_head_r) -> bool {
        const uint32_t len = w2 & 0xffffu, nch = (kHdr + len + 15u) >> 4;
        if (nch > nsmall || nch > kBellChunks) return false;
        const uint32_t need = NEED_U((1u << sll) - 1u, me);  // the whole send_list (:1587)
        if (__ballot(lane < nout && ((need >> lane) & 1u) && out_tail_r - out_head_r >= P.fwd_cap)) return false;
        const uint32_t q = (uint32_t)lane;
        const uint32_t hw2 = (w2 & 0xff00ffffu) | (kSlotMark << 16);
        u32x4 v = {0u, 0u, 0u, 0u};
        if (q == 0) v = u32x4{w0, id, hw2, (uint32_t)now_ticks()};
        else if (q < nch && kind == K_HOST) v = *reinterpret_cast<const u32x4*>(stage + src + 16u * q);
        else if (q < nch) v = gen_chunk(P, kind, me, id, len, src, (int)(int8_t)(w0 >> 24), q);
        fwd_small(v, nch, need);
        if (lane < nout && ((need >> lane) & 1u)) out_tail_r++;
        return true;
    };

    // ---- one vote from child j by lane 0 (_iar_vote_handler :743-812, _vote_merge :1056-1070): phase B1's
    // merge, for the doorbell pass
    auto merge_vote = [&](int origin, int32_t pid, uint32_t pseq, int vote, uint32_t vw) {
        const uint32_t inc = 1u + (vote == 0 ? 0x10000u : 0u);
        if (origin >= P.n) {
            set_error(S, P, ERR_BAD_SLOT, vw);
        } else if (origin == me) {  // a vote for my own proposal (:756-783)
            const uint32_t k = pseq & (P.pend_slots - 1u);
            if (S.own_state[k] != 1 || pid != S.own_pid[k]) {
                set_error(S, P, ERR_VOTE_ORPHAN, (uint32_t)pid);
            } else {
                const uint32_t nw = (S.own_word[k] += inc);
                if ((nw & 0xffffu) == S.own_needed) {
                    const int d = (nw >> 16) == 0 ? 1 : 0;
                    if (d && hjudge) {  // final judge(NULL) (:770-775) is the host's callback (phase B1)
                        log_put<PM>(S, P, lr, LOG_OWN_JREQ, me, -1, (uint32_t)pid, 0, -1, k);
                        atomicAdd(&S.hwait, 1u);
                        S.own_state[k] = 3;
                    } else {
                        if (d) {  // final judge(NULL) (:770-775): every device judge approves NULL
                            atomicAdd(&S.judge_calls, 1ull);
                            if (!host) log_put<PM>(S, P, lr, LOG_JUDGE, me, -1, (uint32_t)pid, 0, 1, 1);
                        }
                        S.own_decision[k] = (uint32_t)d;
                        S.own_state[k] = 2;
                    }
                }
            }
        } else {
            PendState* ps = &PEND(origin, pseq);
            if (ps->valid != PS_ACTIVE || ps->pid != pid) {
                set_error(S, P, ERR_VOTE_ORPHAN, (uint32_t)pid);
            } else {
                const uint32_t nw = (ps->word += inc);
                if ((nw & 0xffffu) == ps->needed)
                    emit_vote<LL>(S, P, me, ps->parent_k, origin, pid, pseq, (nw >> 16) == 0 ? 1 : 0);
            }
        }
    };

    // ---- the doorbell pass (MODE_LL), wave 0 in its poll loop while the other waves wait at the
    // iteration barrier.  It takes the head message of every in-ring -- from the ring's bell when the bell
    // holds it (no slot load, and possibly ahead of the counter), else loaded from the slot the counter
    // shows -- and up to kLLVotes votes of every child (the head one from its vote bell when only the bell
    // has it), then this rank's own originations (device programs): each as the lone fast path handles
    // it, with no full iteration.  A backlog (a ring more than 2 deep, a child more than kLLVotes votes
    // ahead, more rings to load than one round trip covers), a host command, or a message the lone path
    // refuses is the full iteration's (need_full).  Then one drain, and the counters are published (the
    // eager scheme).  The stage area is scratch here (the other waves are parked): bells' data at kLLBell,
    // vote bells' at kLLBellVote, loaded votes at kLLVote, loaded ring heads at kLLRing.  Returns the
    // number of messages handled.
    auto ll_pass = [&](u32x4 ba, u32x4 bb, u32x4 vb, uint64_t in_tail_r, uint64_t vin_tail_r, uint64_t out_head_r,
                       uint64_t hpoll, uint32_t latr, uint32_t errf, bool& need_full) -> uint32_t {
        need_full = false;
        HP(0);
#ifdef RLO_DIAG
        if constexpr (PM == kPmLat || PM == kPmIar)
            if ((P.mode & MODE_HOPPROF) && lane == 0) S.hpt[3] = 0;
#endif
        if (__ballot(errf != 0)) return 0u;
        // the data words to LDS at once (registers are the kernel's scarcest resource): chunk q of in-edge
        // k's bell at kLLBell + 16 (8 k + q), child j's vote bell {word, pid} at kLLBellVote + 8 j
        *reinterpret_cast<u32x4*>(stage + kLLBell + 16u * (uint32_t)lane) = u32x4{ba.x, ba.z, bb.x, bb.z};
        if (TL_ON(P) && lane == 0) S.tl_clk[1] = (uint32_t)now_ticks();
        if (lane < sll) *reinterpret_cast<uint2*>(stage + kLLBellVote + 8u * (uint32_t)lane) = make_uint2(vb.x, vb.z);
        const uint32_t bk = (uint32_t)lane >> 3, bq = (uint32_t)lane & 7u;
        const uint32_t lcap = min(nsmall, kBellChunks);
        // in-ring (k, vc) whose head is h expects bell_tag(h) | vc << 31 in every half of every granule
        const uint32_t e0 = bell_tag((uint32_t)__shfl((int)(uint32_t)in_head_r, (int)(2u * bk)));
        const uint32_t e1 = bell_tag((uint32_t)__shfl((int)(uint32_t)in_head_r, (int)(2u * bk + 1u))) | 0x80000000u;
        const bool inb = (int)bk < n_in;
        const uint64_t B0 = __ballot(inb && ba.y == e0 && ba.w == e0 && bb.y == e0 && bb.w == e0);
        const uint64_t B1 = __ballot(inb && ba.y == e1 && ba.w == e1 && bb.y == e1 && bb.w == e1);
        const uint32_t hn = (kHdr + ((uint32_t)__shfl((int)bb.x, lane & ~7) & 0xffffu) + 15u) >> 4;  // the header's chunks
        const uint64_t gm = hn <= lcap ? (((1ull << hn) - 1ull) << (lane & ~7)) : 0ull;
        const bool g0 = bq == 0u && gm && (B0 & gm) == gm, g1 = bq == 0u && gm && (B1 & gm) == gm;
        const uint64_t fh = __ballot(g0 || g1), fv = __ballot(g1);  // bit 8k: in-edge k's bell is whole (on vc fv)
        const uint32_t evh = bell_tag(vin_head_r);
        const uint64_t vhm = __ballot(lane < sll && vb.y == evh && vb.w == evh);
        const int rk = lane >> 1;
        const bool rhit = lane < n_in2 && ((fh >> (8 * rk)) & 1ull) && ((uint32_t)((fv >> (8 * rk)) & 1ull) == ((uint32_t)lane & 1u));
        const uint64_t ip = lane < n_in2 && in_tail_r > in_head_r ? in_tail_r - in_head_r : 0ull;
        const uint64_t vp = lane < sll && vin_tail_r > vin_head_r ? vin_tail_r - vin_head_r : 0ull;
        const bool ldr = lane < n_in2 && ip > 0ull && !rhit;  // a counter-visible head without its bell: load it
        const uint64_t ldm = __ballot(ldr);
        // a backlog is the full iteration's; the host service (proposals held for verdicts queue behind a ring's
        // head) lets deeper rings stay on the doorbell pass
        constexpr uint64_t kBacklog = PM == kPmHost ? 4ull : 2ull;
        if (__ballot(ip > kBacklog || vp > (uint64_t)kLLVotes) || __popcll(ldm) > 8) { HPC(1); need_full = true; return 0u; }
        HP(1);
        uint32_t ncmd = 0;  // host commands to take (FIFO order, the first kLLCmds)
        bool cbell = false;  // ... the one in the command doorbell (already loaded, at kLLCmd)
        if (host) {  // too little room in the pickup ring: wait for the host
            const uint32_t pk_free = P.log_cap - (uint32_t)(S.pk_tail - rdl64(hpoll, 1));
            if (pk_free < 2u * (uint32_t)__popcll(__ballot(rhit || ldr)) + 2u * P.own_pool + 8u) { HPC(7); return 0u; }
            if (ll_cmds) {
                const uint64_t ct = rdl64(hpoll, 0), hh = S.hin_head;
                ncmd = ct > hh ? (uint32_t)min(ct - hh, (uint64_t)kLLCmds) : 0u;
                if (!ncmd && hpw) {
                    // the tail shows nothing new: the next command may be whole in its doorbell already, as wave 1
                    // copied it (a seqlock: S.cseq = its tag before and after the copy is read)
                    const uint32_t T = bell_tag(hh);
                    const uint32_t s1 = (uint32_t)uni((int)*lds_word(&S.cseq));
                    if (s1 == T) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        uint64_t d = 0;
                        if (lane < 16) d = *lds_dword(stage + kLLCmdBell + 8u * (uint32_t)lane);
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        const uint32_t s2 = (uint32_t)uni((int)*lds_word(&S.cseq));
                        if (s2 == T) {
                            if (lane < 16) *reinterpret_cast<uint64_t*>(stage + kLLCmd + 8u * (uint32_t)lane) = d;
                            ncmd = 1;
                            cbell = true;
                        }
                    }
                }
            } else if (rdl64(hpoll, 0) > S.hin_head) {  // (stage too small for the command scratch)
                need_full = true;
                return 0u;
            }
        }
        const uint32_t nv = (uint32_t)vp;  // votes to load from child j's vote ring (<= kLLVotes)
        // (a latency round of bulk messages is originated by the full path: its announcement, heap slot and
        // scatter job)
        const bool lat_go = (PMODE(MODE_LAT)) && (!BULK || P.len <= P.ring_cap) && S.lat_own_next != 0xffffffffu &&
                            rdl32(latr, 1) == S.lat_own_next;
        const bool iar_dev = (PMODE(MODE_IAR)) != 0;  // (host mode: decisions only -- its proposals are commands)
        const uint64_t nvm = __ballot(nv > 0u);
        // a bulk round of the latency program (its slot free by the release counts phase A last read): the
        // announcement by this pass too, and its scatter posted here -- not a full iteration per round
        [[maybe_unused]] bool blat = false;
        if constexpr (BULK) {
            blat = (PMODE(MODE_LAT)) && P.len > P.ring_cap && S.lat_own_next != 0xffffffffu &&
                   rdl32(latr, 1) == S.lat_own_next &&
                   S.b.sdone[S.b.bulk_q & (bsl - 1u)] >= (uint64_t)(S.b.bulk_q / bsl) * (uint64_t)(P.n - 1);
        }
        if (!fh && !ldm && !vhm && !nvm && !lat_go && !iar_dev && !ncmd && !blat) return 0u;
        if (TL_ON(P) && lane == 0) S.tl_clk[2] = (uint32_t)now_ticks();
        if (ldm || nvm || ncmd) {
            // one round trip: lane 8 s + q loads chunk q of the s-th ring head to load, lane kLLVotes j + i
            // vote i of child j (sc1 loads behind the counters, as phase D0 / B)
            const uint32_t sl = (uint32_t)lane >> 3, q = (uint32_t)lane & 7u;
            int gsel = -1;
            {
                uint32_t c = 0;
                for (uint64_t m = ldm; m; m &= m - 1, c++)
                    if (c == sl) gsel = __builtin_ctzll(m);
            }
            const int gs = gsel < 0 ? 0 : gsel;
            const uint32_t hsel = (uint32_t)__shfl((int)(uint32_t)in_head_r, gs);
            const uint32_t dsel = t.in_data[gs >> 1][gs & 1];
            const uint32_t vj = (uint32_t)lane / kLLVotes, vi = (uint32_t)lane % kLLVotes;
            const uint32_t nvj = (uint32_t)__shfl((int)nv, (int)vj), vhj = (uint32_t)__shfl((int)(uint32_t)vin_head_r, (int)vj);
            const uint32_t vdat = (int)vj < sll ? t.vin_data[vj] : 0u;
            // (branch-free, kOob: the three loads leave back to back, one wait)
            const u32x4 lv = ld_sc1(rf, gsel >= 0 && q < lcap ? dsel + (hsel & fcap_m) * P.fwd_stride + 16u * q : kOob);
            const u32x4 lw = ld_sc1(rv, (int)vj < sll && vi < nvj ? vdat + ((vhj + vi) & vcap_m) * kVoteSlot : kOob);
            // host commands: lane 8 s + q chunk q of command s, from the command ring in host memory
            // (system-scope loads behind the tail poll, as the full path's command DMA)
            u32x4 lc = {0u, 0u, 0u, 0u};
            if (ncmd && !cbell)
                lc = ld_sys(rh, sl < ncmd && q < lcap ? (uint32_t)((S.hin_head + sl) & hcap_m) * P.fwd_stride + 16u * q : kOob);
            *reinterpret_cast<u32x4*>(stage + kLLRing + 16u * (uint32_t)lane) = lv;
            *reinterpret_cast<u32x4*>(stage + kLLVote + 16u * (uint32_t)lane) = lw;
            if (ncmd && !cbell) *reinterpret_cast<u32x4*>(stage + kLLCmd + 16u * (uint32_t)lane) = lc;
        }
        uint32_t done = 0;
        // host commands in FIFO order, as phase C takes them: judge verdicts first of all (a held proposal
        // below then goes on in this pass), bcast and proposal originations from the loaded chunks.  The
        // first command this pass cannot take (quit, bulk, a message longer than the loaded chunks, no room)
        // ends the run; what is left is the full iteration's (need_full) unless only room was missing
        if (ncmd) {
            uint32_t taken = 0;
            for (; taken < ncmd; taken++) {  // uniform
                const u32x4 hd = *reinterpret_cast<const u32x4*>(stage + kLLCmd + 128u * taken);
                const uint32_t htag = (hd.x >> 16) & 0xffu;
                const int vo = (int)(int8_t)(hd.x >> 24);
                if (htag == CMD_JUDGE) {  // verdict of judge(data) for a held proposal (:698)
                    if (lane == 0) {
                        const int og = (int)(hd.x & 0xffffu);
                        PendState* ps = &PEND(og < P.n ? og : 0, hd.z >> 24);
                        if (og < P.n && ps->valid == PS_JREQ && ps->pid == (int32_t)hd.y) {
                            ps->valid = vo ? PS_JYES : PS_JNO;
                            atomicSub(&S.hwait, 1u);
                        } else {
                            set_error(S, P, ERR_HOST_CMD, hd.x);
                        }
                    }
                } else if (htag == CMD_OWN_JUDGE) {  // final judge(NULL) of my proposal (:770-775)
                    if (lane == 0) {
                        const uint32_t k = (hd.z >> 24) & (P.pend_slots - 1u);
                        if (S.own_state[k] == 3 && S.own_pid[k] == (int32_t)hd.y) {
                            S.own_decision[k] = vo ? 1u : 0u;
                            S.own_state[k] = 2;
                            atomicSub(&S.hwait, 1u);
                        } else {
                            set_error(S, P, ERR_HOST_CMD, hd.x);
                        }
                    }
                } else if (htag == TAG_BCAST || htag == TAG_PROPOSAL) {  // RLO_bcast_gen :1581 / RLO_submit_proposal :876
                    const uint32_t len = hd.z & 0xffffu;
                    if (((kHdr + len + 15u) >> 4) > lcap || sll == 0) { HPC(2); need_full = true; break; }
                    if (htag == TAG_BCAST) {
                        if (!originate(K_HOST, (uint32_t)me | (TAG_BCAST << 16) | (0xffu << 24), hd.y, len,
                                       kLLCmd + 128u * taken, out_head_r))
                            break;  // an out-ring is full: later
                        if (lane == 0) atomicAdd(&S.originated, 1ull);
                    } else {
                        // a free pool slot, first from own_rr (phase C's choice); none: later
                        const uint32_t ps2 = (uint32_t)lane < P.pend_slots ? S.own_state[lane] : 0u;
                        const uint64_t busy = __ballot(ps2 != 0u);
                        if ((uint32_t)__popcll(busy) >= P.own_pool) break;
                        uint32_t k = S.own_rr;
                        while ((busy >> k) & 1ull) k = (k + 1u) & (P.pend_slots - 1u);
                        if (!originate(K_HOST, (uint32_t)me | (TAG_PROPOSAL << 16) | (1u << 24), hd.y, len | (k << 24),
                                       kLLCmd + 128u * taken, out_head_r))
                            break;
                        if (lane == 0) {  // proposalPool_proposal_add (:1253-1279)
                            S.own_pid[k] = (int32_t)hd.y;
                            S.own_word[k] = 0;
                            S.own_needed = (uint32_t)sll;  // votes_needed = send_list_len (:881)
                            S.own_state[k] = 1;
                            S.own_rr = k;
                        }
                    }
                } else {  // quit, bulk: the full iteration's
                    HPC(2);
                    need_full = true;
                    break;
                }
            }
            if (taken) {
                if (lane == 0) S.hin_head += taken;
                done += taken;
            }
        }
        // votes: child j's next nv_j from its ring (the loaded slots), or its head from its bell
        for (uint64_t m = nvm | vhm; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            const uint32_t c = (nvm >> j) & 1ull ? rdl32(nv, j) : 1u;
            if (lane == 0) {
                for (uint32_t i = 0; i < c; i++) {
                    if ((nvm >> j) & 1ull) {  // vote slot {origin | vote << 24, pid, pseq, voter}
                        const u32x4 vs = *reinterpret_cast<const u32x4*>(stage + kLLVote + 16u * ((uint32_t)j * kLLVotes + i));
                        merge_vote((int)(vs.x & 0xffffu), (int32_t)vs.y, vs.z & 0xffu, (int)(int8_t)(vs.x >> 24), vs.x);
                    } else {  // vote bell {origin | pseq << 16 | vote << 24, pid}
                        const uint2 vv = *reinterpret_cast<const uint2*>(stage + kLLBellVote + 8u * (uint32_t)j);
                        merge_vote((int)(vv.x & 0xffffu), (int32_t)vv.y, (vv.x >> 16) & 0xffu, (int)(int8_t)(vv.x >> 24), vv.x);
                    }
                }
            }
            if (lane == j) vin_head_r += c;
            done += c;
        }
        // ring heads: from the bell, or the loaded slot
        HP(2);
        const uint64_t rhm = __ballot(rhit);
        for (uint64_t m = rhm | ldm; m; m &= m - 1) {
            const int g = __builtin_ctzll(m);
            const bool fromb = (rhm >> g) & 1ull;
            const uint32_t at = fromb ? kLLBell + 16u * (uint32_t)(8 * (g >> 1)) : kLLRing + 128u * (uint32_t)__popcll(ldm & ((1ull << g) - 1ull));
            u32x4 v = {0u, 0u, 0u, 0u};
            if ((uint32_t)lane < lcap) v = *reinterpret_cast<const u32x4*>(stage + at + 16u * (uint32_t)lane);
            if (((kHdr + (rdl32(v.z, 0) & 0xffffu) + 15u) >> 4) > lcap) {  // longer than one load covers
                need_full = true;
                continue;
            }
            if (TL_ON(P) && lane == 0) S.tl_clk[3] = (uint32_t)now_ticks();
            HP(3);
            const uint32_t need = lone(v, g, 0u, true, out_head_r);
            if (need == kHeld) HPC(6);
            if (need == kHeld || need == kAsked) {  // waits for the host's verdict (asked now: progress)
                if (need == kAsked) done++;
                continue;
            }
            if (need == ~0u) {  // the full path takes it, through its counter
                HPC(3);
                if (!fromb) need_full = true;
                continue;
            }
            if (lane == g) in_head_r++;
            if (lane < nout && ((need >> lane) & 1u)) out_tail_r++;
            done++;
        }
        // my own originations: the pool's decisions, then its next proposals (device programs), or my
        // latency round
        if (iar_dev) {
            const uint32_t ps_ = (uint32_t)lane < P.pend_slots ? S.own_state[lane] : 0u;
            for (uint64_t dm = __ballot(ps_ == 2u); dm; dm &= dm - 1) {  // _iar_decision_bcast :908-917
                const uint32_t k = (uint32_t)__builtin_ctzll(dm);
                const uint32_t id = (uint32_t)S.own_pid[k], dec = S.own_decision[k];
                if (!originate(K_DEC, (uint32_t)me | (TAG_DECISION << 16) | ((dec & 0xffu) << 24), id, 23u | (k << 24), 0u,
                               out_head_r))
                    break;
                if (lane == 0) {
                    atomicAdd(&S.own_decided, 1ull);
                    if (dec) atomicAdd(&S.own_approved, 1ull);
                    log_put<PM>(S, P, lr, LOG_RESULT, me, -1, id, 0, (int)dec, k);
                    S.own_state[k] = 0;
                    S.own_pid[k] = -1;  // proposalPool_rm (:1334-1347) / RLO_proposal_reset (:1649-1673)
                }
                done++;
            }
            for (;;) {  // RLO_submit_proposal :876-906, up to own_pool in flight
                const uint32_t ps2 = (uint32_t)lane < P.pend_slots ? S.own_state[lane] : 0u;
                const uint64_t busy = __ballot(ps2 != 0u);
                if (S.own_iter >= (unsigned long long)S.own_n || (uint32_t)__popcll(busy) >= P.own_pool) break;
                uint32_t k = S.own_rr;
                while ((busy >> k) & 1ull) k = (k + 1u) & (P.pend_slots - 1u);
                const int64_t pi = P.prop_off[lr] + (int64_t)S.own_iter;
                const uint32_t id = (uint32_t)P.prop_pid[pi];
                if (!originate(K_PROP, (uint32_t)me | (TAG_PROPOSAL << 16) | (1u << 24), id,
                               (16u + P.prop_data_len[pi]) | (k << 24), (uint32_t)pi, out_head_r))
                    break;
                if (lane == 0) {  // proposalPool_proposal_add (:1253-1279)
                    S.own_pid[k] = (int32_t)id;
                    S.own_word[k] = 0;
                    S.own_needed = (uint32_t)sll;  // votes_needed = send_list_len (:881)
                    S.own_state[k] = 1;
                    S.own_iter++;
                    S.own_rr = (k + 1u) & (P.pend_slots - 1u);
                }
                done++;
            }
        }
        if (lat_go && originate(K_LAT, (uint32_t)me | (TAG_BCAST << 16) | (0xffu << 24), S.lat_own_next, P.len, 0u,
                                out_head_r)) {
            if (lane == 0) {
                tl_mark(P, S.lat_own_next, TL_ORIGIN);
                atomicAdd(&S.originated, 1ull);
                const uint32_t np = S.lat_pos + 1u;
                S.lat_pos = np;
                S.lat_own_next = np < S.lat_pos_n ? P.lat_own[P.lat_own_off[lr] + np] : 0xffffffffu;
            }
            done++;
        }
        if constexpr (BULK) {
            if (blat) {
                const uint32_t q = S.b.bulk_q, id = S.lat_own_next;
                // the announcement's payload, the descriptor {len, bulk sequence}, as chunk 1 of a K_HOST-style
                // origination from the stage scratch (the judge copy's area: free at this point of the pass)
                if (lane == 0) *reinterpret_cast<u32x4*>(stage + kBellJudge + 16u) = u32x4{P.len, q, 0u, 0u};
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (originate(K_HOST, (uint32_t)me | (TAG_BULK << 16) | (0xffu << 24), id, 16u, kBellJudge, out_head_r)) {
                    if (lane == 0) {
                        tl_mark(P, id, TL_ORIGIN);
                        atomicAdd(&S.originated, 1ull);
                        S.b.bulk_q = q + 1u;
                        const uint32_t np = S.lat_pos + 1u;
                        S.lat_pos = np;
                        S.lat_own_next = np < S.lat_pos_n ? P.lat_own[P.lat_own_off[lr] + np] : 0xffffffffu;
                        queue_job(S.b, P, JCLS_A, JOB_SCATTER, me, lr, q & (bsl - 1u), id, P.len,
                                  bulk_total_tiles(bulk_plan(P.n, P.len, P.bulk_cross != 0), P.len), -1, ~0u, q, 0u);
                    }
                    flush_posts(S.b, P, lane);
                    done++;
                    need_full = true;  // then the bookkeeping (this may have been the program's last origination)
                }
            }
        }
        if (!done) return 0u;
        HPC(4);
        // every store of the pass drained, then the counters (the eager scheme's publish)
        VM_DRAIN();
        HP(7);
        if (lane < nout && out_tail_r != PUB_OUT) { PUB_OUT = out_tail_r; pub64(OTPTR, out_tail_r, sys); }
        if (lane < n_in2 && in_head_r != PUB_IN) { PUB_IN = in_head_r; pub64(IHPTR, in_head_r, sys); }
        if (lane < sll && vin_head_r != PUB_VIN) { PUB_VIN = vin_head_r; pub64(VHPTR, vin_head_r, sys); }
        if (lane < n_in) {
            const uint64_t vt = S.vout_tail[lane];
            if (vt != PUB_VOUT) { PUB_VOUT = vt; pub64(VTPTR, vt, sys); }
        }
        if (host && lane == 0) {
            if (ncmd) pub64_sys(&hctl[kHctlInjHead], S.hin_head);  // the commands taken (the host's sends complete)
            if (S.ev_n) {
                S.pk_tail += S.ev_n;
                S.log_count += S.ev_n;
                S.ev_n = 0;
                pub64_sys(&hctl[kHctlPkTail], S.pk_tail);
            }
        }
        HP(8);
#ifdef RLO_DIAG
        if constexpr (PM == kPmLat || PM == kPmIar)
            if ((P.mode & MODE_HOPPROF) && lane == 0 && done == 1u && S.hpt[3] != 0) {  // one ring message, nothing else
                for (int k = 0; k < 8; k++) S.prof[k] += S.hpt[k + 1] - S.hpt[k];
                S.dbg[0]++;
            }
#endif
        return done;
    };

    // world rank 0 observes round completions of the latency program on its own clock (wave 0, latr lane 1 =
    // the round word just polled): in the spin loop too, where the doorbell pass keeps an idle rank 0 for
    // many rounds (observed only after it, successive rounds read as 0 us apart)
    auto lat_observe = [&](uint32_t latr) {
        const uint32_t done_r = rdl32(latr, 1), seen = S.lat_seen;
        if (done_r > seen) {
            const uint64_t tn = now_ticks();
            for (uint32_t k = seen + (uint32_t)lane; k < done_r && k < P.lat_rounds; k += 64u) P.lat_obs[k] = tn;
            if (lane == 0) S.lat_seen = done_r;
        }
    };

    // BULK, wave 0: which pending receptions are complete -- S.b.cmask over every registered one (nstable := that
    // count, the range phase C's delivery may take); whether any is
    auto bulk_eval = [&]() -> bool {
        bool any = false;
        if constexpr (BULK) {
            const uint32_t nb = (uint32_t)uni((int)S.b.nbact);
            if (TL_ON(P) && lane == 0) S.tl_clk[1] = (uint32_t)now_ticks();
            // my flag lines through one resource: a line's 16 count shards in four 16-B loads (sixteen 4-B loads
            // of one line queued behind each other at the memory: ~1.8 us per poll, vs one load's round trip)
            const __amdgpu_buffer_rsrc_t rfl = mk_rsrc(reinterpret_cast<void*>(uni64(S.b.fbase)), (uint32_t)P.n * bsl * kBulkLine);
            for (uint32_t u = 0; u * 64u < nb; u++) {
                const uint32_t i = u * 64u + (uint32_t)lane;
                bool dn = false;
                if (i < nb) {
                    const uint32_t e = S.b.bact[i];
                    uint32_t tc = 0;
                    if (e >= (uint32_t)P.n * bsl) {
                        bulk_fault(P, 7, e);
                    } else if (P.bulk_cross) {
                        tc = bflag_ld(reinterpret_cast<uint32_t*>(uni64(S.b.fbase) + (uint64_t)e * kBulkLine) + kBulkTflag, sys);
                    } else {
                        u32x4 q[4];
#pragma unroll
                        for (int k = 0; k < 4; k++) q[k] = sys ? ld_sys(rfl, e * kBulkLine + 16u * k) : ld_sc1(rfl, e * kBulkLine + 16u * k);
#pragma unroll
                        for (int k = 0; k < 4; k++) tc += q[k].x + q[k].y + q[k].z + q[k].w;
                    }
                    dn = e < (uint32_t)P.n * bsl && tc >= bpend[e].ntiles;
                    // MODE_TL: when the evaluation that found the copy complete began, when its loads were back
                    if (TL_ON(P) && dn) {
                        tl_put(P, bpend[e].bid, TLC_PASS, lr, (uint32_t)now_ticks());
                        tl_put(P, bpend[e].bid, TLC_ISSUE, lr, S.tl_clk[1]);
                    }
                }
                const uint64_t m = __ballot(dn);
                any |= m != 0ull;
                if (lane == 0) S.b.cmask[u] = m;
            }
            if (lane == 0) S.b.nstable = nb;
        }
        return any;
    };

    for (;;) {
        asm volatile("" : "+v"(lane));  // (see lane's declaration)
        lt_mask = (1ull << lane) - 1ull;
        a_it++;
        // ---------------- A: wave 0 polls; every wave drains its stores of the last iteration
        uint64_t in_tail_r = 0, out_head_r = 0, vin_tail_r = 0, vout_head_r = 0;
        uint32_t errf = 0, sid = 0, latr = 0;
        if (w == 0) {
            // After an iteration that selected nothing, wave 0 re-polls in a tight loop until a
            // polled word moves (the other waves wait at the barrier): a message arriving at an
            // idle rank is seen one poll round trip later instead of after a whole idle iteration.
            // Bounded, so the idle clock and the deadline still tick.
            uint32_t ll_run = 0;
            bool bev = false;  // BULK: this spin evaluated the pending receptions after its doorbell pass
            uint64_t dnw = 0;  // BULK, lane s < B: my heap slot s's release count (done word), polled every spin
            for (uint32_t sp = 0;; sp++) {
                bev = false;
                // host mode: the host-written counters (pinned host memory: a PCIe read, ~1 us more than
                // the ring polls) on every 4th re-poll only, so an idle rank still sees a ring message
                // one VRAM poll after it lands; a command waits at most ~4 re-polls
                // (every spin while a judge verdict is owed: the host answers within a few microseconds)
                // (with command doorbells the next command is polled every spin in its doorbell below)
                if (hpw) {
                    if (lane < 2) hpoll = S.hp[lane];  // wave 1's latest poll
                } else if (host && lane < 2 && ((sp & 3u) == 0u || S.hwait != 0u)) {
                    hpoll = poll64_sys(&hctl_dev[lane == 0 ? kHctlInjTail : kHctlPkHead]);
                }
                if (TL_ON(P) && lane == 0) {
                    S.tl_clk[0] = (uint32_t)now_ticks();
                    if (BULK && S.tl_bfid) { tl_put(P, S.tl_bfid - 1u, TLC_NEXT, lr, S.tl_clk[0]); S.tl_bfid = 0; }
                }
                // branch-free: every lane issues every load of the poll (rlo_kernel_common.hpp kOob), one wait for all.
                // The doorbells first (LL instantiations; a launch without bells reads kOob): nothing that uses a loaded
                // value may stand between the loads, or the compiler waits there
                [[maybe_unused]] u32x4 ba, bb, vb;
                if constexpr (LL) {
                    const uint32_t bk = (uint32_t)lane >> 3, bq = (uint32_t)lane & 7u;
                    const uint32_t bo = llm && (int)bk < n_in ? (in_bell + bk * kBellWords) * 8u + 32u * bq : kOob;
                    ba = ld_sc1(rc, bo);
                    bb = ld_sc1(rc, bo == kOob ? kOob : bo + 16u);
                    vb = ld_sc1(rc, llm && lane < sll ? (vin_bell + 2u * (uint32_t)lane) * 8u : kOob);
                }
                in_tail_r = ld64_sc1(rc, lane < n_in2 ? (inbox + (uint32_t)lane) * 8u : kOob);
                vin_tail_r = ld64_sc1(rc, lane < sll ? (inbox + (uint32_t)(n_in2 + lane)) * 8u : kOob);
                out_head_r = ld64_sc1(rc, lane < nout ? (outbox + (uint32_t)lane) * 8u : kOob);
                vout_head_r = ld64_sc1(rc, lane < n_in ? (outbox + (uint32_t)(nout + lane)) * 8u : kOob);
                errf = ld32_sc1(rc, 0u);  // (the part's error word is its ctrl word 0)
                if constexpr (BULK) {  // my heap slots' release counts (lane s < B), system scope (covers agent scope)
                    const __amdgpu_buffer_rsrc_t rd = mk_rsrc(reinterpret_cast<void*>(uni64(S.b.dbase)), bsl * kBulkLine);
                    dnw = ld64_sys(rd, lane < (int)bsl ? (uint32_t)lane * kBulkLine : kOob);
                }
                // the round in progress (part 0's word when sharded; system scope covers both), every lane; a launch of
                // another program reads its own error word there (never a round: it stops on it anyway)
                if constexpr ((PM & MODE_LAT) != 0u)
                    latr = __hip_atomic_load((PMODE(MODE_LAT)) ? P.lat_round : P.error_flag, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
                if constexpr (LL) {
                    if (llm) {  // my doorbells beside the counters: lane (k, q) chunk q of in-edge k's, lane j child j's vote
                        if ((PMODE(MODE_LAT)) && me == 0) lat_observe(latr);  // every spin: doorbells keep wave 0 here
                        bool need_full = false;
                        const uint32_t nb0 = nact_of(S.b);
                        const uint32_t nll = ll_pass(ba, bb, vb, in_tail_r, vin_tail_r, out_head_r, hpoll, latr, errf, need_full);
                        if (nll) ll_prog = true;
                        if (need_full) { SPIN_WHY(2); break; }  // the full iteration takes the rest
                        // a bulk announcement registered: its copy is often complete already (the movers started at
                        // the origination, the announcement walks the tree) -- evaluated and delivered right away
                        if (BULK && nact_of(S.b) != nb0) { SPIN_WHY(3); break; }
                        if (nll) {
                            // keep serving from here; every 64 passes the full iteration's bookkeeping runs
                            if (++ll_run < 64u) { sp = 0; continue; }
                            SPIN_WHY(3);
                            break;
                        }
                    }
                }
                if ((PMODE(MODE_LAT)) && me == 0 && !(LL && llm)) lat_observe(latr);  // (with bells: above)
                if (!idle_prev || sp >= kIdleSpin) { SPIN_WHY(idle_prev ? 1 : 0); break; }
                // pending receptions: their completion counts are polled here, every spin, and the first complete
                // one ends the spin (phase C delivers it) -- not a full iteration per poll.  Queued job posts (a
                // reception's GATHER) are the full iteration's to write out
                bool bmoved = false;
                if constexpr (BULK) {
                    if (uni((int)S.b.npost) != 0) { SPIN_WHY(4); break; }
                    if (uni((int)S.b.nbact) != 0) {
                        bev = true;
                        if (bulk_eval()) { SPIN_WHY(5); break; }
                    }
                    bmoved = lane < (int)bsl && dnw != S.b.sdone[lane];  // a released heap slot of mine (an origination may wait)
                }
                // with doorbells only new work counts: a counter that caught up with what the bells already
                // delivered, credits (nothing waits for them in an idle iteration), another rank's round.  Nor
                // do the host's words: the doorbell pass takes the commands (need_full for the ones it cannot)
                // and waits for pickup room itself -- a full iteration on every pickup the host consumed would
                // stand between a judge request and its verdict
                const bool moved =
                    llm ? (in_tail_r != S.snap[0][lane] && in_tail_r > in_head_r) ||
                              (vin_tail_r != S.snap[1][lane] && vin_tail_r > vin_head_r) ||
                              (latr != p_lat && rdl32(latr, 1) == S.lat_own_next) || errf != 0
                        : in_tail_r != S.snap[0][lane] || vin_tail_r != S.snap[1][lane] || out_head_r != S.snap[2][lane] ||
                              vout_head_r != S.snap[3][lane] || hpoll != p_h || latr != p_lat || errf != 0 || bmoved;
                if (__ballot(moved)) { SPIN_WHY(6); break; }
            }
            if (hpw && lane == 0) S.a_done = a_it;  // wave 1 stops polling the host
            S.snap[0][lane] = in_tail_r; S.snap[1][lane] = vin_tail_r; S.snap[2][lane] = out_head_r;
            S.snap[3][lane] = vout_head_r; p_h = hpoll; p_lat = latr;
            // host mode: a heartbeat for the host's watchdog every 4096 iterations (what this rank's
            // wave 0 last saw of its command tail / pickup head, and how far it got)
            if (host && (n_iter & 4095u) == 0 && lane < 3) pub64_sys(&hctl[kHctlBeat + lane], lane == 2 ? n_iter : hpoll);
            if constexpr (BULK) {
                // my heap slots' release counts (the last spin's poll), and which pending receptions are complete
                if (lane < (int)bsl) S.b.sdone[lane] = dnw;
                if (!bev) (void)bulk_eval();  // (else the spin's last evaluation stands: nothing was registered since)
            }
            if ((PMODE(MODE_LAT)) && me == 0) lat_observe(latr);
            if ((PMODE(MODE_STORM)) && sched_next + lane < sched_n && (uint32_t)lane < P.window)
                sid = P.sched_ids[sched_base + sched_next + lane];
        } else if (hpw && w == 1) {
            // the host poller: until wave 0 ends its spin, the next command's doorbell (16 B to each of lanes 0-15,
            // to LDS at kLLCmdBell: the doorbell pass checks its tags) and the command tail / pickup head (-> S.hp),
            // all through scalar loads (spoll_cmd).  Every load of a round is waited for before the stop word is
            // read, so the last round's values are in LDS before the barrier
            for (;;) {
                const uint64_t hh = uni64(S.hin_head);
                // scalar loads (spoll_cmd): the doorbell's first two chunks, the command tail and the pickup head in
                // one round trip; a longer command's other chunks (its header whole and tagged for hh) with vector
                // loads, once
                const uint8_t* slot = reinterpret_cast<const uint8_t*>(
                    uni64(reinterpret_cast<uint64_t>(P.hll + ((uint64_t)lr * P.hin_cap + (hh & hcap_m)) * kLLCmdSlotB)));
                su16 sa;
                uint64_t ht = 0, hk = 0;
                u32x4 cv = {0u, 0u, 0u, 0u};
                uint32_t scov = 2u;  // chunks the scalar loads covered
                if constexpr (PM == kPmHost) {
                    su16 sb;
                    su8 sc;
                    spoll_cmd5(slot, &hctl_dev[kHctlInjTail], &hctl_dev[kHctlPkHead], sa, sb, sc, ht, hk);
#pragma unroll
                    for (int p = 0; p < 4; p++) {
                        if (lane == p) cv = u32x4{sa[4 * p], sa[4 * p + 1], sa[4 * p + 2], sa[4 * p + 3]};
                        if (lane == 4 + p) cv = u32x4{sb[4 * p], sb[4 * p + 1], sb[4 * p + 2], sb[4 * p + 3]};
                    }
                    if (lane == 8) cv = u32x4{sc[0], sc[1], sc[2], sc[3]};
                    if (lane == 9) cv = u32x4{sc[4], sc[5], sc[6], sc[7]};
                    scov = 5u;
                } else {
                    spoll_cmd(slot, &hctl_dev[kHctlInjTail], &hctl_dev[kHctlPkHead], sa, ht, hk);
#pragma unroll
                    for (int p = 0; p < 4; p++)
                        if (lane == p) cv = u32x4{sa[4 * p], sa[4 * p + 1], sa[4 * p + 2], sa[4 * p + 3]};
                }
                if (lane == 0) { S.hp[0] = ht; S.hp[1] = hk; }
                {
                    const uint32_t T0 = bell_tag(hh);
                    const bool head_ok = sa[1] == T0 && sa[3] == T0 && sa[5] == T0 && sa[7] == T0;
                    if (head_ok && ((kHdr + (sa[4] & 0xffffu) + 15u) >> 4) > scov && lane >= (int)(2u * scov) && lane < 16)
                        cv = ld_sys(rll, (uint32_t)(hh & hcap_m) * kLLCmdSlotB + 16u * (uint32_t)lane);
                }
                // whole: every 8-byte half of its chunks (lanes 2q, 2q + 1 = chunk q) carries hh + 1.  Then its
                // words go to LDS under the seqlock S.cseq (0 while they are rewritten), once per command
                const uint32_t T = bell_tag(hh);
                const uint64_t tok = __ballot(lane < 16 && cv.y == T && cv.w == T);
                const uint32_t cn = (kHdr + (rdl32(cv.x, 1) & 0xffffu) + 15u) >> 4;  // header word 2: length
                const uint64_t cm = (1ull << (2u * min(cn, kBellChunks))) - 1ull;
                if ((tok & 3ull) == 3ull && cn <= kBellChunks && (tok & cm) == cm &&
                    (uint32_t)uni((int)S.cseq) != T) {
                    if (lane == 0) *lds_word(&S.cseq) = 0u;
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane < 16)
                        *lds_dword(stage + kLLCmdBell + 8u * (uint32_t)lane) = (uint64_t)cv.x | ((uint64_t)cv.z << 32);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) *lds_word(&S.cseq) = T;
                }
                if (__builtin_amdgcn_readfirstlane((int)S.a_done) == (int)a_it) break;
            }
        }
        VM_DRAIN();
        BAR();  // every payload / vote store of the previous iteration has left its wave
        PROF_STAMP(0);

        // ---------------- C (wave 0): publish the previous iteration, select this one
        if (w == 0) {
            if (lane < nout && out_tail_r != PUB_OUT) { PUB_OUT = out_tail_r; pub64(OTPTR, out_tail_r, sys); }
            if (lane < n_in2 && in_head_r != PUB_IN) { PUB_IN = in_head_r; pub64(IHPTR, in_head_r, sys); }
            if (lane < sll && vin_head_r != PUB_VIN) { PUB_VIN = vin_head_r; pub64(VHPTR, vin_head_r, sys); }
            if (lane < n_in) {
                const uint64_t vt = S.vout_tail[lane];
                if (vt != PUB_VOUT) { PUB_VOUT = vt; pub64(VTPTR, vt, sys); }
                S.vout_head[lane] = vout_head_r;
            }
            peer_failed = __builtin_amdgcn_readfirstlane(errf) != 0;
            PSX(1);
            // pull worlds: relay slots whose references every child consumed are free again (the
            // records are in order; out_head_r = the children's consumption counts just polled)
            uint32_t relay_free = kMaxCand;
            if (PULL_ON) {
                const uint32_t nq = S.rq_n;
                uint32_t nrel = 0, e = S.rq_h;
                uint64_t rel = S.relay_rel;
                for (; nrel < nq; nrel++, e = (e + 1u) % (uint32_t)kRelQ) {
                    const bool ok = lane >= nout || out_head_r >= S.rq_out[e][lane];
                    if (__ballot(!ok)) break;
                    rel = S.rq_relay[e];
                }
                if (lane == 0 && nrel) { S.rq_h = e; S.rq_n = nq - nrel; S.relay_rel = rel; }
                const uint64_t used = S.relay_tail - rel;
                relay_free = used >= P.relay_cap ? 0u : P.relay_cap - (uint32_t)used;
                if (lane == 0) S.relay_free = relay_free;
            }
            // host mode: publish the command head / pickup tail of the previous iteration; the pickup
            // ring bounds this iteration's events: a ring message makes <= 2 (action + decision), plus
            // <= 2 per own proposal in flight (final-judge request, result)
            bool hblock = false;
            uint32_t hlim = kMaxCand;
            if (host) {
                if (lane == 0) pub64_sys(&hctl[kHctlInjHead], S.hin_head);
                if (lane == 1) pub64_sys(&hctl[kHctlPkTail], S.pk_tail);
                const uint64_t pk_head = rdl64(hpoll, 1);
                const uint32_t pk_free = P.log_cap - (uint32_t)(S.pk_tail - pk_head);
                const uint32_t own_ev = 2u * P.own_pool + 2u;
                hblock = pk_free < own_ev + 4u;
                hlim = hblock ? 0u : (pk_free - own_ev) / 2u;
                if ((PMODE(MODE_HDIAG)) && lane == 0) {
                    S.hd[3]++;
                    if (hblock) S.hd[2]++;
                }
            }
            if constexpr (BULK) {
                // completed bulk receptions: delivered now.  Device programs: counted, logged and
                // checksummed by a VERIFY job (which then releases the slot); host mode: one pickup
                // event each (the host copies the bytes out and posts RLO_CMD_BULK_RELEASE)
                const uint32_t nb = S.b.nbact;
                // the last bulk_eval covered exactly [0, nst): an entry appended since has no valid mask bit
                // (cmask words past that range keep older iterations' bits)
                const uint32_t nst = S.b.nstable;
                if (nb) {
                    uint32_t climit = kMaxPend;
                    if (host) {
                        const uint32_t pk_free = P.log_cap - (uint32_t)(S.pk_tail - rdl64(hpoll, 1));
                        climit = pk_free >= 24u ? (pk_free - 16u) / 2u : 0u;
                    }
                    uint32_t seen = 0, kept = 0;
                    for (uint32_t u = 0; u * 64u < nb; u++) {
                        const uint32_t i = u * 64u + (uint32_t)lane;
                        const uint64_t m = S.b.cmask[u];
                        const uint64_t mv = u * 64u < nst ? m & (nst - u * 64u >= 64u ? ~0ull : ((1ull << (nst - u * 64u)) - 1ull)) : 0ull;
                        bool fin = ((mv >> lane) & 1ull) && seen + (uint32_t)__popcll(mv & lt_mask) < climit;
                        seen += (uint32_t)__popcll(mv);
                        const uint32_t e = i < nb ? S.b.bact[i] : 0u;
                        if (fin) {
                            const int o = (int)(e / bsl);
                            const uint32_t sl = e % bsl;
                            const BulkPend pe = bpend[e];
                            const uint32_t ob = atomicAnd(&S.b.bonw[e >> 5], ~(1u << (e & 31u)));
                            if (!((ob >> (e & 31u)) & 1u) || pe.pad0 != (0x5A000000u | ((uint32_t)o << 8) | sl))
                                bulk_fault(P, 11, (e << 8) | (pe.pad0 & 0xffu));
                            if (host) {
                                log_put<PM>(S, P, lr, LOG_DELIVER | (TAG_BULK << 8), o, pe.from, pe.bid, pe.len, -1, sl);
                            } else {
                                tl_mark(P, pe.bid, kTlGlobal + P.n_local + (uint32_t)lr);
                                atomicAdd(&S.bcast_delivered, 1ull);
                                const uint32_t li =
                                    log_put<PM>(S, P, lr, LOG_DELIVER | (TAG_BULK << 8), o, pe.from, pe.bid, pe.len, -1, 0, true);
                                queue_job(S.b, P, JCLS_A, JOB_VERIFY, o, lr, sl, pe.bid, pe.len,
                                         (pe.len + kVerifyTile - 1u) / kVerifyTile, pe.from, li, pe.q, 0u);
                                if (PMODE(MODE_LAT)) {  // the last of N-1 pickups completes the round
                                    const uint32_t old =
                                        sys ? __hip_atomic_fetch_add(&P.lat_count[pe.bid], 1u, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_SYSTEM)
                                            : atomicAdd(&P.lat_count[pe.bid], 1u);
                                    if (old + 1u == (uint32_t)(P.n - 1)) {
                                        tl_mark(P, pe.bid, TL_ROUND);
                                        P.lat_out[pe.bid] = (uint64_t)((uint32_t)now_ticks() - pe.t0);
                                        if (sys) __hip_atomic_store(P.lat_round, pe.bid + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                                        else __hip_atomic_store(P.lat_round, pe.bid + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    }
                                }
                            }
                        }
                        // compact the pending list in place (a kept entry only moves down)
                        const bool keep = i < nb && !fin;
                        const uint64_t km = __ballot(keep);
                        if (keep) S.b.bact[kept + (uint32_t)__popcll(km & lt_mask)] = e;
                        kept += (uint32_t)__popcll(km);
                    }
                    if (lane == 0) {
                        S.b.nbact = kept;
                        S.b.nstable = kept;
                        if (kept != nb) S.progressed = 1;
                    }
                    if (host && kept != nb) {  // their events count against this iteration's pickup room
                        const uint32_t ev = nb - kept;
                        hlim = hlim > (ev + 1u) / 2u ? hlim - (ev + 1u) / 2u : 0u;
                    }
                }
            }
            // votes to merge (wave 1), at most 256 per iteration: trim the ring prefixes
            // (a doorbell may have delivered beyond the counter: head > tail until the counter catches up)
            const uint32_t va = (lane < sll && !hblock && vin_tail_r > vin_head_r) ? (uint32_t)min(vin_tail_r - vin_head_r, (uint64_t)256) : 0u;
            uint32_t vtot = 0, vex = 0;
            if (__ballot(va > 0)) vex = wave_excl_scan(va, &vtot);
            uint32_t vtake = va;
            if (vtot > 256u) {
                vtake = vex >= 256u ? 0u : (vex + va > 256u ? 256u - vex : va);
                vtot = 256u;
            }
            if (lane < sll) { S.vbase[lane] = vex; S.va[lane] = vtake; S.vhead[lane] = vin_head_r; }
            vin_head_r += vtake;  // merged by wave 1 before the next publish
            // in-rings: fair per-ring quotas
            const uint32_t ra = lane < n_in2 && in_tail_r > in_head_r ? (uint32_t)min(in_tail_r - in_head_r, (uint64_t)kMaxCand) : 0u;
            const uint32_t reserve = host ? kPass + P.pend_slots : ((PMODE(MODE_IAR)) ? P.pend_slots + 1u : 0u);  // host: stage block; the pool's originations
            const uint64_t ract = __ballot(ra > 0 && !hblock);
            const int nact = __popcll(ract);
            // max-min fair (water-filling) quotas: a ring's share that a short ring leaves unused goes
            // to the long rings, so a rank fed mostly by one hot parent (a wall rank) drains it in big
            // batches instead of 256/nact per iteration (the per-iteration cost hardly depends on the
            // batch size)
            const uint32_t budget = min(kMaxCand - reserve, hlim);
            const uint32_t want = hblock ? 0u : min(ra, win_r);
            uint32_t take = want;
            {
                uint32_t wtot = 0;
                if (nact) wave_excl_scan(want, &wtot);
                if (wtot > budget) {
                    uint32_t lvl = budget / (uint32_t)nact;
                    for (int it = 0; it < 4; it++) {
                        uint32_t s = 0;
                        wave_excl_scan(min(want, lvl), &s);
                        const uint32_t nabove = (uint32_t)__popcll(__ballot(want > lvl));
                        if (!nabove || s >= budget) break;
                        const uint32_t add = (budget - s) / nabove;
                        if (!add) break;
                        lvl += add;
                    }
                    take = min(want, lvl);
                }
            }
            const bool backlog = __ballot(ra > take) != 0;
            uint32_t R;
            const uint32_t base = wave_excl_scan(take, &R);
            if (lane < n_in2) { S.ring_base[lane] = base; S.ring_take[lane] = take; S.ring_head[lane] = in_head_r; }
            rbase_r = base;
            rtake_r = take;
            noi_r = 0;
            if (lane < nout) {
                S.out_tail0[lane] = out_tail_r;
                S.ofree[lane] = P.fwd_cap - (uint32_t)(out_tail_r - out_head_r);
                S.n_oi[lane] = 0;
            }
            if (lane < kGroups) S.first_bad[lane] = 0xffffffffu;
            if (lane + 64 < kGroups) S.first_bad[lane + 64] = 0xffffffffu;
            PSX(2);
            // local originations
            uint32_t C = R, loc_kind = 0, nstorm = 0, storm_base = 0, lat_id = 0xffffffffu;
            int64_t prop_idx = -1;
            bool hprop_ok = false;  // host mode: a pool slot is free for one host proposal this iteration
            if ((PMODE(MODE_IAR)) && !hblock) {
                // the proposal pool: every decided slot originates its decision (:560-563, :908-917),
                // then free slots (round-robin from own_rr) take the next proposals of my list, up to
                // own_pool in flight (:876-906).  Lane k holds slot k
                const uint32_t ps_ = (uint32_t)lane < P.pend_slots ? S.own_state[lane] : 0u;
                const uint64_t dm = __ballot(ps_ == 2u);
                const uint64_t busy = __ballot(ps_ != 0u);
                uint32_t nd = 0, np = 0;
                if (lane == 0) {
                    for (uint64_t m = dm; m; m &= m - 1) S.loc_slot[nd++] = (uint8_t)__builtin_ctzll(m);
                    const int64_t left = S.own_n - (int64_t)S.own_iter;
                    const uint32_t room = P.own_pool > (uint32_t)__popcll(busy) ? P.own_pool - (uint32_t)__popcll(busy) : 0u;
                    uint32_t want = left < (int64_t)room ? (uint32_t)(left > 0 ? left : 0) : room;
                    uint32_t k = S.own_rr;
                    for (uint32_t i = 0; i < P.pend_slots && np < want; i++, k = (k + 1u) & (P.pend_slots - 1u))
                        if (!((busy >> k) & 1ull)) S.loc_slot[nd + np++] = (uint8_t)k;
                    if (host) {  // the slot a host proposal would take (np == 0: host ranks have no list)
                        for (uint32_t i = 0; i < P.pend_slots && ((busy >> k) & 1ull); i++) k = (k + 1u) & (P.pend_slots - 1u);
                        S.loc_slot[2 * kPoolMax - 1] = (uint8_t)k;
                    }
                    S.own_rr = k;
                }
                hprop_ok = (uint32_t)__popcll(busy) < P.own_pool;
                nd = rdl32(nd, 0);
                np = rdl32(np, 0);
                if (nd + np) {
                    loc_kind = nd ? K_DEC : K_PROP;
                    if (np) prop_idx = P.prop_off[lr] + (int64_t)S.own_iter;
                    C += nd + np;
                }
                if (lane == 0) { S.loc_nd = nd; S.loc_n = nd + np; }
            }
            uint32_t hbase = C, nh = 0, gap_lo = C;
            if (host && !hblock) {
                // commands in FIFO order.  The pending slots (up to 64) are pulled whole into the
                // stage block of candidates 192..255 with ONE LDS-DMA round trip; a leading run of
                // control commands (judge verdicts, quit) is applied now, the run of originations
                // behind it becomes candidates in place (a proposal only when no own proposal is
                // active, and it ends the run)
                // (a command doorbell may have run the head past the tail this poll saw)
                const uint64_t pend_n = rdl64(hpoll, 0) > S.hin_head ? rdl64(hpoll, 0) - S.hin_head : 0ull;
                if ((PMODE(MODE_HDIAG)) && lane == 0) {  // how long seen commands wait here
                    if (pend_n) {
                        S.hd[0]++;
                        if (!S.hd_t0) S.hd_t0 = now_ticks();
                    } else if (S.hd_t0) {
                        const uint64_t d = now_ticks() - S.hd_t0;
                        S.hd[4 + (d < 2000u ? 0 : d < 10000u ? 1 : d < 50000u ? 2 : 3)]++;
                        S.hd_t0 = 0;
                    }
                }
                const uint32_t np = (uint32_t)min(pend_n, (uint64_t)kPass);
                if (np) {
                    const uint32_t nit = np * nsmall;
                    for (uint32_t i0 = 0; i0 < nit; i0 += 64) {
                        const uint32_t i = i0 + lane;
                        if (i < nit) {
                            const uint32_t mi = div_small(i, nmagic), q = i - mi * nsmall;
                            const uint32_t off = (uint32_t)((S.hin_head + mi) & hcap_m) * P.fwd_stride;
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(rh, lds_ptr(STG(kHostBase, 0) + (i0 << 4)), 16,
                                                                     off + 16u * q, 0, 0, kAuxSc1 | 1);
                        }
                    }
                    VM_DRAIN();
                    asm volatile("" ::: "memory");
                    const bool inq = (uint32_t)lane < np;
                    const u32x4 hd = inq ? *reinterpret_cast<const u32x4*>(STG(kHostBase + lane, 0)) : u32x4{0u, 0u, 0u, 0u};
                    const uint32_t htag = (hd.x >> 16) & 0xffu;
                    const uint64_t cm = __ballot(inq && htag >= 16u);
                    const uint32_t ncp = ~cm == 0ull ? 64u : (uint32_t)__builtin_ctzll(~cm);
                    if ((uint32_t)lane < ncp) {
                        const int vo = (int)(int8_t)(hd.x >> 24);
                        if (htag == CMD_JUDGE) {  // verdict of judge(data) for a held proposal (:698)
                            const int og = (int)(hd.x & 0xffffu);
                            PendState* ps = &PEND(og < P.n ? og : 0, hd.z >> 24);
                            if (og < P.n && ps->valid == PS_JREQ && ps->pid == (int32_t)hd.y) {
                                ps->valid = vo ? PS_JYES : PS_JNO;
                                atomicSub(&S.hwait, 1u);
                            } else {
                                set_error(S, P, ERR_HOST_CMD, hd.x);
                            }
                        } else if (htag == CMD_OWN_JUDGE) {  // final judge(NULL) of my proposal (:770-775)
                            const uint32_t k = (hd.z >> 24) & (P.pend_slots - 1u);
                            if (S.own_state[k] == 3 && S.own_pid[k] == (int32_t)hd.y) {
                                S.own_decision[k] = vo ? 1u : 0u;
                                S.own_state[k] = 2;
                                atomicSub(&S.hwait, 1u);
                            } else {
                                set_error(S, P, ERR_HOST_CMD, hd.x);
                            }
                        } else if (htag == CMD_QUIT) {
                            S.quit = 1;
                        } else if (BULK && htag == CMD_BULK_RELEASE) {  // the host copied a bulk delivery out
                            const int og = (int)(hd.x & 0xffffu);
                            const uint32_t sl = hd.z >> 24;
                            if (og < P.n && og != me && sl < bsl) bulk_slot_release(P, me, og, sl, sys);
                            else set_error(S, P, ERR_HOST_CMD, hd.x);
                        } else {
                            set_error(S, P, ERR_HOST_CMD, hd.x);
                        }
                    }
                    const bool org = inq && (uint32_t)lane >= ncp &&
                                     (htag == TAG_BCAST || htag == TAG_PROPOSAL || (BULK && htag == TAG_BULK));
                    const uint64_t om = ncp >= 64u ? 0ull : __ballot(org) >> ncp;
                    uint32_t run = ~om == 0ull ? 64u - ncp : (uint32_t)__builtin_ctzll(~om);
                    const uint64_t pm = ncp >= 64u ? 0ull
                                                   : (__ballot(org && htag == TAG_PROPOSAL) >> ncp) &
                                                         (run >= 64 ? ~0ull : ((1ull << run) - 1ull));
                    if (pm) {
                        const uint32_t fp = (uint32_t)__builtin_ctzll(pm);
                        run = hprop_ok ? fp + 1u : fp;
                        if ((PMODE(MODE_HDIAG)) && lane == 0 && run == fp) S.hd[1]++;
                    }
                    nh = run;
                    gap_lo = C;
                    hbase = kHostBase + ncp;
                    if ((uint32_t)lane >= ncp && (uint32_t)lane < ncp + nh) {
                        S.cand[kHostBase + lane].src = (uint32_t)((S.hin_head + lane) & hcap_m) * P.fwd_stride;
                        S.cand[kHostBase + lane].group = kGroupLocal + K_HOST;
                    }
                    if (lane == 0) { S.hhead = S.hin_head + ncp; S.hin_head += ncp; }
                    if (nh) C = hbase + nh;
                }
            }
            if (!LL && (PMODE(MODE_STORM)) && sched_next < sched_n) {  // (no storm runs with doorbells)
                // throttle: originate only into shallow out-rings so forwarding never waits behind originations
                const bool deep = lane < nout && (out_tail_r - out_head_r) * 2 >= P.fwd_cap;
                const bool allow = !backlog && R < 2 * kPass && __ballot(deep) == 0;
                if ((PMODE(MODE_PROF)) && lane == 0) { if (!allow) S.dbg[5]++; else S.dbg[2]++; }
                if (allow) {
                    const int64_t rem = sched_n - sched_next;
                    uint32_t ww = rem < (int64_t)P.window ? (uint32_t)rem : P.window;
                    if (ww > kMaxCand - C) ww = kMaxCand - C;
                    if constexpr (BULK) {
                        // per-bcast lengths; a bulk one needs its heap slot back from every receiver
                        // of the previous use (done(me, s)); the window ends before one that does not
                        uint32_t ln = 0, isb = 0;
                        if ((uint32_t)lane < ww) {
                            ln = P.len_hi > P.len_lo ? storm_len_of(P.seed, sid, P.len_lo, P.len_hi) : P.len;
                            isb = ln > P.ring_cap ? 1u : 0u;
                        }
                        uint32_t nbk = 0;
                        const uint32_t q = S.b.bulk_q + wave_excl_scan(isb, &nbk);
                        const bool ok = !isb || S.b.sdone[q & (bsl - 1u)] >= (uint64_t)(q / bsl) * (uint64_t)(P.n - 1);
                        const uint64_t bad = __ballot((uint32_t)lane < ww && !ok);
                        if (bad) ww = (uint32_t)__builtin_ctzll(bad);
                        if (bad && lane == 0) atomicAdd((unsigned long long*)&P.jctl[kJctlSlotWaits], 1ull);  // diagnostics: slot waits
                        if ((uint32_t)lane < ww) {
                            S.b.bq[lane] = isb ? q : ~0u;
                            S.b.blen[lane] = ln;
                        }
                    }
                    storm_base = C;
                    nstorm = ww;
                    C += ww;
                    if ((uint32_t)lane < ww) S.storm_ids[lane] = sid;
                }
            }
            if ((PMODE(MODE_LAT)) && C < kMaxCand) {
                // my next round (prefetched) starts when the previous round completed everywhere
                bool lat_ok = true;
                if constexpr (BULK) {
                    if (P.len > P.ring_cap) {
                        const uint32_t q = S.b.bulk_q;
                        lat_ok = S.b.sdone[q & (bsl - 1u)] >= (uint64_t)(q / bsl) * (uint64_t)(P.n - 1);
                    }
                }
                if (lat_ok && S.lat_own_next != 0xffffffffu && rdl32(latr, 1) == S.lat_own_next) { lat_id = S.lat_own_next; C++; }
            }
            // ---- lone-message fast path (wave 0 alone): exactly one candidate, a small ring bcast,
            // decision or proposal (device judge), no votes, and room in every out-ring it needs ->
            // load it, apply its effects, store it to its children and drain, here (lone(), above); the
            // other waves see C == 0 and skip to the bookkeeping.  (My own originations stay on the full
            // path here; the doorbell pass makes them.)  A hop of the latency program or of an IAR round
            // costs one slot load and one store drain instead of the full iteration's seven phases (~17K
            // cycles, tools/lat_anatomy.py).
            uint32_t fastdone = 0;
            // (host-service mode too, for bcasts and decisions -- its proposals take the full path for
            // the host-judge hold and the JUDGED events -- when the pickup ring has room for their events)
            if ((!host || hlim >= 2u) && R == 1u && C == 1u && vtot == 0u && !(PMODE(MODE_PROF | MODE_NOFAST))) {
                const int fg = __builtin_ctzll(__ballot(lane < n_in2 && take > 0u));
                const uint64_t h0 = rdl64(in_head_r, fg);
                const uint32_t fsrc = (uint32_t)uni((int)t.in_data[fg >> 1][fg & 1]) + (uint32_t)(h0 & fcap_m) * P.fwd_stride;
                u32x4 v = {0u, 0u, 0u, 0u};
                if ((uint32_t)lane < nsmall) v = ld_sc1(rf, fsrc + 16u * (uint32_t)lane);  // header + payload, one trip
                const uint32_t fneed = lone(v, fg, fsrc, false, out_head_r);
                if (fneed == kHeld || fneed == kAsked) {  // held for the host's verdict: nothing consumed
                    VM_DRAIN();  // a judge request's record and PBuf before the pickup tail (bookkeeping)
                    if (lane == fg) rtake_r = 0u;
                    R = 0;
                    C = 0;
                    fastdone = fneed == kAsked ? 1u : 0u;
                } else if (fneed != ~0u) {
                    VM_DRAIN();  // wave 0's stores: published in the bookkeeping below
                    // the bookkeeping sees: in-ring g admitted its one message (rtake_r), these out-rings one each
                    noi_r = lane < nout ? ((fneed >> lane) & 1u) : 0u;
                    R = 0;
                    C = 0;
                    fastdone = 1;
                }
            }
            if (lane == 0) {
                S.ract = ract;
                S.vtot = vtot;
                S.R = R; S.C = C; S.nstorm = nstorm; S.storm_base = storm_base; S.loc_kind = loc_kind;
                S.lat_id = lat_id; S.prop_idx = prop_idx; S.nbig = 0; S.progressed = fastdone | (ll_prog ? 1u : 0u);
                S.hbase = hbase; S.nh = nh; S.gap_lo = gap_lo; S.gap_hi = hbase; S.nchmax = 0;
                S.exit_now = done_w0;
                if (PMODE(MODE_PROF)) S.dbg[0] += R;
            }
            ll_prog = false;
        }
        BAR();  // selection visible
        PST(7, 3);
        if (S.exit_now) {  // the final counters are published
            if constexpr (BULK) {
                if (w == 0) flush_posts(S.b, P, lane);  // (phase C's last posts, e.g. a VERIFY)
            }
            break;
        }
        const uint32_t R = S.R, C = S.C;
        const uint32_t nstorm = S.nstorm, storm_base = S.storm_base, loc_kind = S.loc_kind;

        // an iteration with nothing to do goes straight to the bookkeeping (uniform: read after the barrier)
        if (C != 0 || S.vtot != 0) {
            // ---------------- B (wave 1): vote slots (children -> me): loads now, merge after the wait
            const uint32_t vtot = S.vtot;
            u32x4 vreg[4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
            if (w == 1 && vtot) {
    #pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t i = (uint32_t)u * 64u + lane;
                    if (i < vtot) {
                        int j = 0;
                        while (i >= S.vbase[j] + S.va[j]) j++;
                        const uint64_t slot = S.vhead[j] + (i - S.vbase[j]);
                        vreg[u] = ld_sc1(rv, t.vin_data[j] + (uint32_t)(slot & vcap_m) * kVoteSlot);
                    }
                }
            }

            // ---------------- D0: this wave's ring slots -> registers (sc1 loads) -> LDS, ONE round trip.
            // Loads to registers, not LDS-DMA: sc1 loads to registers behind the counter poll are the
            // measured hand-off form without an acquire (MI355X_MICROARCH.md, "Valid forms", row 1);
            // LDS-DMA is not (its lines can stay in L1, and a 128-B line also holds the head of the
            // next, maybe unwritten, slot: seen as stale headers in ~1 of 10 suite runs).
            const uint32_t c_lo = (uint32_t)w * kPass, c_hi = min(c_lo + kPass, R);
            if (c_lo < c_hi) {
                // lane g = in-ring g: its run of candidates, read once (no LDS round trip per ring)
                uint32_t gb = 0, ge = 0, gdat = 0;
                uint64_t gh = 0;
                if (lane < n_in2) {
                    gb = S.ring_base[lane];
                    ge = gb + S.ring_take[lane];
                    gh = S.ring_head[lane];
                    gdat = t.in_data[lane >> 1][lane & 1];
                }
                const uint64_t hit = __ballot(lane < n_in2 && max(gb, c_lo) < min(ge, c_hi));
                // lane = candidate c_lo + lane: its in-ring and slot offset
                const uint32_t cc = c_lo + (uint32_t)lane;
                uint32_t src = 0;
                for (uint64_t m = hit; m; m &= m - 1) {  // rings with candidates in this wave (uniform loop)
                    const int g = __builtin_ctzll(m);
                    const uint32_t b0 = rdl32(gb, g), e0 = rdl32(ge, g), gd = rdl32(gdat, g);
                    const uint64_t h0 = rdl64(gh, g);
                    if (cc >= b0 && cc < e0) {
                        src = gd + (uint32_t)((h0 + (cc - b0)) & fcap_m) * P.fwd_stride;
                        S.cand[cc].src = src;
                        S.cand[cc].group = (uint32_t)g;
                    }
                }
                // item i = (candidate i / nsmall, chunk i % nsmall), in batches of 8 loads per lane: one
                // round trip when nsmall <= 8, ceil(nsmall / 8) for the medium slots (<= 24 chunks) that
                // take the small copy path too
                const uint32_t nit = (c_hi - c_lo) * nsmall;
                // (8 waves: slots <= 8 chunks, one batch -- the loop is compiled out)
                for (uint32_t i0 = 0; i0 < (W == 8 ? 1u : nit); i0 += 512u) {
                    u32x4 sv[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        if (i0 + (uint32_t)u * 64u < nit) {  // uniform: every lane takes part in the shuffle
                            const uint32_t i = i0 + (uint32_t)u * 64u + (uint32_t)lane;
                            const uint32_t mi = div_small(i, nmagic), q = i - mi * nsmall;
                            const uint32_t so = (uint32_t)__shfl((int)src, (int)(mi & 63u));
                            if (i < nit) sv[u] = ld_sc1(rf, so + 16u * q);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const uint32_t i = i0 + (uint32_t)u * 64u + (uint32_t)lane;
                        if (i < nit) *reinterpret_cast<u32x4*>(STG(c_lo, 0) + (i << 4)) = sv[u];
                    }
                }
            }
            VM_DRAIN();  // wave 1: its vote loads
            PST(1, 7);

            // ---------------- B1 (wave 1): merge the votes (_iar_vote_handler :743-812)
            if (w == 1 && vtot) {
    #pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t i = (uint32_t)u * 64u + lane;
                    if (i >= vtot) continue;
                    const u32x4 v = vreg[u];
                    const int origin = (int)(v.x & 0xffffu);
                    const int vote = (int)(int8_t)(v.x >> 24);
                    const int32_t pid = (int32_t)v.y;
                    const uint32_t pseq = v.z;
                    const uint32_t inc = 1u + (vote == 0 ? 0x10000u : 0u);
                    if (origin >= P.n) {
                        set_error(S, P, ERR_BAD_SLOT, v.x);
                    } else if (origin == me) {  // a vote for my own proposal (:756-783)
                        const uint32_t k = pseq & (P.pend_slots - 1u);  // the pool slot (proposalPool_vote_merge :1286)
                        if (S.own_state[k] != 1 || pid != S.own_pid[k]) {
                            set_error(S, P, ERR_VOTE_ORPHAN, (uint32_t)pid);
                        } else {
                            const uint32_t nw = atomicAdd(&S.own_word[k], inc) + inc;
                            if ((nw & 0xffffu) == S.own_needed) {
                                const int d = (nw >> 16) == 0 ? 1 : 0;
                                if (d && hjudge) {  // final judge(NULL) (:770-775) is the host's callback
                                    log_put<PM>(S, P, lr, LOG_OWN_JREQ, me, -1, (uint32_t)pid, 0, -1, k);
                                    atomicAdd(&S.hwait, 1u);
                                    S.own_state[k] = 3;
                                } else {
                                    if (d) {  // final judge(NULL) (:770-775): every device judge approves NULL
                                        atomicAdd(&S.judge_calls, 1ull);
                                        if (!host) log_put<PM>(S, P, lr, LOG_JUDGE, me, -1, (uint32_t)pid, 0, 1, 1);
                                    }
                                    S.own_decision[k] = (uint32_t)d;
                                    S.own_state[k] = 2;
                                }
                            }
                        }
                    } else {  // _vote_merge (:1056-1070)
                        PendState* ps = &PEND(origin, pseq);
                        if (ps->valid != PS_ACTIVE || ps->pid != pid) {
                            set_error(S, P, ERR_VOTE_ORPHAN, (uint32_t)pid);
                        } else {
                            const uint32_t nw = atomicAdd(&ps->word, inc) + inc;
                            if ((nw & 0xffffu) == ps->needed)
                                emit_vote<LL>(S, P, me, ps->parent_k, origin, pid, pseq, (nw >> 16) == 0 ? 1 : 0);
                        }
                    }
                }
                if (lane == 0) S.progressed = 1;
            }

            // ---------------- D: classify this wave's messages
            const uint32_t c = (uint32_t)w * kPass + lane;
            const bool active = c < C && !(c >= S.gap_lo && c < S.gap_hi);  // host mode: no candidates in the gap
            uint32_t kind = K_BAD, w0 = 0, id = 0, w2 = 0, t0 = 0, src = 0, kids = 0, group = 0;
            int from = -1, judge = 1;
            bool want_jreq = false;  // host mode: a proposal whose verdict has not been asked for yet
            [[maybe_unused]] uint32_t bdesc_len = 0, bdesc_q = 0;  // a local bulk origination's descriptor
            if (active && c < R) {
                const u32x4 h = *reinterpret_cast<const u32x4*>(STG(c, 0));
                group = S.cand[c].group;
                src = S.cand[c].src;
                w0 = h.x; id = h.y; w2 = h.z; t0 = h.w;
                from = t.in_src[group >> 1];
                kind = K_RING;
                const int origin = (int)(w0 & 0xffffu);
                const uint32_t tag = (w0 >> 16) & 0xffu;
                const uint32_t mk = (w2 >> 16) & 0xffu;
                if (mk != kSlotMark && !(PULL_ON && mk == kRefMark && tag == TAG_BCAST && ((kHdr + (w2 & 0xffffu) + 15u) >> 4) > nsmall)) {
                    // a slot whose bytes were not visible behind its published tail: every header
                    // carries the mark from its origination, so this is a protocol violation -- stop
                    // loudly instead of forwarding zeros (rings are uncached, rlo_world.cpp)
                    atomicAdd(&S.stale, 1ull);
                    set_error(S, P, ERR_BAD_SLOT, 0x57A1Eu);
                    kind = K_BAD;
                } else if (origin >= P.n || (tag == TAG_BCAST && (PMODE(MODE_LAT)) && id >= P.lat_rounds)) {
                    set_error(S, P, ERR_BAD_SLOT, w0);
                    kind = K_BAD;  // consumed, never forwarded, no side effects
                } else if (tag == TAG_BCAST || tag == TAG_DECISION || (BULK && tag == TAG_BULK)) {
                    kids = kids_of(me, origin, from, level, last_wall, scc, sll, sl_r);
                } else if (tag == TAG_PROPOSAL) {
                    // PBuf [pid][vote][data_len u64][data] at slot + 16 (rootless_ops.c:1402-1410)
                    const uint32_t plen = w2 & 0xffffu;
                    if (hjudge) {  // the host judges: hold the proposal at the head of its ring until the verdict
                        PendState* ps = &PEND(origin, w2 >> 24);
                        const uint8_t pv = ps->valid;
                        if ((pv == PS_JYES || pv == PS_JNO) && ps->pid == (int32_t)id) {
                            judge = pv == PS_JYES ? 1 : 0;
                        } else {
                            judge = -1;
                            if (own_has(S, P, (int32_t)id)) set_error(S, P, ERR_PID_COLLISION, id);  // :690-692
                            // ask once; an entry still held by an earlier proposal of the same pool slot
                            // (its decision is ahead in this ring, applied this iteration) waits
                            else want_jreq = pv == PS_NONE;
                        }
                    } else if (PEND(origin, w2 >> 24).valid != PS_NONE) {
                        judge = -1;  // held one iteration: the entry's previous proposal is decided in this batch
                    } else {
                        uint32_t dl = nsmall > 1 ? reinterpret_cast<const u32x4*>(STG(c, 1))->z : 0u;
                        if (dl > plen - 16u) dl = plen > 16u ? plen - 16u : 0u;
                        judge = judge_eval(P, rf, me, my_mask, (int32_t)id, src + kHdr + 16u, dl);
                    }
                    kids = judge == 1 ? kids_of(me, origin, from, level, last_wall, scc, sll, sl_r) : 0u;
                } else {
                    set_error(S, P, ERR_BAD_SLOT, w0);
                    kind = K_BAD;
                }
            } else if (active) {
                t0 = (uint32_t)now_ticks();
                kids = (1u << sll) - 1u;
                if (c >= storm_base && c < storm_base + nstorm) {
                    kind = K_STORM;
                    group = kGroupLocal + K_STORM;
                    id = S.storm_ids[c - storm_base];
                    w0 = (uint32_t)me | (TAG_BCAST << 16) | (0xffu << 24);
                    w2 = P.len;
                    if constexpr (BULK) {
                        const uint32_t bq = S.b.bq[c - storm_base];
                        w2 = S.b.blen[c - storm_base];
                        if (bq != ~0u) {  // a bulk bcast: the ring carries its announcement
                            bdesc_len = w2;
                            bdesc_q = bq;
                            w0 = (uint32_t)me | (TAG_BULK << 16) | (0xffu << 24);
                            w2 = 16u;
                        }
                    }
                } else if (host && c >= S.hbase && c < S.hbase + S.nh) {  // host origination (RLO_bcast_gen :1581)
                    const u32x4 h = *reinterpret_cast<const u32x4*>(STG(c, 0));
                    kind = K_HOST;
                    group = kGroupLocal + K_HOST;
                    src = S.cand[c].src;
                    id = h.y;
                    if (((h.x >> 16) & 0xffu) == TAG_PROPOSAL) {  // RLO_submit_proposal :876-906 (payload = PBuf)
                        w0 = (uint32_t)me | (TAG_PROPOSAL << 16) | (1u << 24);
                        w2 = (h.z & 0xffffu) | ((uint32_t)S.loc_slot[2 * kPoolMax - 1] << 24);  // its pool slot
                    } else if (BULK && ((h.x >> 16) & 0xffu) == TAG_BULK) {  // payload = descriptor {len, q}
                        w0 = (uint32_t)me | (TAG_BULK << 16) | (0xffu << 24);
                        w2 = 16u;
                    } else {
                        w0 = (uint32_t)me | (TAG_BCAST << 16) | (0xffu << 24);
                        w2 = h.z & 0xffffu;
                    }
                    if ((w2 & 0xffffu) + kHdr > P.fwd_stride) {
                        set_error(S, P, ERR_HOST_CMD, h.x);
                        kind = K_BAD;
                        kids = 0;
                    }
                } else if (loc_kind && c >= R && c < R + S.loc_n) {  // the pool's decisions, then proposals
                    const uint32_t i = c - R, k = S.loc_slot[i];
                    if (i < S.loc_nd) {  // _iar_decision_bcast :908-917
                        kind = K_DEC;
                        group = kGroupLocal + K_DEC;
                        id = (uint32_t)S.own_pid[k];
                        w0 = (uint32_t)me | (TAG_DECISION << 16) | ((S.own_decision[k] & 0xffu) << 24);
                        w2 = 23u | (k << 24);
                    } else {  // RLO_submit_proposal :876-906
                        const int64_t pi = S.prop_idx + (int64_t)(i - S.loc_nd);
                        kind = K_PROP;
                        group = kGroupLocal + K_PROP;
                        src = (uint32_t)pi;
                        id = (uint32_t)P.prop_pid[pi];
                        w0 = (uint32_t)me | (TAG_PROPOSAL << 16) | (1u << 24);
                        w2 = (16u + P.prop_data_len[pi]) | (k << 24);
                    }
                } else {
                    kind = K_LAT;
                    group = kGroupLocal + K_LAT;
                    id = S.lat_id;
                    w0 = (uint32_t)me | (TAG_BCAST << 16) | (0xffu << 24);
                    w2 = P.len;
                    if constexpr (BULK) {
                        if (P.len > P.ring_cap) {
                            bdesc_len = P.len;
                            bdesc_q = S.b.bulk_q;
                            w0 = (uint32_t)me | (TAG_BULK << 16) | (0xffu << 24);
                            w2 = 16u;
                        }
                    }
                }
                // stage the header (+ the payload of a small message) like a received slot; the header
                // carries the slot mark every hop checks
                w2 = (w2 & 0xff00ffffu) | (kSlotMark << 16);
                const uint32_t nch = (kHdr + (w2 & 0xffffu) + 15u) >> 4;
                *reinterpret_cast<u32x4*>(STG(c, 0)) = u32x4{w0, id, w2, t0};
                if (BULK && bdesc_len) {  // the announcement's payload: {len, bulk sequence}
                    *reinterpret_cast<u32x4*>(STG(c, 1)) = u32x4{bdesc_len, bdesc_q, 0u, 0u};
                } else if (nch <= nsmall && kind != K_HOST && kind != K_BAD) {
                    for (uint32_t q = 1; q < nch; q++)
                        *reinterpret_cast<u32x4*>(STG(c, q)) =
                            gen_chunk(P, kind, me, id, w2 & 0xffffu, src, (int)(int8_t)(w0 >> 24), q);
                }
            }
            const int origin = (int)(w0 & 0xffffu);
            const uint32_t need = active ? need_of(kids, origin, sll, sl_r) : 0u;
            for (uint64_t jb = __ballot(want_jreq); jb; jb &= jb - 1) {  // host judge requests (uniform loop)
                const int l = __builtin_ctzll(jb);
                const uint32_t lsrc = rdl32(src, l), lw2 = rdl32(w2, l), lid = rdl32(id, l);
                const int lorg = (int)(rdl32(w0, l) & 0xffffu), lfrom = (int)rdl32((uint32_t)from, l);
                const uint32_t plen = lw2 & 0xffffu;
                uint32_t slot = 0;
                if (lane == 0) {
                    PendState* ps = &PEND(lorg, lw2 >> 24);
                    ps->pid = (int32_t)lid;
                    ps->valid = PS_JREQ;
                    slot = log_put<PM>(S, P, lr, LOG_JREQ, lorg, lfrom, lid, plen, -1, lw2 >> 24);
                    atomicAdd(&S.hwait, 1u);  // (lane 0 of several waves)
                }
                slot = rdl32(slot, 0);
                uint8_t* dst = P.log_payload + ((size_t)lr * P.log_cap + slot) * P.log_stride;
                for (uint32_t q = (uint32_t)lane; 16u * q < plen && 16u * q < P.log_stride; q += 64u)
                    st_sys16(dst + 16u * q, ld_sc1(rf, lsrc + kHdr + 16u * q));
            }
            PST(2, 7);

            // ---------------- E: admission: credits per out-ring, FIFO prefix per source.  The ballot
            // loops visit only the out-rings some lane of this wave needs (a wall rank uses about half)
            const uint32_t wneed = wave_or(need);
            if (lane < nout) S.wcnt[w][lane] = 0;
            for (uint32_t m = wneed; m; m &= m - 1) {
                const int oi = __builtin_ctz(m);
                const uint64_t b = __ballot((need >> oi) & 1u);
                if (lane == 0) S.wcnt[w][oi] = (uint32_t)__popcll(b);
            }
            BAR();
            uint32_t room_r = 0;  // lane oi: free slots of out-ring oi left for this wave
            bool tight_l = false;  // lane oi: the whole workgroup wants more of out-ring oi than is free
            if (lane < nout) {
                uint32_t pre = 0, tot = 0;
                for (int v = 0; v < kWaves; v++) {
                    const uint32_t x = S.wcnt[v][lane];
                    if (v < w) pre += x;
                    tot += x;
                }
                const uint32_t f = S.ofree[lane];
                room_r = f > pre ? f - pre : 0u;
                tight_l = tot > f;
            }
            bool fits = active && judge >= 0;
            // only a tight out-ring can refuse a message (a wall rank has ~2 of its ~15)
            for (uint32_t m = wneed & (uint32_t)__ballot(tight_l); m; m &= m - 1) {
                const int oi = __builtin_ctz(m);
                const bool bit = (need >> oi) & 1u;
                const uint64_t b = __ballot(bit);
                if (b && bit && (uint32_t)__popcll(b & lt_mask) >= rdl32(room_r, oi)) {
                    fits = false;
                    if ((PMODE(MODE_PROF | MODE_HIST)) == MODE_PROF) atomicAdd(&S.hist[oi], 1u);  // misfits per out-ring
                }
            }
            if (active && !fits) atomicMin(&S.first_bad[group], c);
            BAR();  // every wave has read wcnt and posted its first misfit per source
            const bool admitted = active && fits && c < S.first_bad[group];
            const uint32_t an = admitted ? need : 0u;
            const uint32_t len = w2 & 0xffffu;
            const bool isbig = admitted && ((kHdr + len + 15u) >> 4) > nsmall;
            const uint32_t nch_s = (kHdr + len + 15u) >> 4;  // small path: chunks, kept in the olist entry
            const uint32_t wadm = wave_or(an);
            // this wave's admitted count per out-ring differs from its wanted count (wcnt, above) only
            // where a refused message wanted that ring: recount just those
            for (uint32_t m = wave_or(active && !admitted ? need : 0u); m; m &= m - 1) {
                const int oi = __builtin_ctz(m);
                const uint64_t b = __ballot((an >> oi) & 1u);
                if (lane == 0) S.wcnt[w][oi] = (uint32_t)__popcll(b);
            }
            {  // chunks per message on the small copy path this iteration (storm: all equal)
                const uint32_t mx = wave_max(admitted && !isbig ? (kHdr + len + 15u) >> 4 : 0u);
                if (lane == 0 && mx) atomicMax(&S.nchmax, mx);
            }
            BAR();
            uint32_t pre_r = 0;  // lane oi: slots of out-ring oi taken by lower waves
            if (lane < nout) {
                uint32_t tot = 0;
                for (int v = 0; v < kWaves; v++) {
                    const uint32_t x = S.wcnt[v][lane];
                    if (v < w) pre_r += x;
                    tot += x;
                }
                if (w == 0) { S.n_oi[lane] = tot; noi_r = tot; }
            }
            for (uint32_t m = wadm; m; m &= m - 1) {
                const int oi = __builtin_ctz(m);
                const bool bit = (an >> oi) & 1u;
                const uint64_t b = __ballot(bit);
                if (bit) {
                    const uint32_t rel = rdl32(pre_r, oi) + (uint32_t)__popcll(b & lt_mask);
                    OL(oi, rel) = (uint16_t)(c | (isbig ? kBigFlag : (nch_s << 9)));  // c < 512: 9 bits; nch <= 63: 6 bits
                    if (isbig) S.pos[c][oi >> 1] = (uint16_t)rel;
                }
            }
            const uint64_t amask = __ballot(admitted);
            PST(3, 7);

            // ---------------- F: side effects of admitted messages
            const uint32_t tag = (w0 >> 16) & 0xffu;
            const int vote = (int)(int8_t)(w0 >> 24);
            const uint32_t pseq = w2 >> 24;
            uint32_t logidx = ~0u;
            bool lat_deliv = false;
            uint32_t lat_tn = 0;
            if (admitted) {
                if (kind == K_RING) {
                    if (tag == TAG_BCAST) {  // delivered to this rank's pickup queue (:583-589)
                        if (PMODE(MODE_HIST | MODE_LAT)) {
                            const uint64_t tn = now_ticks();
                            if (PMODE(MODE_HIST)) atomicAdd(&S.hist[hist_bin((uint32_t)tn - t0)], 1u);
                            if (PMODE(MODE_LAT)) {  // round bookkeeping after the forwards are issued (G)
                                tl_mark(P, id, kTlGlobal + (uint32_t)lr);
                                tl_parent(P, id, lr, from);
                                lat_deliv = true;
                                lat_tn = (uint32_t)tn - t0;
                            }
                        }
                        // aux: device ticks (10 ns) from origination to this pickup (latency diagnostics)
                        logidx = log_put<PM>(S, P, lr, LOG_DELIVER | (TAG_BCAST << 8), origin, from, id, len, -1,
                                         (uint32_t)now_ticks() - t0);
                    } else if (tag == TAG_PROPOSAL) {  // _iar_proposal_handler (:668-726)
                        const int32_t pid = (int32_t)id;
                        const int k = (int)(group >> 1);
                        atomicAdd(&S.proposals_recv, 1ull);
                        if (own_has(S, P, pid)) {
                            set_error(S, P, ERR_PID_COLLISION, (uint32_t)pid);  // :690-692 (the reference never votes)
                        } else {
                            atomicAdd(&S.judge_calls, 1ull);
                            if (!host) log_put<PM>(S, P, lr, LOG_JUDGE, origin, from, (uint32_t)pid, len, judge, 0);
                            else if (!hjudge) {  // device judge in host mode: the host learns the verdict and keeps
                                                 // the PBuf for action() (rootless_ops.c:842), no round trip
                                const uint32_t slot = log_put<PM>(S, P, lr, LOG_JUDGED, origin, from, (uint32_t)pid, len, judge,
                                                              pseq);
                                uint8_t* dst = P.log_payload + ((size_t)lr * P.log_cap + slot) * P.log_stride;
                                for (uint32_t q = 0; 16u * q < len && 16u * q < P.log_stride; q++)
                                    st_sys16(dst + 16u * q, ld_sc1(rf, src + kHdr + 16u * q));
                            }
                            PendState* ps = &PEND(origin, pseq);
                            if (!judge) {  // declined: vote 0, not forwarded, not pending (:700-706)
                                ps->valid = PS_NONE;
                                emit_vote<LL>(S, P, me, (uint32_t)k, origin, pid, pseq, 0);
                            } else {
                                const uint32_t nk = (uint32_t)__builtin_popcount(kids);
                                ps->pid = pid;
                                ps->word = 0;
                                ps->parent_k = (uint16_t)k;
                                ps->needed = (uint8_t)nk;
                                ps->pseq = pseq | ((len - 16u) << 8);
                                ps->valid = PS_ACTIVE;
                                if (nk == 0) emit_vote<LL>(S, P, me, (uint32_t)k, origin, pid, pseq, 1);
                            }
                        }
                    } else if (tag == TAG_DECISION) {  // :603-615, _iar_decision_handler :814-859
                        PendState* ps = &PEND(origin, pseq);
                        if (ps->valid == PS_ACTIVE && ps->pid == (int32_t)id) {
                            if (vote != 0) {
                                atomicAdd(&S.actions, 1ull);
                                log_put<PM>(S, P, lr, LOG_ACTION, origin, from, id, 0, 1, ps->pseq >> 8);
                            }
                            ps->valid = PS_NONE;
                        }
                        atomicAdd(&S.dec_delivered, 1ull);
                        if (vote != 0) atomicAdd(&S.dec_approved, 1ull);
                        log_put<PM>(S, P, lr, LOG_DELIVER | (TAG_DECISION << 8), origin, from, id, 7, vote, 0);
                    } else if constexpr (BULK) {
                      if (tag == TAG_BULK) {
                        // a bulk announcement: pending until my copy is complete; my movers push my
                        // stripe on to the other receivers once the origin's scatter landed it
                        const u32x4 dsc = *reinterpret_cast<const u32x4*>(STG(c, 1));
                        const uint32_t sl = dsc.y & (bsl - 1u);
                        const BulkPlan pl = bulk_plan(P.n, dsc.x, P.bulk_cross != 0);
                        const uint32_t e = (uint32_t)origin * bsl + sl;
                        // complete = every tile of the message landed here AND my own gather tiles (the
                        // pushes of my stripe out of this copy) are done
                        const uint32_t nt =
                            P.n > 2 ? bulk_stripe_tiles(pl, dsc.x, (uint32_t)((me - origin - 1 + P.n) % P.n)) : 0u;
                        {  // the same message announced here twice (it must arrive exactly once)
                            const BulkPend pv = bpend[e];
                            if (pv.pad0 == (0x5A000000u | ((uint32_t)origin << 8) | sl) && pv.bid == id &&
                                atomicCAS((unsigned long long*)&P.jctl[kJctlFault], 0ull,
                                          ((uint64_t)me << 56) | ((uint64_t)(e & 0xffu) << 48) | ((uint64_t)(id & 0xffffu) << 32) |
                                              ((uint64_t)(from & 0xffff) << 16) | (pv.from & 0xffff)) == 0ull)
                                bulk_fault(P, 12, (e << 12) | (id & 0xfffu));
                        }
                        tl_mark(P, id, kTlGlobal + (uint32_t)lr);
                        tl_parent(P, id, lr, from);
                        const uint32_t ob = atomicOr(&S.b.bonw[e >> 5], 1u << (e & 31u));
                        if ((ob >> (e & 31u)) & 1u) {  // still live: which message was, which one came
                            const BulkPend od = bpend[e];
                            const uint32_t tf = bulk_tcount(P, bulk_flags(P, me, origin, sl), sys);
                            if (atomicCAS((unsigned long long*)&P.jctl[kJctlFault], 0ull,
                                          ((uint64_t)me << 56) | ((uint64_t)(e & 0xffu) << 48) | ((uint64_t)(od.bid & 0xffffu) << 32) |
                                              ((uint64_t)(id & 0xffffu) << 16) | ((tf & 0xffu) << 8) | (od.ntiles & 0xffu)) == 0ull)
                                bulk_fault(P, 10, (e << 12) | (id & 0xfffu));
                        }
                        const BulkPend np_ = BulkPend{id, dsc.x, bulk_total_tiles(pl, dsc.x) + nt, from, t0, dsc.y,
                                                      0x5A000000u | ((uint32_t)origin << 8) | sl, 0u};
                        bpend[e] = np_;
                        S.b.bact[atomicAdd(&S.b.nbact, 1u)] = e;
                        if (nt) queue_job(S.b, P, JCLS_B, JOB_GATHER, origin, lr, sl, id, dsc.x, nt, from, ~0u, dsc.y, 0u);
                      }
                    }
                } else if (kind == K_PROP || (kind == K_HOST && tag == TAG_PROPOSAL)) {
                    // proposalPool_proposal_add (:1253-1279): slot pseq takes the proposal
                    const uint32_t k = pseq & (P.pend_slots - 1u);
                    S.own_pid[k] = (int32_t)id;
                    S.own_word[k] = 0;
                    S.own_needed = (uint32_t)sll;  // votes_needed = send_list_len (:881)
                    S.own_state[k] = 1;
                    if (kind == K_PROP) atomicAdd(&S.own_iter, 1ull);  // admitted proposals are a prefix of the list
                } else if (kind == K_DEC) {
                    const uint32_t k = pseq & (P.pend_slots - 1u);
                    atomicAdd(&S.own_decided, 1ull);
                    if (vote) atomicAdd(&S.own_approved, 1ull);
                    log_put<PM>(S, P, lr, LOG_RESULT, me, -1, id, 0, vote, k);
                    S.own_state[k] = 0;
                    S.own_pid[k] = -1;  // proposalPool_rm (:1334-1347) / RLO_proposal_reset (:1649-1673)
                } else if (kind == K_LAT) {
                    tl_mark(P, id, TL_ORIGIN);
                    const uint32_t np = S.lat_pos + 1u;
                    S.lat_pos = np;
                    S.lat_own_next = np < S.lat_pos_n ? P.lat_own[P.lat_own_off[lr] + np] : 0xffffffffu;
                    if constexpr (BULK) {
                        if (tag == TAG_BULK) S.b.bulk_q++;
                    }
                }
                if (BULK && kind != K_RING && tag == TAG_BULK) {  // my bulk bcast: scatter it (RLO_bcast_gen :1581)
                    uint32_t blen = bdesc_len, bq = bdesc_q;
                    if (kind == K_HOST) {  // the host wrote {len, q} and the bytes (heap slot (me, me, s))
                        const u32x4 dsc = *reinterpret_cast<const u32x4*>(STG(c, 1));
                        blen = dsc.x;
                        bq = dsc.y;
                    }
                    queue_job(S.b, P, JCLS_A, JOB_SCATTER, me, lr, bq & (bsl - 1u), id, blen,
                             bulk_total_tiles(bulk_plan(P.n, blen, P.bulk_cross != 0), blen), -1, ~0u, bq,
                             kind == K_HOST ? 1u : 0u);
                }
            }
            // pull worlds: a large bcast this rank sends on gets a slot of its relay ring -- the copy its
            // children load (RelQ records free it once they consumed the references).  With the relay
            // ring full it is pushed whole instead, as in small-slot worlds: the relay ring is one
            // resource shared by every tree through this rank, so waiting for a slot could close a cycle
            // of waits around the skip ring -- pushing never waits for it
            uint32_t relay = ~0u;
            if (PULL_ON) {
                const bool rl = isbig && an != 0u && tag == TAG_BCAST;
                const uint64_t bm = __ballot(rl);
                if (bm) {
                    uint32_t rb0 = 0;
                    if (lane == 0) rb0 = atomicAdd(&S.relay_n, (uint32_t)__popcll(bm));
                    rb0 = rdl32(rb0, 0);
                    const uint32_t rb = rb0 + (uint32_t)__popcll(bm & lt_mask), rfree = S.relay_free;
                    if (rl && rb < rfree) relay = t.orig_data + (uint32_t)((S.relay_tail + rb) & (P.relay_cap - 1u)) * P.fwd_stride;
                    if (lane == 0 && rb0 < rfree) S.ref_any = 1;
                    if ((PMODE(MODE_PROF)) && lane == 0 && rb0 + (uint32_t)__popcll(bm) > rfree)  // pushed: relay full
                        atomicAdd((unsigned long long*)&S.dbg[4], (unsigned long long)(rb0 + (uint32_t)__popcll(bm) - max(rb0, rfree)));
                }
            }
            if (active) {
                CandL& cl = S.cand[c];
                cl.w0 = w0; cl.id = id; cl.w2 = w2; cl.t0 = t0;
                cl.src = src; cl.need = an; cl.logidx = logidx; cl.kind = kind; cl.relay = relay;
            }
            {  // wave-aggregated counters (one LDS op per wave instead of 64 same-address atomics)
                const uint64_t bdel = __ballot(admitted && kind == K_RING && tag == TAG_BCAST);
                const uint64_t borg = __ballot(admitted && (kind == K_STORM || kind == K_LAT ||
                                                            (kind == K_HOST && (tag == TAG_BCAST || tag == TAG_BULK))));
                const uint64_t bbig = __ballot(isbig);
                if (lane == 0) {
                    if (bdel) atomicAdd(&S.bcast_delivered, (unsigned long long)__popcll(bdel));
                    if (borg) atomicAdd(&S.originated, (unsigned long long)__popcll(borg));
                    if (amask) S.progressed = 1;
                }
                if (bbig) {
                    uint32_t bb = 0;
                    if (lane == 0) bb = atomicAdd(&S.nbig, (uint32_t)__popcll(bbig));
                    bb = rdl32(bb, 0);
                    if (isbig) S.big[bb + (uint32_t)__popcll(bbig & lt_mask)] = (uint16_t)c;
                }
                if (PMODE(MODE_PROF)) {
                    uint32_t tot;
                    wave_excl_scan(admitted ? (uint32_t)__builtin_popcount(kids) : 0u, &tot);
                    if (lane == 0) atomicAdd((unsigned long long*)&S.dbg[6], (unsigned long long)tot);
                }
            }
            BAR();  // olist / cand / n_oi / big complete
            PST(4, 7);
            if constexpr (BULK) {
                if (w == 0) flush_posts(S.b, P, lane);  // this iteration's job posts, before its copies
            }

            // ---------------- G1: stage the first round of large-message groups (before any store)
            // (the 8-wave doorbell instantiation runs programs whose every message takes the small path:
            // the host sets MODE_LL only then, rlo_world.cpp ll_mode; 8-wave worlds have small slots anyway)
            const uint32_t nbig = (LL && W == 8) ? 0u : S.nbig;
            // staging rounds of all of stage2: load -> store -> wait.  (MODE_PIPE, A/B: two halves, round r+1's
            // loads in flight while round r is stored -- measured slower, the rounds halve)
            const bool pipe = s2_units >= 2u * kSubMax && (PMODE(MODE_PIPE));
            const uint32_t hu = pipe ? min(s2_units / 2u, 64u) : min(s2_units, 128u);  // units per round
            const uint32_t hg = pipe ? 64u : 128u;                                     // groups per round
            const uint32_t gsub = min(kSubMax, hu), gspan = 64u * gsub;                 // a group's units, chunks
            // groups hold PAYLOAD chunks (payload chunk p is slot chunk p + 1): the header is known from
            // classification and is stored from registers.  blk_q0[g] = first payload chunk | first unit << 16
            auto plan_big = [&](uint32_t h) {  // wave 0: the next (message, group) pairs for half h, lane-parallel
                if (w == 0) {
                    const uint32_t bm = S.bm, bq0 = S.bq0;
                    const uint32_t goff = h * hg, uoff = h * hu;
                    const uint32_t mi = bm + (uint32_t)lane;
                    uint32_t ng = 0, nu = 0, cc = 0, q0 = 0;
                    if (mi < nbig) {
                        cc = S.big[mi];
                        const uint32_t pch = ((S.cand[cc].w2 & 0xffffu) + 15u) >> 4;  // payload chunks
                        q0 = lane == 0 ? bq0 : 0u;
                        ng = (pch - q0 + gspan - 1u) / gspan;
                        nu = (pch - q0 + 63u) >> 6;
                    }
                    uint32_t totg, totu;
                    const uint32_t sg = wave_excl_scan(ng, &totg), su = wave_excl_scan(nu, &totu);
                    // the first message that does not fit whole is the cursor: its whole groups that fit go
                    // now (every lane before it fits, so sg <= hg and su <= hu there)
                    const uint64_t cut = __ballot(ng != 0 && (sg + ng > hg || su + nu > hu));
                    const uint32_t l = cut ? (uint32_t)__builtin_ctzll(cut) : 64u;
                    const uint32_t fitg = (uint32_t)lane == l ? min(hg - sg, (hu - su) / gsub) : 0u;
                    const uint32_t nw = (uint32_t)lane < l ? ng : fitg;
                    for (uint32_t k = 0; k < nw; k++) {
                        S.blk_c[goff + sg + k] = cc;
                        S.blk_q0[goff + sg + k] = (q0 + gspan * k) | ((uoff + su + gsub * k) << 16);
                    }
                    uint32_t nbm, nbq0, nblk;
                    if (cut) {
                        const uint32_t f = rdl32(fitg, (int)l);
                        nbm = bm + l;
                        nbq0 = rdl32(q0, (int)l) + gspan * f;
                        nblk = rdl32(sg, (int)l) + f;
                    } else {
                        nbm = min(bm + 64u, nbig);
                        nbq0 = 0;
                        nblk = totg;
                    }
                    if (lane == 0) { S.bm = nbm; S.bq0 = nbq0; S.nblk2[h] = nblk; }
                }
            };
            // wave w issues the loads of (and later stores) the blocks b = w, w + 4, ... of half h; the
            // caller waits (VM_DRAIN) before they are read
            auto issue_big = [&](uint32_t h) {
                const uint32_t nblk = S.nblk2[h];
                for (uint32_t b0 = (uint32_t)w; b0 < nblk; b0 += kWaves) {
                    const uint32_t b = h * hg + b0;
                    const uint32_t cc = S.blk_c[b], qw = S.blk_q0[b], q0b = qw & 0xffffu;
                    const CandL& cl = S.cand[cc];
                    const uint32_t pch = ((cl.w2 & 0xffffu) + 15u) >> 4;  // payload chunks
                    const uint32_t nsub = min(gsub, (pch - q0b + 63u) >> 6);
#pragma unroll 1
                    for (uint32_t u = 0; u < nsub; u++) {  // payload chunk q0 + lane + 64 u lands at unit + u, 16 lane
                    const uint32_t pq = q0b + lane + 64u * u;
                    uint8_t* dst = stage2 + ((qw >> 16) + u) * 1024u;
                    if (cl.kind == K_RING) {
                        if (PULL_ON && ((cl.w2 >> 16) & 0xffu) == kRefMark) {
                            // pulled: the payload from the sender's relay slot (the reference staged as
                            // chunk 1 in phase D0)
                            const u32x4 ref = *reinterpret_cast<const u32x4*>(STG(cc, 1));
                            const uint32_t roff = (uint32_t)uni((int)ref.x);
                            // a reference that is not one (unwritten / torn chunk): stop loudly, load nothing
                            const bool rok = uni((int)ref.y) == (int)~roff && (uint32_t)uni((int)ref.z) == kRefMagic;
                            if (!rok && lane == 0) set_error(S, P, ERR_BAD_SLOT, 0x5EF0000u | (pq & 0xffffu));
                            // (the extent made uniform too: read from LDS it is a VGPR, and a VGPR resource
                            // wraps every LDS-DMA load of the pulled payloads in a readfirstlane waterfall loop)
                            const __amdgpu_buffer_rsrc_t rr =
                                mk_rsrc(reinterpret_cast<void*>(uni64(t.in_base[cl.group >> 1]) + roff),
                                        (uint32_t)uni((int)(rok ? (pch + 1u) * 16u : 0u)));
                            if (rok && pq < pch) {
                                if (sys) __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, lds_ptr(dst), 16, 16u * (pq + 1u), 0, 0, kAuxSc1 | 1);
                                else __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, lds_ptr(dst), 16, 16u * (pq + 1u), 0, 0, kAuxSc1);
                            }
                        } else if (pq < pch) {
                            dma16(rf, dst, cl.src + 16u * (pq + 1u));
                        }
                    } else if (cl.kind == K_HOST) {  // payload from the command slot
                        if (pq < pch)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(rh, lds_ptr(dst), 16, cl.src + 16u * (pq + 1u), 0, 0, kAuxSc1 | 1);
                    } else if (pq < pch) {
                        *reinterpret_cast<u32x4*>(dst + 16u * lane) =
                            gen_chunk(P, cl.kind, me, cl.id, cl.w2 & 0xffffu, cl.src, (int)(int8_t)(cl.w0 >> 24), pq + 1u);
                    }
                    }
                }
            };
            // agent acquire after a drain (without the leading vmcnt(0) of the fence builtin): these
            // LDS-DMA loads may leave lines in L1 that straddle into the next, maybe unwritten, slot, and
            // the next iteration must not read them from there.  It completes under the stores, and
            // phase A's VM_DRAIN (or the eager drain) waits for it
            // MODE_PROF: wave 0's cycles waiting for a round's loads (and stores) in dbg[3], the rounds in
            // dbg[4] (push worlds: pull worlds count relay-full pushes there)
            auto big_drain = [&]() {
                if ((PMODE(MODE_PROF)) && tid == 0) {
                    const uint64_t c0 = __builtin_amdgcn_s_memtime();
                    VM_DRAIN();
                    S.dbg[3] += __builtin_amdgcn_s_memtime() - c0;
                    if (!PULL_ON) S.dbg[4]++;
                } else {
                    VM_DRAIN();
                }
            };
            if (nbig) {
                if (tid == 0) { S.bm = 0; S.bq0 = 0; }
                plan_big(0u);
                BAR();
                issue_big(0u);
                big_drain();
                ACQ_NEXT();
            }

            // ---------------- G2: small messages.  Out-ring oi (oi = w, w + 4, ...) receives its
            // admitted messages' staged slots as contiguous (message, chunk) items
#ifdef RLO_AB_NQ2  // A/B probe (wrong bytes by design): the copy loop walks 2 chunks per message
            const uint32_t nq = min(max(S.nchmax, 1u), 2u);
#else
            const uint32_t nq = max(S.nchmax, 1u);  // items per message: the largest small message
#endif
            const uint32_t qmagic = nq > 1 ? 0xFFFFFFFFu / nq + 1u : 0u;
            // the (out-ring, message, chunk) items of all out-rings form one sequence split evenly over
            // the four waves (a rank whose traffic sits on every other out-ring -- rank 0 sends on the
            // wrapped channel only -- would otherwise store from two waves).  A lane walks its items as
            // (message r, chunk q) pairs stepped incrementally (no division or quarter-rate multiply per
            // item: this loop is instruction-latency bound), four per round: their olist reads, then their
            // stage reads, then their stores (two per round: 64 B storm -2 %, 256 B -4 %, r4_storm_ab.txt).
            // What a round costs is its instructions, not its bytes: storing only 2 of a message's chunks
            // took no time off (the same store instructions, fewer lanes), walking only 2 chunks took 8 % /
            // 35 % off the 64 B / 256 B storm (RLO_AB_NQ2); one store per (message, chunk) per out-ring
            // from a wave's own messages (each chunk read once) took 20 % / 50 % more (fewer lanes per store)
            const uint32_t dr = div_small(64u, qmagic), dq = 64u - dr * nq;
            const uint32_t stg_msg = nsmall << 4, stride = P.fwd_stride;
            const uint32_t nit_r = lane < nout ? S.n_oi[lane] * nq : 0u;
            uint32_t items = 0;
            const uint32_t ibase_r = wave_excl_scan(nit_r, &items);
            const uint32_t lo = items * (uint32_t)w / (uint32_t)kWaves, hi = items * (uint32_t)(w + 1) / (uint32_t)kWaves;
            for (uint64_t mo = __ballot(nit_r != 0 && ibase_r < hi && ibase_r + nit_r > lo); mo; mo &= mo - 1) {
                const int oi = __builtin_ctzll(mo);
                const uint32_t ib = rdl32(ibase_r, oi), ie = ib + rdl32(nit_r, oi);
                const uint32_t a = max(lo, ib) - ib, b = min(hi, ie) - ib;  // this wave's items of ring oi
                const uint32_t s0 = (uint32_t)S.out_tail0[oi];  // slot arithmetic mod fwd_cap (pow2)
                const __amdgpu_buffer_rsrc_t ro = mk_rsrc(reinterpret_cast<void*>(ORING(oi)), oring_bytes);
                uint32_t i = a + (uint32_t)lane;
                uint32_t r = div_small(i, qmagic), q = i - r * nq;
                for (; i < b; i += 256u) {
                    uint32_t rr[4], qq[4], e[4];
                    rr[0] = r;
                    qq[0] = q;
#pragma unroll
                    for (int u = 1; u < 4; u++) {
                        rr[u] = rr[u - 1] + dr;
                        qq[u] = qq[u - 1] + dq;
                        if (qq[u] >= nq) { qq[u] -= nq; rr[u]++; }
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) e[u] = i + 64u * u < b ? (uint32_t)OL(oi, rr[u]) : (uint32_t)kBigFlag;
                    u32x4 x[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const bool v = !(e[u] & kBigFlag) && qq[u] < ((e[u] >> 9) & 0x3fu);
                        x[u] = u32x4{0u, 0u, 0u, 0u};
                        if (v) x[u] = *reinterpret_cast<const u32x4*>(stage + __umul24(e[u] & 0x1ffu, stg_msg) + (qq[u] << 4));
                        e[u] = v ? 1u : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (e[u]) st_ring(ro, __umul24((s0 + rr[u]) & fcap_m, stride) + (qq[u] << 4), x[u], sys);
                    r = rr[3] + dr;
                    q = qq[3] + dq;
                    if (q >= nq) { q -= nq; r++; }
                }
            }
            if (admitted && !isbig && kind == K_RING && tag == TAG_BCAST) {  // pickup: checksum (+ log payload)
                const uint32_t nch = (kHdr + len + 15u) >> 4;
                acc_sum += chunk_mix(0xFFFFFFFFu, u32x4{(uint32_t)origin, id, TAG_BCAST, len});
                for (uint32_t q = 1; q < nch; q++) {
                    const u32x4 v = *reinterpret_cast<const u32x4*>(STG(c, q));
                    acc_sum += chunk_mix(q - 1u, v);
                    if (logidx != ~0u)
                        st_sys16(P.log_payload + ((size_t)lr * P.log_cap + logidx) * P.log_stride + 16u * (q - 1), v);
                }
            }


            // ---------------- G3: large messages, 64 x 16 B per wave store instruction.  The out-rings'
            // bases and start tails lane-distributed (lane oi), a message's slot positions read with one
            // LDS load per block (lane j): the per-(block, out-ring) work is register-only -- it was a
            // chain of dependent LDS loads, ~400 cycles per out-ring per block with one wave per SIMD
            if (nbig) {
                // (4 waves: the large-slot kernel; the 8-wave kernel, where large messages are rare, keeps
                // the LDS reads -- it has no registers to spare)
                constexpr bool kRegs = W == 4;
                const uint32_t ot0_r = kRegs && lane < nout ? (uint32_t)S.out_tail0[lane] : 0u;  // mod fwd_cap (pow2)
                const uint64_t oring_r = kRegs && lane < nout ? t.out_ring[lane >> 1][lane & 1] : 0ull;
#define G3_SLOT(oi) (kRegs ? rdl32(ot0_r, oi) + rdl32(posr, (oi) >> 1) : (uint32_t)S.out_tail0[oi] + S.pos[cc][(oi) >> 1])
#define G3_RING(oi) (kRegs ? rdl64(oring_r, oi) : ORING(oi))
                uint32_t cur = 0;  // the half staged for this round
                for (;;) {
                    const bool more = S.bm < nbig;  // uniform: S.bm was last written before a barrier
                    if (more && pipe) {
                        BAR();  // every wave is done with the other half's blocks (stage2 and blk_*)
                        plan_big(cur ^ 1u);
                        BAR();
                        issue_big(cur ^ 1u);  // in flight while this round's half is stored
                    }
                    const uint32_t nblk = S.nblk2[cur];
                    for (uint32_t b0 = (uint32_t)w; b0 < nblk; b0 += kWaves) {
                        const uint32_t b = cur * hg + b0;
                        const uint32_t cc = S.blk_c[b], qw = S.blk_q0[b], q0b = qw & 0xffffu;
                        const CandL& cl = S.cand[cc];
                        const uint32_t blen = cl.w2 & 0xffffu, pch = (blen + 15u) >> 4;  // payload chunks
                        const uint32_t nsub = min(gsub, (pch - q0b + 63u) >> 6);     // uniform
                        const uint32_t rly = cl.relay;
                        const uint32_t posr = kRegs && lane < sll ? (uint32_t)S.pos[cc][lane] : 0u;  // slot in out-ring (j, vc)
                        // the header (slot chunk 0) from registers, by lane 0 of the message's first group
                        const bool hdr = q0b == 0u && lane == 0;
                        const uint32_t hw2 = cl.w2 & 0xff00ffffu;
                        const bool bc = cl.kind == K_RING && ((cl.w0 >> 16) & 0xffu) == TAG_BCAST;
                        if (bc && hdr) acc_sum += chunk_mix(0xFFFFFFFFu, u32x4{cl.w0 & 0xffffu, cl.id, TAG_BCAST, blen});
                        if (PULL_ON && rly != ~0u && q0b == 0u) {
                            // pulled on: each child gets header (kRefMark) + reference to my relay copy
                            const u32x4 hv = lane == 0 ? u32x4{cl.w0, cl.id, hw2 | (kRefMark << 16), cl.t0}
                                                       : u32x4{rly, ~rly, kRefMagic, 0u};
                            for (uint32_t a2 = (uint32_t)uni((int)cl.need); a2; a2 &= a2 - 1) {
                                const int oi = __builtin_ctz(a2);
                                const uint32_t slot = G3_SLOT(oi);
                                const __amdgpu_buffer_rsrc_t ro = mk_rsrc(reinterpret_cast<void*>(G3_RING(oi)), oring_bytes);
                                if (lane <= 1) st_ring(ro, (slot & fcap_m) * P.fwd_stride + 16u * lane, hv, sys);
                            }
                        }
                        // the group's units two at a time (registers: 4 x 16 B live across the out-ring walk)
                        for (uint32_t u0 = 0; u0 < nsub; u0 += kPair) {  // uniform
                            u32x4 vv[kPair];  // payload chunk q0 + lane + 64 (u0 + u)
#pragma unroll
                            for (uint32_t u = 0; u < kPair; u++)
                                if (u0 + u < nsub) vv[u] = *reinterpret_cast<const u32x4*>(stage2 + ((qw >> 16) + u0 + u) * 1024u + 16u * lane);
                            const uint32_t pq = q0b + lane + 64u * u0;
                            if (PULL_ON && rly != ~0u) {
#pragma unroll
                                for (uint32_t u = 0; u < kPair; u++)  // the relay copy (slot chunks 1 ..)
                                    if (u0 + u < nsub && pq + 64u * u < pch) st_ring(rf, rly + 16u * (pq + 64u * u + 1u), vv[u], sys);
                            } else {
                                const u32x4 hv = u32x4{cl.w0, cl.id, hw2 | (kSlotMark << 16), cl.t0};
                                for (uint32_t a2 = (uint32_t)uni((int)cl.need); a2; a2 &= a2 - 1) {  // uniform loop
                                    const int oi = __builtin_ctz(a2);
                                    const uint32_t slot = G3_SLOT(oi);
                                    const __amdgpu_buffer_rsrc_t ro = mk_rsrc(reinterpret_cast<void*>(G3_RING(oi)), oring_bytes);
                                    const uint32_t s0 = (slot & fcap_m) * P.fwd_stride;
#pragma unroll
                                    for (uint32_t u = 0; u < kPair; u++)
                                        if (u0 + u < nsub && pq + 64u * u < pch) st_ring(ro, s0 + 16u * (pq + 1u) + 1024u * u, vv[u], sys);
                                    if (hdr && u0 == 0u) st_ring(ro, s0, hv, sys);
                                }
                            }
                            if (bc) {
#pragma unroll
                                for (uint32_t u = 0; u < kPair; u++) {
                                    const uint32_t pp = pq + 64u * u;
                                    if (u0 + u < nsub && pp < pch) {
                                        acc_sum += chunk_mix(pp, vv[u]);
                                        if (cl.logidx != ~0u && 16u * (pp + 1u) <= P.log_stride)
                                            st_sys16(P.log_payload + ((size_t)lr * P.log_cap + cl.logidx) * P.log_stride + 16u * pp, vv[u]);
                                    }
                                }
                            }
                        }
                    }
                    if (!more) break;
                    if (pipe) {
                        cur ^= 1u;
                    } else {  // one stage2 block: load -> store -> wait, round by round
                        BAR();
                        plan_big(cur);
                        BAR();
                        issue_big(cur);
                    }
                    big_drain();  // the next half's loads (and this round's stores: vmcnt is in order)
                    ACQ_NEXT();
                }
#undef G3_SLOT
#undef G3_RING
            }
            if (lat_deliv) {  // latency program: the last of N-1 pickups completes the round
                const uint32_t old = sys ? __hip_atomic_fetch_add(&P.lat_count[id], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                         : atomicAdd(&P.lat_count[id], 1u);
                if (old + 1u == (uint32_t)(P.n - 1)) {
                    tl_mark(P, id, TL_ROUND);
                    P.lat_out[id] = (uint64_t)lat_tn;  // one clock only when the world is one part
                    if (sys) __hip_atomic_store(P.lat_round, id + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    else __hip_atomic_store(P.lat_round, id + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            PST(5, 7);
        }

        // every store of this iteration (payloads, votes, pickup records) drained, so the producer
        // counters are published at the end of this iteration, not after the next poll
        if (eager && (C != 0 || S.vtot != 0)) {
            VM_DRAIN();
            BAR();
        }
        // ---------------- consume (wave 0): in-ring prefixes, producer counts, bookkeeping
        if (w == 0) {
            if constexpr (BULK) flush_posts(S.b, P, lane);  // posts of an iteration without phase F (phase C's)
            if (lane < n_in2) {
                const uint32_t bse = rbase_r, tk = rtake_r, fb = S.first_bad[lane];
                if (fb < bse + tk) n_stalls++;  // lane 0's copy is flushed (sum over lanes at exit)
                uint32_t adm = fb == 0xffffffffu ? tk : (fb > bse ? fb - bse : 0u);
                if (adm > tk) adm = tk;
                in_head_r += adm;
                if (adm < tk) win_r = max(adm + adm / 2u, 16u);
                else if (adm == tk && tk == win_r) win_r = min(2u * win_r, (uint32_t)kMaxCand);
                if (PMODE(MODE_PROF)) atomicAdd((unsigned long long*)&S.dbg[1], (unsigned long long)adm);
            }
            PSX(4);
            if (eager) {
                if (lane < n_in2 && in_head_r != PUB_IN) { PUB_IN = in_head_r; pub64(IHPTR, in_head_r, sys); }
                if (lane < n_in) {
                    const uint64_t vt = S.vout_tail[lane];
                    if (vt != PUB_VOUT) { PUB_VOUT = vt; pub64(VTPTR, vt, sys); }
                }
            }
            if (lane < nout) {
                out_tail_r += noi_r;
                // pull worlds: this iteration's relay slots are released once the children consumed up
                // to these tails (coalesced into the newest record when all kRelQ are pending)
                if (PULL_ON && S.ref_any) {
                    const uint32_t qn = S.rq_n;
                    const uint32_t e = (S.rq_h + (qn == (uint32_t)kRelQ ? qn - 1u : qn)) % (uint32_t)kRelQ;
                    S.rq_out[e][lane] = out_tail_r;
                }
            }
            if (PULL_ON && lane == 0) {
                if (S.ref_any) {
                    const uint32_t qn = S.rq_n;
                    const uint32_t e = (S.rq_h + (qn == (uint32_t)kRelQ ? qn - 1u : qn)) % (uint32_t)kRelQ;
                    S.relay_tail += min(S.relay_n, S.relay_free);  // the requests beyond the free slots were pushed
                    S.rq_relay[e] = S.relay_tail;
                    if (qn < (uint32_t)kRelQ) S.rq_n = qn + 1u;
                }
                S.relay_n = 0;
                S.ref_any = 0;
            }
            if (lane < nout) {
                // this iteration's stores are drained (see above): publish now, not after the next
                // poll -- one poll round trip less per hop
                if (eager && out_tail_r != PUB_OUT) { PUB_OUT = out_tail_r; pub64(OTPTR, out_tail_r, sys); }
                if ((PMODE(MODE_PROF | MODE_HIST)) == MODE_PROF) {  // per out-ring: admitted, free at start
                    S.hist[32 + lane] += noi_r;
                    S.hist[64 + lane] += S.ofree[lane] >> 4;
                }
                if (PMODE(MODE_PROF))
                    atomicMax((unsigned long long*)&S.dbg[7], (unsigned long long)(out_tail_r - S.out_tail0[lane] +
                                                                                   (P.fwd_cap - S.ofree[lane])));
            }
            PSX(5);
            if constexpr (BULK) {
                if (nstorm) {  // the admitted prefix of the storm window used its bulk sequences
                    const uint32_t fb = S.first_bad[kGroupLocal + K_STORM];
                    uint32_t adm = fb == 0xffffffffu ? nstorm : (fb > storm_base ? fb - storm_base : 0u);
                    if (adm > nstorm) adm = nstorm;
                    const uint64_t bm = __ballot((uint32_t)lane < adm && S.b.bq[lane] != ~0u);
                    if (lane == 0) S.b.bulk_q += (uint32_t)__popcll(bm);
                }
            }
            if (lane == 0) {
                if (nstorm) {
                    const uint32_t fb = S.first_bad[kGroupLocal + K_STORM];
                    uint32_t adm = fb == 0xffffffffu ? nstorm : (fb > storm_base ? fb - storm_base : 0u);
                    if (adm > nstorm) adm = nstorm;
                    sched_next += adm;
                }
                if (host) {
                    if (S.nh) {
                        const uint32_t fb = S.first_bad[kGroupLocal + K_HOST];
                        uint32_t adm = fb == 0xffffffffu ? S.nh : (fb > S.hbase ? fb - S.hbase : 0u);
                        if (adm > S.nh) adm = S.nh;
                        S.hin_head = S.hhead + adm;
                    }
                    if (S.ev_n) {
                        S.pk_tail += S.ev_n;
                        S.log_count += S.ev_n;
                        S.ev_n = 0;
                        pub64_sys(&hctl[kHctlPkTail], S.pk_tail);
                    }
                }
                n_iter++;
                if (S.progressed) {  // the clock is read on the 1st and every 64th idle iteration only
                    n_busy++;
                    idle_n = 0;
                } else if ((++idle_n & 63u) == 1u) {
                    const uint64_t tn = now_ticks();
                    if (idle_n == 1) idle_since = tn;
                    else if (tn - idle_since > P.timeout_ticks) set_error(S, P, ERR_TIMEOUT, 0);
                }
                if ((n_iter & 1023u) == 0 && now_ticks() - t_start > P.deadline_ticks) set_error(S, P, ERR_TIMEOUT, 1);
                bool done = true;
                if (PMODE(MODE_STORM)) done &= sched_next == sched_n;
                if (PMODE(MODE_STORM | MODE_LAT)) done &= (int64_t)S.bcast_delivered == expect_bcast;
                if (PMODE(MODE_LAT)) done &= S.lat_pos >= S.lat_pos_n;
                if ((PMODE(MODE_IAR)) && !host) {
                    bool idle = true;
                    for (uint32_t k = 0; k < P.pend_slots; k++) idle &= S.own_state[k] == 0u;
                    done &= (int64_t)S.own_iter == S.own_n && idle && (int64_t)S.dec_delivered == S.expect_dec;
                }
                if (host) done = S.quit != 0;
                if (S.error == ERR_TIMEOUT) done = true;
                if (peer_failed) done = true;  // another rank failed: stop everyone
                done_w0 = done;
            }
            done_w0 = __builtin_amdgcn_readfirstlane((int)done_w0) != 0;  // lane 0 updated these
            sched_next = (int64_t)uni64((uint64_t)sched_next);
            // (BULK: pending receptions are polled in the spin, bulk_eval)
            idle_prev = C == 0 && S.vtot == 0 && !done_w0 && !(PMODE(MODE_NOSPIN));
        }
        PROF_STAMP(6);
    }
#undef STG
#undef OL
#undef OTPTR
#undef IHPTR
#undef VHPTR
#undef VTPTR
#undef ORING
#undef PUB_IN
#undef PUB_OUT
#undef PUB_VIN
#undef PUB_VOUT

    // ---------------- flush statistics
    if constexpr (BULK) {
        if (tid == 0 && !(P.mode & (MODE_PROF | MODE_TL | MODE_HOPPROF))) {  // diagnostics in stats.dbg: pending receptions at exit
            const uint32_t nb = S.b.nbact;
            S.dbg[0] = ((uint64_t)S.b.bulk_q << 32) | nb;
            for (uint32_t i = 0; i < 3 && i < nb; i++) {
                const uint32_t e = S.b.bact[i];
                const uint32_t tf = bulk_tcount(P, bulk_flags(P, me, (int)(e / bsl), e % bsl), sys);
                const uint32_t sf = bflag_ld(bulk_flags(P, me, (int)(e / bsl), e % bsl), sys);
                S.dbg[1 + 2 * i] = ((uint64_t)e << 32) | bpend[e].ntiles;
                S.dbg[2 + 2 * i] = ((uint64_t)sf << 32) | tf;
            }
            for (uint32_t i = 0; i < bsl && i < 1; i++) S.dbg[7] = S.b.sdone[0] | (S.b.sdone[bsl > 1 ? 1 : 0] << 32);
        }
    }
    __syncthreads();
    if (w == 0) atomicAdd((unsigned long long*)&S.stalls, (unsigned long long)n_stalls);
    atomicAdd((unsigned long long*)&P.stats[lr].bcast_sum, acc_sum);
    for (int i = tid; i < kHistBins; i += kBlock) P.stats[lr].hist[i] = S.hist[i];
    if (tid < 8) { P.stats[lr].prof[tid] = S.prof[tid]; P.stats[lr].dbg[tid] = S.dbg[tid]; }
    if constexpr (BULK) {
        if (tid == 0) {  // after every job this workgroup posted: the movers may stop once all did
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            atomicAdd((unsigned long long*)&P.jctl[kJctlExited], 1ull);
        }
    }
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
        st.iterations = n_iter;
        st.busy_iterations = n_busy;
        st.stalls = S.stalls;
        st.unmarked_slots = S.stale;
        st.log_count = S.log_count;
        st.t_start = t_start;
        st.t_end = now_ticks();
        st.error = S.error;
        st.error_aux = S.error_aux;
        if (host && (PMODE(MODE_HDIAG)))
            for (int i = 0; i < 8; i++) pub64_sys(&hctl[kHctlDiag + i], S.hd[i]);
        if (host) pub64_sys(&hctl[kHctlState], 2ull);  // this rank stopped serving
    }
}

}  // namespace rlo

// C-ABI launch shims used by rlo_world.cpp.  variant: 8 = 8 waves, 4 = 4 waves, 5 = 4 waves with
// bulk messages (mover workgroups + mixed storm lengths); the Shared / LDS layout depends on it.  A
// program with doorbells (MODE_LL: latency, IAR, host service) runs the doorbell instantiation of its
// variant, the storm the one without (its registers untouched)
template <int W, bool B, bool L, bool H = false, uint32_t PM = rlo::kPmAll>
static hipError_t grant_dyn_lds(size_t dyn_lds) {
    static size_t granted = 0;
    if (dyn_lds > granted) {  // > 64 KiB of dynamic LDS must be requested explicitly
        hipError_t e = hipFuncSetAttribute((const void*)rlo::rlo_progress_kernel<W, B, L, H, PM>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn_lds);
        if (e != hipSuccess) return e;
        granted = dyn_lds;
    }
    return hipSuccess;
}

template <int W, bool B, bool L, bool H = false, uint32_t PM = rlo::kPmAll>
static hipError_t launch_v(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream) {
    hipError_t e = grant_dyn_lds<W, B, L, H, PM>(dyn_lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((rlo::rlo_progress_kernel<W, B, L, H, PM>), dim3(blocks), dim3(64 * W), dyn_lds, stream, *p);
    return hipGetLastError();
}

template <int W, bool B, bool L, bool H = false, uint32_t PM = rlo::kPmAll>
static hipError_t occ_one(int* blocks, size_t dyn_lds) {
    hipError_t e = grant_dyn_lds<W, B, L, H, PM>(dyn_lds);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, rlo::rlo_progress_kernel<W, B, L, H, PM>, 64 * W, dyn_lds);
}

// the occupancy of <W, B, L, H> = the least over its general instantiation and every program-specialised one that
// rlo_launch_progress launches for it (PMs...): co-residency is decided from this answer, so a specialised kernel
// that fell below its general twin would leave workgroups of a persistent launch unscheduled
template <int W, bool B, bool L, bool H, uint32_t... PMs>
static hipError_t occ_v(int* blocks, size_t dyn_lds) {
    hipError_t e = occ_one<W, B, L, H>(blocks, dyn_lds);
    if (e != hipSuccess) return e;
    const hipError_t es[] = {hipSuccess, [&]() -> hipError_t {
        int b = 0;
        const hipError_t r = occ_one<W, B, L, H, PMs>(&b, dyn_lds);
        if (r == hipSuccess && b < *blocks) *blocks = b;
        return r;
    }()...};
    for (hipError_t x : es)
        if (x != hipSuccess) return x;
    return hipSuccess;
}

// programs that hold proposals in a world with HBM pending tables run the PH instantiations (no bulk
// worlds: their N x B bound keeps the table small)
static bool wants_ph(const rlo::Params* p) {
    return p->pend_hbm != nullptr && (p->mode & (rlo::MODE_IAR | rlo::MODE_HOST)) != 0;
}

// The kernels of the device programs the bench times are specialised by program (PM): 8 waves -- the storm
// (no doorbells), the latency program and the iar program (doorbells; the iar one with the LDS or the HBM
// pending table); bulk worlds -- the latency program (C3) and the storm (C5); and the host service the drop-in
// runs (doorbells; every variant, LDS or HBM tables).  The host's occupancy answer (rlo_occupancy*) is the least over the
// general instantiation and these; the Makefile guard holds every 8-wave instantiation to 2 waves per SIMD.
extern "C" hipError_t rlo_launch_progress(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream, int variant) {
    const bool ll = (p->mode & rlo::MODE_LL) != 0;
    const uint32_t prog = p->mode & (rlo::MODE_STORM | rlo::MODE_LAT | rlo::MODE_IAR | rlo::MODE_HOST);
    const bool hll = ll && (prog & rlo::MODE_HOST) != 0;  // the drop-in's host service (HOST | IAR) with doorbells
    if (wants_ph(p) && variant != 5) {
        if (variant == 8) {
            if (ll && prog == rlo::MODE_IAR) return launch_v<8, false, true, true, rlo::kPmIar>(p, blocks, dyn_lds, stream);
            if (hll) return launch_v<8, false, true, true, rlo::kPmHost>(p, blocks, dyn_lds, stream);
            return ll ? launch_v<8, false, true, true>(p, blocks, dyn_lds, stream) : launch_v<8, false, false, true>(p, blocks, dyn_lds, stream);
        }
        if (hll) return launch_v<4, false, true, true, rlo::kPmHost>(p, blocks, dyn_lds, stream);
        return ll ? launch_v<4, false, true, true>(p, blocks, dyn_lds, stream) : launch_v<4, false, false, true>(p, blocks, dyn_lds, stream);
    }
    if (variant == 8) {
        if (ll && prog == rlo::MODE_LAT) return launch_v<8, false, true, false, rlo::kPmLat>(p, blocks, dyn_lds, stream);
        if (ll && prog == rlo::MODE_IAR) return launch_v<8, false, true, false, rlo::kPmIar>(p, blocks, dyn_lds, stream);
        if (!ll && prog == rlo::MODE_STORM) return launch_v<8, false, false, false, rlo::kPmStorm>(p, blocks, dyn_lds, stream);
        if (hll) return launch_v<8, false, true, false, rlo::kPmHost>(p, blocks, dyn_lds, stream);
        return ll ? launch_v<8, false, true>(p, blocks, dyn_lds, stream) : launch_v<8, false, false>(p, blocks, dyn_lds, stream);
    }
    if (variant == 5) {  // bulk worlds: the C3 leg's latency program (doorbells) and the C5 storm, specialised too
        if (ll && prog == rlo::MODE_LAT) return launch_v<4, true, true, false, rlo::kPmLat>(p, blocks, dyn_lds, stream);
        if (!ll && prog == rlo::MODE_STORM) return launch_v<4, true, false, false, rlo::kPmStorm>(p, blocks, dyn_lds, stream);
        if (hll) return launch_v<4, true, true, false, rlo::kPmHost>(p, blocks, dyn_lds, stream);
        return ll ? launch_v<4, true, true>(p, blocks, dyn_lds, stream) : launch_v<4, true, false>(p, blocks, dyn_lds, stream);
    }
    if (hll) return launch_v<4, false, true, false, rlo::kPmHost>(p, blocks, dyn_lds, stream);
    return ll ? launch_v<4, false, true>(p, blocks, dyn_lds, stream) : launch_v<4, false, false>(p, blocks, dyn_lds, stream);
}

extern "C" size_t rlo_kernel_static_lds(int variant) {
    if (variant == 8) return sizeof(rlo::Shared<8, false>);
    if (variant == 5) return sizeof(rlo::Shared<4, true>);
    return sizeof(rlo::Shared<4, false>);
}

// variant | RLO_VARIANT_PH (16): the PH instantiation of variant 8 / 4
extern "C" hipError_t rlo_occupancy(int* blocks, size_t dyn_lds, int variant) {
    if (variant == (8 | 16)) return occ_v<8, false, false, true>(blocks, dyn_lds);
    if (variant == (4 | 16)) return occ_v<4, false, false, true>(blocks, dyn_lds);
    if (variant == 8) return occ_v<8, false, false, false, rlo::kPmStorm>(blocks, dyn_lds);
    if (variant == 5) return occ_v<4, true, false, false, rlo::kPmStorm>(blocks, dyn_lds);
    return occ_v<4, false, false, false>(blocks, dyn_lds);
}

// the doorbell instantiation of a variant: the 4-wave ones may take more than 256 registers (one wave
// per SIMD: worlds whose ranks have a CU each), so a world gets doorbells only where this answer covers it
extern "C" hipError_t rlo_occupancy_ll(int* blocks, size_t dyn_lds, int variant) {
    if (variant == (8 | 16)) return occ_v<8, false, true, true, rlo::kPmIar, rlo::kPmHost>(blocks, dyn_lds);
    if (variant == (4 | 16)) return occ_v<4, false, true, true, rlo::kPmHost>(blocks, dyn_lds);
    if (variant == 8) return occ_v<8, false, true, false, rlo::kPmLat, rlo::kPmIar, rlo::kPmHost>(blocks, dyn_lds);
    if (variant == 5) return occ_v<4, true, true, false, rlo::kPmLat, rlo::kPmHost>(blocks, dyn_lds);
    return occ_v<4, false, true, false, rlo::kPmHost>(blocks, dyn_lds);
}
