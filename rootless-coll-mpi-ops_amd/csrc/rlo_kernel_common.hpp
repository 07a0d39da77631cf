// rlo_kernel_common.hpp -- device types and helpers shared by the persistent progress kernel (rlo_kernel.hip) and
// the hop kernel (rlo_hop.hip): ring / doorbell access, topology (the skip-ring child sets), the device judges, the
// event log / pickup records, votes, generated payloads.  Every helper cites the reference line it restates.
#pragma once
#include <hip/hip_runtime.h>

#include "rlo_device.hpp"

namespace rlo {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static constexpr int kAuxSc1 = 16;  // cache policy: sc1 (agent scope, write-through / L1 bypass)
static constexpr uint32_t kGolden32 = 0x9E3779B9u;
static constexpr uint64_t kGolden64 = 0x9E3779B97F4A7C15ull;
static constexpr int kPass = 64;  // messages per wave per iteration
static constexpr uint32_t kIdleSpin = 256;  // tight re-polls after an idle iteration (~0.1 ms at most)
static constexpr int kRelQ = 16;  // pull worlds: relay-ring release records (coalesced when full)
// the doorbell pass's scratch in the stage area (>= 4 KiB: 256 candidates x 16 B): bells' data, vote bells'
// data, loaded votes, loaded ring heads, a message's judge copy
static constexpr uint32_t kLLBell = 0, kLLBellVote = 1024, kLLVote = 1152, kLLRing = 2176, kBellJudge = 3328;
static constexpr uint32_t kLLVotes = 4;  // votes per child a doorbell pass takes
// host mode: the pass also takes up to kLLCmds host commands, command s's chunk q loaded at kLLCmd + 16 (8 s + q)
// (the stage area is >= 5 KiB there: 256 candidates x nsmall >= 2 chunks)
static constexpr uint32_t kLLCmd = 4096, kLLCmds = 8;
// the command doorbell of the next expected command (rlo_shm.hpp ll_cmd_put), as polled: 16 lanes x 16 B
static constexpr uint32_t kLLCmdBell = 5120;
// lone(): a proposal held for the host's verdict (nothing consumed); kAsked: its judge request was written now
static constexpr uint32_t kHeld = 0xFFFFFFFEu, kAsked = 0xFFFFFFFDu;

enum CandKind : uint32_t { K_RING = 0, K_STORM = 1, K_PROP = 2, K_DEC = 3, K_LAT = 4, K_HOST = 5, K_BAD = 7 };
// PendState.valid: proposal held at a non-originator / host-judge progress (MODE_HOST)
enum PendValid : uint8_t { PS_NONE = 0, PS_ACTIVE = 1, PS_JREQ = 2, PS_JYES = 3, PS_JNO = 4 };
static constexpr int kGroupLocal = 2 * kMaxIn;  // groups [0, 64) = in-rings (k*2+vc); 64.. local kinds
static constexpr int kGroups = kGroupLocal + 8;
static constexpr uint16_t kBigFlag = 0x8000u;

struct PendState {      // a proposal held at a non-originator (queue_iar_pending, :1138)
    int32_t pid;
    uint32_t word;      // votes received (low 16 b) | zero votes (high 16 b)
    uint16_t parent_k;  // in-edge the proposal came from (the vote goes back on it)
    uint8_t needed;     // fwd_send_cnt (:694)
    uint8_t valid;
    uint32_t pseq;      // proposal sequence (low 8 b) | proposal data_len << 8
};

// ------------------------------------------------------------------ helpers

// Workgroup barrier without the global-memory fence of __syncthreads() (which would wait for
// every in-flight payload store): only this wave's LDS results must have landed.  The "memory"
// clobbers keep the compiler from moving memory accesses across it.
#define BAR()                                              \
    do {                                                   \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
        __builtin_amdgcn_s_barrier();                      \
        asm volatile("" ::: "memory");                     \
    } while (0)
#define VM_DRAIN() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
// agent-scope acquire after LDS-DMA of ring slots (large messages), without the leading vmcnt(0)
// of __builtin_amdgcn_fence: callers have drained their loads (MODE_NOACQ: diagnostic A/B, unsafe)
#define ACQ_NEXT()                                                             \
    do {                                                                       \
        if (!(P.mode & MODE_NOACQ)) asm volatile("buffer_inv sc1" ::: "memory"); \
    } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSc1);
}
// Branch-free polls.  A poll written as `x = 0; if (lane < k) x = load(...)` makes the compiler copy the loaded value
// into x's register at the join -- behind a vmcnt wait -- so a poll of several such loads became two or three round
// trips in a row (counters, then bells, then vote bells: rlo_kernel.isa, VERDICT r5 "next" 1).  Here every lane
// issues the load; a lane with nothing to poll reads at kOob, past the resource's end, where the hardware's range
// check returns zeros.  The loads of a poll then leave back to back and one wait covers them all
constexpr uint32_t kOob = 0xFFFFFFF0u;
__device__ __forceinline__ uint64_t ld64_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxSc1);
    return (uint64_t)v.x | ((uint64_t)v.y << 32);
}
__device__ __forceinline__ uint64_t ld64_sys(__amdgpu_buffer_rsrc_t r, uint32_t off) {  // system scope (sc0 sc1)
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxSc1 | 1);
    return (uint64_t)v.x | ((uint64_t)v.y << 32);
}
__device__ __forceinline__ uint32_t ld32_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kAuxSc1);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSc1);
}
__device__ __forceinline__ uint8_t ld8_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, kAuxSc1);
}
__device__ __forceinline__ __attribute__((address_space(3))) void* lds_ptr(uint8_t* p) {
    return (__attribute__((address_space(3))) void*)(p);
}
// LDS-DMA: 64 lanes x 16 B of the forward region -> LDS (lane i lands at dst + 16 i; dst uniform)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint8_t* dst, uint32_t off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds_ptr(dst), 16, off, 0, 0, kAuxSc1);
}
__device__ __forceinline__ uint64_t poll64(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Stores through addresses the kernel loads from memory (the topology's remote counters and bells, the vote rings) are
// made through GLOBAL pointers: a generic (flat) store counts in lgkmcnt as well as vmcnt, so every later LDS wait of
// the wave -- s_waitcnt lgkmcnt(0) before the next LDS read -- waited for the store to reach memory (a counter publish
// or a vote held the next hop's LDS work up for a whole memory round trip)
typedef __attribute__((address_space(1))) uint64_t gu64;
__device__ __forceinline__ gu64* gptr64(uint64_t addr) { return (gu64*)addr; }
// a counter store into a (possibly peer) part: agent scope inside one GPU, system scope when
// the world spans GPUs (the store then crosses xGMI into the peer's HBM)
__device__ __forceinline__ void pub64(uint64_t addr, uint64_t v, bool sys) {
    gu64* p = gptr64(addr);
    if (sys) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B slot store into a remote ring through a wave-uniform ring base (buffer rsrc built on the fly)
__device__ __forceinline__ void st_ring(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v, bool sys) {
    if (sys) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSc1 | 1);
    else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSc1);
}
// 16-B write-through store that reaches host memory (pinned pickup rings) or HBM for the log
__device__ __forceinline__ void st_sys16(void* p, u32x4 v) {
    // two 8-B system-scope stores (sc0 sc1: write-through to host memory / visible to every XCD).
    // Not inline asm: the compiler cannot see an asm store's pending reads of its address and data
    // registers and may reuse them at once -- job records were seen with a neighbour's words in them
    gu64* q = gptr64(reinterpret_cast<uint64_t>(p));  // (global, not flat: see gu64)
    __hip_atomic_store(q, (uint64_t)v.x | ((uint64_t)v.y << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 1, (uint64_t)v.z | ((uint64_t)v.w << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 16-B command-slot load from pinned host memory (written by the host CPU)
__device__ __forceinline__ u32x4 ld_sys(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSc1 | 1);
}
__device__ __forceinline__ uint64_t poll64_sys(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The host service's wave-1 poller reads pinned host memory through the SCALAR data path (s_load ... glc: a miss in
// the scalar cache every time, so each poll sees the host's latest stores); only a command longer than 16 payload
// bytes, once seen, has its other chunks read with vector loads.  Its vector loads to host memory held up
// the other waves' VRAM loads on the CU: a wave timing dependent 16-B uncached VRAM loads saw 0.134 us per load
// beside an idle wave, 0.672 us beside one polling host memory with vector loads, 0.136 us beside one polling it with
// scalar loads (tools/probe/poll_interference.hip, profiles/r5_poll_interference.txt) -- and wave 0's doorbell polls
// are such loads.  Loads only: nothing is ever written through the scalar cache.
typedef uint32_t su16 __attribute__((ext_vector_type(16)));
// host-service kernels: the doorbell's first 160 B (chunks 0-4: a command with <= 64 payload bytes -- the drop-in's
// small bcasts and proposals -- in one round trip) and the two host words
typedef uint32_t su8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void spoll_cmd5(const uint8_t* slot, const uint64_t* w0, const uint64_t* w1, su16& a, su16& b,
                                           su8& c, uint64_t& x0, uint64_t& x1) {
    asm volatile(
        "s_load_dwordx16 %0, %5, 0x0 glc\n\t"
        "s_load_dwordx16 %1, %5, 0x40 glc\n\t"
        "s_load_dwordx8 %2, %5, 0x80 glc\n\t"
        "s_load_dwordx2 %3, %6, 0x0 glc\n\t"
        "s_load_dwordx2 %4, %7, 0x0 glc\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(a), "=&s"(b), "=&s"(c), "=&s"(x0), "=&s"(x1)
        : "s"(slot), "s"(w0), "s"(w1)
        : "memory");
}
// the first 64 B of a command doorbell (chunks 0-1: a verdict, a judge(NULL) verdict, the header of any command)
// and two host words (command tail, pickup head), one round trip
__device__ __forceinline__ void spoll_cmd(const uint8_t* slot, const uint64_t* w0, const uint64_t* w1, su16& a,
                                          uint64_t& x0, uint64_t& x1) {
    asm volatile(
        "s_load_dwordx16 %0, %3, 0x0 glc\n\t"
        "s_load_dwordx2 %1, %4, 0x0 glc\n\t"
        "s_load_dwordx2 %2, %5, 0x0 glc\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(a), "=&s"(x0), "=&s"(x1)
        : "s"(slot), "s"(w0), "s"(w1)
        : "memory");
}
__device__ __forceinline__ void pub64_sys(uint64_t* p, uint64_t v) {
    __hip_atomic_store(gptr64(reinterpret_cast<uint64_t>(p)), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t poll32(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }
// MODE_TL (the timeline of a latency round) exists in the diagnostics build only (make DIAG=1, -DRLO_DIAG): its
// clocks and probes sit on wave 0's hop path, and the product kernel carries none of that code
#ifdef RLO_DIAG
#define TL_ON(P) (((P).mode & MODE_TL) != 0u)
#else
#define TL_ON(P) false
#endif
// MODE_TL: the clock of event `ev` of latency round r (rlo_device.hpp kTlGlobal; the latest writer wins)
// (global pointers: a generic store counts in lgkmcnt, and the next clock read -- s_memrealtime, an lgkmcnt wait --
// then waited for the store to reach memory: the probes read ~0.8 us of their own stores into the hop)
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ void tl_mark(const Params& P, uint32_t r, uint32_t ev) {
    if (TL_ON(P) && r < P.tl_rounds)
        __hip_atomic_fetch_max((gu32*)(P.tl + r * (kTlGlobal + kTlCols * P.n_local) + ev), (uint32_t)now_ticks(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// MODE_TL: per-rank column col (rlo_device.hpp TlCol) of local rank lr for round r := v
__device__ __forceinline__ void tl_put(const Params& P, uint32_t r, uint32_t col, int lr, uint32_t v) {
    if (TL_ON(P) && r < P.tl_rounds) ((gu32*)P.tl)[r * (kTlGlobal + kTlCols * P.n_local) + kTlGlobal + col * P.n_local + lr] = v;
}
__device__ __forceinline__ void tl_parent(const Params& P, uint32_t r, int lr, int from) {
    tl_put(P, r, TLC_PARENT, lr, (uint32_t)(from + 1));
}

// per-ring state lives lane-distributed in registers; a wave-uniform index reads it with v_readlane
__device__ __forceinline__ uint32_t rdl32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int l) {
    return ((uint64_t)rdl32((uint32_t)(v >> 32), l) << 32) | rdl32((uint32_t)v, l);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)(uint32_t)uni((int)(v >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)v);
}

// i / d for the small d = nsmall (<= 24) and i < 2^16: multiply-high by ceil(2^32 / d)
__device__ __forceinline__ uint32_t div_small(uint32_t i, uint32_t magic) { return magic ? __umulhi(i, magic) : i; }

// MODE_TL (wave 0): why the spin ended -- dbg[0] the last iteration was not idle, [1] spin bound, [2] the doorbell
// pass needs the full iteration, [3] 64 passes, [4] job posts queued, [5] a bulk copy complete, [6] a polled word moved
#define SPIN_WHY(k)                                           \
    do {                                                      \
        if (TL_ON(P) && lane == 0) S.dbg[(k)]++;    \
    } while (0)
// MODE_HOPPROF (diagnostics build): lane 0 of wave 0 stamps point k of a doorbell hop
#ifdef RLO_DIAG
// (the program-specialised doorbell kernels only: the general ones have no registers to spare)
#define HP(k)                                                                                  \
    do {                                                                                       \
        if constexpr (PM == kPmLat || PM == kPmIar)                           \
            if ((P.mode & MODE_HOPPROF) && lane == 0) S.hpt[(k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// ... and S.dbg[k] counts why a doorbell pass handed over to the full iteration (hop_prof.py prints them)
#define HPC(k)                                                                                 \
    do {                                                                                       \
        if constexpr (PM == kPmLat || PM == kPmIar)                           \
            if ((P.mode & MODE_HOPPROF) && lane == 0) S.dbg[(k)]++;                            \
    } while (0)
#else
#define HP(k) \
    do {      \
    } while (0)
#define HPC(k) \
    do {       \
    } while (0)
#endif
// MODE_PROF: thread 0 charges the shader cycles since the last stamp to phase `ph`
#define PROF_STAMP(ph)                                  \
    do {                                                \
        if ((P.mode & MODE_PROF) && tid == 0) {         \
            uint64_t c_ = __builtin_amdgcn_s_memtime(); \
            S.prof[ph] += c_ - S.prof_t;                \
            S.prof_t = c_;                              \
        }                                               \
    } while (0)
// RLO_PROF_SPLIT (diagnostic build): slots 1-6 split the wave-0 phases (1 publish, 2 quotas,
// 3 originations, 4 in-ring heads, 5 out-ring tails, 6 lane-0 bookkeeping); the all-wave phases go to 7
#ifdef RLO_PROF_SPLIT
#define PST(a, b) PROF_STAMP(b)
#define PSX(b) PROF_STAMP(b)
#else
#define PST(a, b) PROF_STAMP(a)
#define PSX(b) \
    do {       \
    } while (0)
#endif

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + kGolden64;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// storm payload word k (DESIGN.md "Storm workload"; the oracle's rlo_testvec.h states the same)
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

// slot mark (w2 bits 16..23 of every slot header, rlo_device.hpp): rings are zeroed at creation,
// so a staged header without the mark is a slot whose bytes were not visible yet
static constexpr uint32_t kSlotMark = 0xA5u;
// pull worlds (Params.pull): a large bcast's header carries kRefMark instead, and its first payload
// chunk is the reference {byte offset of the sender's relay slot in the sender's part, ~offset, kRefMagic, 0}
static constexpr uint32_t kRefMark = 0x5Au;
static constexpr uint32_t kRefMagic = 0x52454631u;  // "REF1": reference chunk = {off, ~off, magic, 0}

__device__ __forceinline__ uint32_t mask_bytes(uint32_t w, int keep) {  // keep the low `keep` bytes
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

// child index set j of send_list: originate (:1587) or _bc_forward (:1116-1223); sl_r = send_list
// distributed over lanes
__device__ __forceinline__ uint32_t kids_of(int me, int origin, int from, int level, int last_wall, int scc, int sll,
                                            uint32_t sl_r) {
    if (from < 0) return (1u << sll) - 1u;
    if (level <= 0) return 0u;
    if (from > last_wall) return (1u << (scc + 1)) - 1u;
    uint32_t m = 0;
    for (int j = 0; j < scc; j++)
        if (!passed_origin(me, origin, (int)rdl32(sl_r, j))) m |= 1u << j;
    return m;
}

// out-ring bits oi = 2j + vc; vc = 1 once the message has wrapped past rank N-1 (child < origin):
// the "dateline" virtual channel that keeps the ring dependency graph acyclic
__device__ __forceinline__ uint32_t need_of(uint32_t kids, int origin, int sll, uint32_t sl_r) {
    uint32_t need = 0;
    for (int j = 0; j < sll; j++)
        if ((kids >> j) & 1u) need |= 1u << (2 * j + ((int)rdl32(sl_r, j) < origin ? 1 : 0));
    return need;
}

// the same two for a wave-uniform message (the lone path): lane j tests send_list[j] at once -- three ballots
// instead of two serial loops of v_readlane + compare over the send list
__device__ __forceinline__ uint32_t spread_bits(uint32_t x) {  // bit j -> bit 2j (x < 2^16)
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
}
__device__ __forceinline__ uint32_t kids_of_u(int me, int origin, int from, int level, int last_wall, int scc, int sll,
                                              uint32_t sl_r, int lane) {
    if (from < 0) return (1u << sll) - 1u;
    if (level <= 0) return 0u;
    if (from > last_wall) return (1u << (scc + 1)) - 1u;
    return (uint32_t)__ballot(lane < scc && !passed_origin(me, origin, (int)sl_r));
}
__device__ __forceinline__ uint32_t need_of_u(uint32_t kids, int origin, int sll, uint32_t sl_r, int lane) {
    const bool kid = lane < sll && ((kids >> lane) & 1u);
    const uint32_t b1 = (uint32_t)__ballot(kid && (int)sl_r < origin);  // wrapped past rank N-1: vc 1
    const uint32_t b0 = (uint32_t)__ballot(kid && !((int)sl_r < origin));
    return spread_bits(b0) | (spread_bits(b1) << 1);
}

// latency histogram of 10 ns ticks: values < 4 exact, then 4 sub-bins per octave (to ~2^33 ticks)
__device__ __forceinline__ uint32_t hist_bin(uint64_t d) {
    if (d < 4) return (uint32_t)d;
    int o = 63 - __builtin_clzll(d);
    uint32_t b = (uint32_t)(o - 1) * 4u + (uint32_t)((d >> (o - 2)) & 3u);
    return b < kHistBins ? b : kHistBins - 1;
}

template <class SH>
__device__ __forceinline__ void set_error(SH& S, const Params& P, uint32_t code, uint32_t aux) {
    if (atomicCAS(&S.error, 0u, code) == 0u) {
        S.error_aux = aux;
        atomicCAS(P.error_flag, 0u, code);
        for (uint32_t q = 0; q < P.n_parts; q++)  // every other part stops too (they poll their own word)
            if (P.err_flag[q] != P.error_flag) __hip_atomic_store(P.err_flag[q], code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ uint32_t judge_hash(uint64_t seed, uint32_t rank, int32_t pid) {
    return (uint32_t)(splitmix64(seed ^ ((uint64_t)rank << 32) ^ (uint32_t)pid) % 1000000u);
}

// device judge registry.  arg = proposal data (data_len bytes, zero-extended: the reference's calloc'd
// receive buffer) read through byte_at(i) -- from the ring slot, or from LDS for a doorbell's message.
// ISP restates testcases.c:18-37.  The originator's final call passes NULL (:773): device judges approve it.
template <class F>
__device__ __forceinline__ int judge_eval_f(const Params& P, int me, uint32_t my_mask, int32_t pid, F byte_at,
                                            uint32_t data_len) {
    switch (P.judge_kind) {
        case JUDGE_MASK:
            return my_mask ? 0 : 1;
        case JUDGE_HASH:
            return judge_hash(P.judge_seed, me, pid) < P.judge_ppm ? 0 : 1;
        case JUDGE_ISP: {
            const char* mine = P.judge_isp + P.judge_isp_off[me];
            if (mine[0] == 0) return 1;
            for (uint32_t i = 0;; i++) {  // strcmp(mine, arg)
                char a = i < data_len ? (char)byte_at(i) : 0;
                if (a != mine[i]) break;
                if (a == 0) return 1;
            }
            char a0 = data_len ? (char)byte_at(0u) : 0;
            return ((signed char)a0 < (signed char)mine[0]) ? 0 : 1;
        }
        default:
            return 1;
    }
}
__device__ __forceinline__ int judge_eval(const Params& P, __amdgpu_buffer_rsrc_t rf, int me, uint32_t my_mask, int32_t pid,
                                          uint32_t arg_off, uint32_t data_len) {
    return judge_eval_f(P, me, my_mask, pid, [&](uint32_t i) { return ld8_sc1(rf, arg_off + i); }, data_len);
}

// a volatile LDS word through an LDS-typed pointer (ds_read / ds_write: a generic one is a flat access, counted in
// vmcnt as well as lgkmcnt -- every wait for it also waited for the wave's stores in flight, PCIe ones included)
typedef volatile __attribute__((address_space(3))) uint32_t lds_vu32;
__device__ __forceinline__ lds_vu32* lds_word(uint32_t* p) { return (lds_vu32*)(p); }
typedef volatile __attribute__((address_space(3))) uint64_t lds_vu64;
__device__ __forceinline__ lds_vu64* lds_dword(uint8_t* p) { return (lds_vu64*)(p); }

// one event record: the parity log (MODE_LOG, linear) or the host pickup ring (MODE_HOST, the
// slot after this iteration's earlier events; the selection phase guaranteed the room).  Returns the
// record's payload index (~0u: no payload), or with want_rec the record index itself
template <uint32_t PMK, class SH>  // PMK: the kernel's program mask (no host-mode code where it has none)
__device__ __forceinline__ uint32_t log_put(SH& S, const Params& P, int lr, uint32_t kind, int origin, int from,
                                            uint32_t id, uint32_t len, int vote, uint32_t aux, bool want_rec = false,
                                            bool tagged_payload = false) {
    if (!(P.mode & (MODE_LOG | MODE_HOST))) return ~0u;
    uint32_t i;
    if ((PMK & MODE_HOST) && (P.mode & MODE_HOST)) {  // the tagged record (rlo_device.hpp kPkRecBytes): no drain
        const uint64_t seq = S.pk_tail + atomicAdd(&S.ev_n, 1u);              // and no tail publish before the host
        i = (uint32_t)(seq & (uint64_t)(P.log_cap - 1u));
        const uint32_t t16 = pk_tag16(seq, P.pk_epoch) << 16;
        const bool pl = P.log_payload && (kind == (LOG_DELIVER | (TAG_BCAST << 8)) || kind == LOG_JREQ || kind == LOG_JUDGED);
        const uint32_t pidx = pl ? (i | (tagged_payload ? kPkTaggedPayload : 0u)) : kPkNoPayload;
        u32x4* dst = reinterpret_cast<u32x4*>(&P.log[(size_t)lr * P.log_cap + i]);
        st_sys16(dst, u32x4{kind | t16, (uint32_t)origin, ((uint32_t)(from + 1) & 0xffffu) | t16, id});
        st_sys16(dst + 1, u32x4{len, ((uint32_t)vote & 0xffffu) | t16, aux, pidx | t16});
        return want_rec ? i : (pl ? i : ~0u);
    } else {
        i = (uint32_t)atomicAdd(&S.log_count, 1ull);
        if (i >= P.log_cap) {
            set_error(S, P, ERR_LOG_FULL, i);
            return ~0u;
        }
    }
    LogRec r;
    r.kind = kind;
    r.origin = origin;
    r.from = from;
    r.id = id;
    r.len = len;
    r.vote = vote;
    r.aux = aux;
    r.payload_idx = (P.log_payload && (kind == (LOG_DELIVER | (TAG_BCAST << 8)) || kind == LOG_JREQ || kind == LOG_JUDGED)) ? i : ~0u;
    u32x4* dst = reinterpret_cast<u32x4*>(&P.log[(size_t)lr * P.log_cap + i]);
    st_sys16(dst, u32x4{r.kind, (uint32_t)r.origin, (uint32_t)r.from, r.id});
    st_sys16(dst + 1, u32x4{r.len, (uint32_t)r.vote, r.aux, r.payload_idx});
    return want_rec ? i : r.payload_idx;
}

// chunk q >= 1 of a doorbell-pass event's payload (v: the message's 16-B chunk q) into pickup slot `slot` of my
// ring, in the tagged form (two 8-B units per 8 payload bytes); host mode only
template <class SH>
__device__ __forceinline__ void pk_payload_tagged(const SH& S, const Params& P, int lr, uint32_t slot, uint32_t q, u32x4 v) {
    const uint64_t seq = S.pk_tail + ((slot - (uint32_t)S.pk_tail) & (P.log_cap - 1u));
    const uint32_t tg = pk_tag(seq, P.pk_epoch);
    const __amdgpu_buffer_rsrc_t rp =
        mk_rsrc(P.log_payload + (size_t)lr * P.log_cap * P.log_stride, P.log_cap * P.log_stride);
    st_ring(rp, slot * P.log_stride + 32u * (q - 1u), u32x4{v.x, tg, v.y, tg}, true);
    st_ring(rp, slot * P.log_stride + 32u * (q - 1u) + 16u, u32x4{v.z, tg, v.w, tg}, true);
}

// a received proposal carries one of my own in-flight pids (the reference checks its one
// my_own_proposal, :690-692; here every slot of the pool)
template <class SH>
__device__ __forceinline__ bool own_has(const SH& S, const Params& P, int32_t pid) {
    bool hit = false;
    for (uint32_t k = 0; k < P.pend_slots; k++) hit |= S.own_state[k] != 0u && S.own_pid[k] == pid;
    return hit;
}

// vote up towards the parent over in-edge k: one 16-byte write-through slot (_vote_back, :728-741),
// and with doorbells (LLB) the parent's vote bell for this edge, tagged with the vote's sequence
template <bool LLB, class SH>
__device__ __forceinline__ void emit_vote(SH& S, const Params& P, int me, uint32_t k,
                                          int origin, int32_t pid, uint32_t pseq, int vote) {
    unsigned long long p = atomicAdd((unsigned long long*)&S.vout_tail[k], 1ull);
    if (p - S.vout_head[k] >= P.vote_cap) {
        set_error(S, P, ERR_VOTE_RING, k);
        return;
    }
    if (LLB && (P.mode & MODE_LL)) {  // {origin | pseq << 16 | vote << 24, T, pid, T}: every 8-B half tagged
        const uint32_t T = bell_tag(p);
        gu64* b = gptr64(S.t.vout_bell[k]);
        const uint64_t w0 = (uint64_t)(((uint32_t)origin & 0xffffu) | ((pseq & 0xffu) << 16) | ((uint32_t)(vote & 0xff) << 24)) |
                            ((uint64_t)T << 32);
        const uint64_t w1 = (uint64_t)(uint32_t)pid | ((uint64_t)T << 32);
        if (P.sys_scope) {
            __hip_atomic_store(b, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(b + 1, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            __hip_atomic_store(b, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(b + 1, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const uint64_t lo = (uint64_t)((uint32_t)origin | ((uint32_t)(vote & 0xff) << 24)) | ((uint64_t)(uint32_t)pid << 32);
    const uint64_t hi = (uint64_t)(pseq & 0xffu) | ((uint64_t)(uint32_t)me << 32);
    gu64* dst = gptr64(S.t.vout_ring[k] + (uint64_t)(p & (P.vote_cap - 1)) * kVoteSlot);
    if (P.sys_scope) {
        __hip_atomic_store(dst, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dst + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        __hip_atomic_store(dst, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dst + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// exclusive wave-wide prefix sum with DPP row shifts + row broadcasts (no LDS traffic)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    return x - v;
}

// wave-wide OR / MAX with the same DPP pattern, result uniform (lane 63 broadcast)
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    uint32_t x = v;
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    uint32_t x = v;
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// payload chunk q >= 1 of a locally originated message (payload bytes [16(q-1), 16q))
__device__ __forceinline__ u32x4 gen_chunk(const Params& P, uint32_t kind, int me, uint32_t id, uint32_t len,
                                           uint32_t src, int vote, uint32_t q) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (kind == K_STORM || kind == K_LAT) {
        const uint32_t k0 = 2u * (q - 1u);
        const int b0 = (int)len - (int)(8u * k0);
        uint64_t a = b0 > 0 ? storm_word((uint32_t)me, id, k0) : 0ull;
        uint64_t b = b0 > 8 ? storm_word((uint32_t)me, id, k0 + 1u) : 0ull;
        v.x = mask_bytes((uint32_t)a, b0);
        v.y = mask_bytes((uint32_t)(a >> 32), b0 - 4);
        v.z = mask_bytes((uint32_t)b, b0 - 8);
        v.w = mask_bytes((uint32_t)(b >> 32), b0 - 12);
    } else if (kind == K_PROP) {  // PBuf [pid][vote=1][data_len u64][data] (:1369-1396)
        const uint32_t dl = P.prop_data_len[src];
        if (q == 1) {
            v.x = id; v.y = 1u; v.z = dl; v.w = 0u;
        } else {
            const uint8_t* d = P.prop_data + P.prop_data_off[src];
            uint32_t w[4];
#pragma unroll
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
    } else if (kind == K_DEC) {  // PBuf(pid, decision, 7, "IAR_DEC") (:908-917)
        if (q == 1) {
            v.x = id; v.y = (uint32_t)vote; v.z = 7u; v.w = 0u;
        } else if (q == 2) {
            v.x = 0x5F524149u; v.y = 0x00434544u;
        }
    }
    return v;
}

}  // namespace rlo
