// rlo_world.cpp -- host side of the engine: overlay topology, the global HBM layout of
// the mailbox rings, parts (one per process / GPU) and their connection through hipIpc,
// programs (storm / latency / iar), launch and result readout.  Exposes the C ABI of
// include/rlo_hip.h.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <mutex>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "rlo_device.hpp"
#include "rlo_hip.h"
#include "rlo_shm.hpp"

// variant: 8 = 8-wave, 4 = 4-wave, 5 = 4-wave with bulk messages (rlo_kernel.hip)
extern "C" hipError_t rlo_launch_progress(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream, int variant);
extern "C" size_t rlo_kernel_static_lds(int variant);
extern "C" hipError_t rlo_occupancy(int* blocks, size_t dyn_lds, int variant);
extern "C" hipError_t rlo_occupancy_ll(int* blocks, size_t dyn_lds, int variant);
extern "C" hipError_t rlo_launch_hop(const rlo::Params* p, int blocks, size_t dyn_lds, hipStream_t stream);
extern "C" hipError_t rlo_occupancy_hop(int* blocks, size_t dyn_lds, int ph);

static_assert(sizeof(rlo_rank_stats_t) == sizeof(rlo::RankStats), "stats ABI");
static_assert(sizeof(rlo_log_rec_t) == sizeof(rlo::LogRec), "log ABI");

namespace {

thread_local int g_last_hip = 0;

// A/B and diagnostic switches from the environment (RLO_WAVES, RLO_NSMALL, RLO_CACHED_RINGS, RLO_LAZY_PUB,
// RLO_NO_IDLE_SPIN, RLO_NO_ACQUIRE, RLO_NO_FAST, RLO_BIG_PIPE, RLO_HOST_DIAG, RLO_BAR_CMDS,
// RLO_NO_HDP_FLUSH) exist only in the diagnostics build (make DIAG=1 -> lib_diag/, -DRLO_DIAG): some of
// them are unsafe by design (RLO_NO_ACQUIRE drops an acquire, RLO_CACHED_RINGS brings back rings that
// failed rarely), so the product library reads none of them
const char* diag_env(const char* name) {
#ifdef RLO_DIAG
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

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

// ------------------------------------------------------------------ global layout
// Computed identically by every part from (n, part boundaries, payload, ring slots), so
// parts agree on every offset without exchanging tables.
struct Edge { int src, dst, j, k; };

struct Layout {
    int n = 0, nparts = 0;
    std::vector<int> pb;          // part boundaries [nparts + 1]
    std::vector<int> part_of;     // [n]
    std::vector<Topo> T;          // [n]
    std::vector<Edge> E;
    std::vector<std::vector<int>> in_edges;
    int max_in = 0, max_fan = 0;
    uint32_t cap = 0, stride = 0, vote_cap = 0;
    std::vector<uint64_t> fwd_bytes, vote_bytes, ctrl_words;  // per part
    std::vector<uint64_t> fwd_off, vote_off;                  // per edge (vc 0 ring; vc 1 follows)
    std::vector<uint32_t> inbox, outbox;                      // per rank: word index in its part's ctrl
    std::vector<uint32_t> fbell, vbell;                       // per rank: its doorbells (rlo_device.hpp) in its ctrl
    std::vector<uint64_t> lat_base;                           // per part: the shared latency block (rlo_device.hpp)
    // bulk messages (rlo_device.hpp): heap slot (r, o, s) and flag line (r, o, s) in r's part, then
    // the done lines (o, s) of the part's origins
    uint64_t bulk_max = 0;
    uint32_t bslots = 0, bcap = 0;
    std::vector<uint64_t> heap_bytes, bflag_bytes;            // per part
    uint32_t pend_slots = 2;  // proposal pool: pending entries per origin (rlo_device.hpp Params.pend_slots)
    // pulled payloads (rlo_device.hpp Params.pull): a large bcast crosses an edge as header +
    // reference, the receiver loads the payload from the sender's relay ring; every rank has one
    // (cap slots, after the forward rings of its part) holding the large bcasts it sends on
    bool pull = false;
    uint32_t relay_cap = 0;
    std::vector<uint64_t> orig_off;  // [n] byte offset of rank r's relay ring in its part's region
};

int build_layout(int n, int nparts, const int32_t* pb, uint32_t max_payload, uint32_t ring_slots, uint64_t bulk_max,
                 uint32_t bulk_slots, Layout& L) {
    if (n < 2 || n > 65535 || nparts < 1 || nparts > rlo::kMaxParts) return RLO_E_INVAL;
    L.n = n;
    L.nparts = nparts;
    L.pb.assign(nparts + 1, 0);
    if (pb) {
        for (int p = 0; p <= nparts; p++) L.pb[p] = pb[p];
    } else {  // contiguous, as even as possible
        for (int p = 0; p <= nparts; p++) L.pb[p] = (int)((int64_t)n * p / nparts);
    }
    if (L.pb[0] != 0 || L.pb[nparts] != n) return RLO_E_INVAL;
    for (int p = 0; p < nparts; p++)
        if (L.pb[p + 1] <= L.pb[p]) return RLO_E_INVAL;
    L.part_of.assign(n, 0);
    for (int p = 0; p < nparts; p++)
        for (int r = L.pb[p]; r < L.pb[p + 1]; r++) L.part_of[r] = p;
    L.stride = rlo::kHdr + max_payload;

    L.T.assign(n, Topo{});
    for (int r = 0; r < n; r++)
        if (topo_of(n, r, &L.T[r])) return RLO_E_INVAL;
    L.in_edges.assign(n, {});
    for (int r = 0; r < n; r++)
        for (int j = 0; j < L.T[r].sll; j++) {
            L.in_edges[L.T[r].send_list[j]].push_back((int)L.E.size());
            L.E.push_back({r, L.T[r].send_list[j], j, 0});
        }
    for (int c = 0; c < n; c++) {
        if ((int)L.in_edges[c].size() > rlo::kMaxIn) return RLO_E_INVAL;
        L.max_in = std::max(L.max_in, (int)L.in_edges[c].size());
        for (int k = 0; k < (int)L.in_edges[c].size(); k++) L.E[L.in_edges[c][k]].k = k;
    }
    for (int r = 0; r < n; r++) L.max_fan = std::max(L.max_fan, L.T[r].sll);

    // ring capacity: every part's forward region must fit one 32-bit buffer resource
    std::vector<uint64_t> rings(nparts, 0), vrings(nparts, 0);
    for (const Edge& e : L.E) {
        rings[L.part_of[e.dst]] += 2;
        vrings[L.part_of[e.src]] += 1;
    }
    // pulled payloads (not in bulk worlds): the default where slots hold messages beyond the small
    // copy path (> 24 chunks); RLO_PULL=0 pushes, RLO_PULL=1 also pulls in medium-slot worlds.  Since
    // the large-message rounds move whole messages per group, pulling is faster than pushing (1 KiB
    // storm 37.6 -> 35.8 ms, 4 KiB 86.8 -> 79.3 ms, profiles/r2s5_sizes_groups_ab.txt)
    {
        const char* pe = std::getenv("RLO_PULL");
        const bool want = pe ? std::atoi(pe) != 0 : L.stride / 16u > 24u;
        L.pull = want && L.stride > 8u * 16u && !bulk_max;
    }
    if (L.pull)
        for (int r = 0; r < n; r++) rings[L.part_of[r]] += 1;  // the relay ring
    const uint64_t max_rings = *std::max_element(rings.begin(), rings.end());
    // default depth (tools/sweep.py, profiles/r1s5_sweep64.log): small slots (the 8-wave path,
    // payload <= 112 B) keep the wall ranks' hot rings from refusing: 64 B storm at 256 ranks
    // 512 slots 16.1M, 1024 25.8M, 2048 29.2M, 4096 29.4M bcast/s; medium slots (the small copy path,
    // payload <= 368 B) too: 256 B storm 6.58M -> 7.04M (profiles/r3_storm_slots.txt); large slots stay at
    // 512 (1 KiB: no gain)
    uint32_t cap = ring_slots ? pow2_ceil(ring_slots) : (L.stride <= 384u ? 2048u : 512u);
    const uint64_t limit = 0xFFFF0000ull;
    if (max_rings * cap * L.stride > limit) cap = pow2_floor(limit / (max_rings * L.stride));
    if (cap < 16) return RLO_E_INVAL;
    L.cap = cap;
    // a vote slot is taken per proposal in flight through the edge: N origins x pool slots each
    L.vote_cap = std::max<uint32_t>(64u, pow2_ceil(L.pend_slots * (uint32_t)n));

    const uint64_t ring_bytes = (uint64_t)cap * L.stride;
    L.fwd_bytes.assign(nparts, 0);
    L.vote_bytes.assign(nparts, 0);
    L.fwd_off.assign(L.E.size(), 0);
    L.vote_off.assign(L.E.size(), 0);
    for (size_t e = 0; e < L.E.size(); e++) {
        const int pd = L.part_of[L.E[e].dst], ps = L.part_of[L.E[e].src];
        L.fwd_off[e] = L.fwd_bytes[pd];
        L.fwd_bytes[pd] += 2 * ring_bytes;
        L.vote_off[e] = L.vote_bytes[ps];
        L.vote_bytes[ps] += (uint64_t)L.vote_cap * rlo::kVoteSlot;
    }
    L.orig_off.assign(n, 0);
    if (L.pull) {
        // relay rings: 4x the ring depth where the part's region stays one buffer resource (a relay slot
        // is released only once every child consumed it, which lags the ring credits)
        L.relay_cap = cap;
        for (uint32_t f = 4; f > 1; f /= 2) {
            bool fits = true;
            for (int p = 0; p < nparts; p++) {
                const uint64_t nlp = (uint64_t)(L.pb[p + 1] - L.pb[p]);
                fits &= L.fwd_bytes[p] + nlp * f * ring_bytes <= limit;
            }
            if (fits) { L.relay_cap = f * cap; break; }
        }
        for (int r = 0; r < n; r++) {
            L.orig_off[r] = L.fwd_bytes[L.part_of[r]];
            L.fwd_bytes[L.part_of[r]] += (uint64_t)L.relay_cap * L.stride;
        }
    }
    if (*std::max_element(L.vote_bytes.begin(), L.vote_bytes.end()) > limit) return RLO_E_INVAL;

    // control words: per part a header (word 0 = error flag), then per rank an inbox block
    // (tails of its in-rings + vote in-rings) and an outbox block (heads), 128-B aligned
    L.ctrl_words.assign(nparts, 0);
    L.lat_base.clear();
    L.inbox.assign(n, 0);
    L.outbox.assign(n, 0);
    L.fbell.assign(n, 0);
    L.vbell.assign(n, 0);
    for (int p = 0; p < nparts; p++) {
        uint64_t words = rlo::kCtrlHdrWords;
        for (int r = L.pb[p]; r < L.pb[p + 1]; r++) {
            L.inbox[r] = (uint32_t)words;
            words += (2 * L.in_edges[r].size() + L.T[r].sll + 15) & ~15ull;
            L.outbox[r] = (uint32_t)words;
            words += (2 * L.T[r].sll + L.in_edges[r].size() + 15) & ~15ull;
        }
        L.lat_base.push_back(words);
        words += rlo::kLatWords;
        for (int r = L.pb[p]; r < L.pb[p + 1]; r++) {  // doorbells: forward per in-edge, vote per child
            L.fbell[r] = (uint32_t)words;
            words += (uint64_t)L.in_edges[r].size() * rlo::kBellWords;
            L.vbell[r] = (uint32_t)words;
            words += (2ull * L.T[r].sll + 15) & ~15ull;
        }
        L.ctrl_words[p] = words;
    }
    L.heap_bytes.assign(nparts, 0);
    L.bflag_bytes.assign(nparts, 0);
    if (bulk_max) {
        // 2 heap slots per origin by default, 1 where N x 2 would pass the pending-reception bound (C5 at 8 GPUs)
        L.bslots = bulk_slots ? bulk_slots : ((uint64_t)n * 2u <= (uint64_t)rlo::kMaxPend ? 2u : 1u);
        if ((L.bslots & (L.bslots - 1)) || L.bslots > 8 || (uint64_t)n * L.bslots > (uint64_t)rlo::kMaxPend) return RLO_E_INVAL;
        if (bulk_max > 0xFFF00000ull) return RLO_E_INVAL;  // a slot is addressed by one buffer resource
        L.bulk_max = bulk_max;
        L.bcap = (uint32_t)((bulk_max + 65535u) & ~65535ull);
        for (int p = 0; p < nparts; p++) {
            const uint64_t nlp = (uint64_t)(L.pb[p + 1] - L.pb[p]);
            L.heap_bytes[p] = nlp * (uint64_t)n * L.bslots * L.bcap;
            L.bflag_bytes[p] = (nlp * (uint64_t)n * L.bslots + nlp * L.bslots) * rlo::kBulkLine;
        }
    }
    return RLO_OK;
}

// one part's connection record: what a peer needs to map this part's regions
struct PartBlob {
    uint32_t magic, version;
    int32_t part, nparts, n, device;
    uint32_t cap, stride, vote_cap, pad;
    uint64_t token;  // identifies the hosting process
    uint64_t fwd_ptr, vote_ptr, ctrl_ptr;
    uint64_t fwd_bytes, vote_bytes, ctrl_bytes;
    char bus[32];
    hipIpcMemHandle_t hf, hv, hc;
    uint64_t heap_ptr, bflag_ptr, heap_bytes, bflag_bytes;
    hipIpcMemHandle_t hh, hb;
    uint64_t nonce;  // written at the start of every region at creation: a peer's mapping must show it
};
static_assert(sizeof(PartBlob) <= RLO_PART_BLOB_BYTES, "blob");
constexpr uint32_t kBlobMagic = 0x524C4F50u;  // "RLOP"

uint64_t process_token() {
    static uint64_t tok = 0;
    if (!tok) {
        std::random_device rd;
        tok = ((uint64_t)rd() << 32) ^ rd() ^ ((uint64_t)getpid() << 17) ^ (uint64_t)(uintptr_t)&tok;
        if (!tok) tok = 1;
    }
    return tok;
}

}  // namespace

struct rlo_world {
    Layout L;
    int part = 0, nl = 0, rb = 0;  // my part, local rank count, first local rank
    int device = 0;
    uint32_t max_payload = 0, flags = 0;
    int cus = 0, blocks_per_cu = 0;
    bool connected = false;
    int sys_scope = 0;  // system-scope remote stores / publishes: some peer on another GPU or in another process
    uint32_t peers = 0;  // RLO_PEER_*
    // local regions (the rings / counters this part consumes)
    uint8_t* fwd = nullptr;
    uint8_t* vote = nullptr;
    uint64_t* ctrl = nullptr;
    // every part's regions as addresses in this process
    std::vector<uint8_t*> pf, pv;
    std::vector<uint64_t*> pc;
    std::vector<void*> opened;  // hipIpc mappings to close
    std::vector<uint8_t> peer_done;  // part q's regions are mapped (rlo_part_import / rlo_part_connect)
    std::vector<rlo::RankTopo> topo;
    DevBuf<rlo::RankTopo> d_topo;
    DevBuf<rlo::RankStats> d_stats;
    // program
    bool have_program = false;
    rlo::Params P{};
    DevBuf<int64_t> d_sched_off, d_expect_bcast, d_prop_off, d_expect_dec;
    DevBuf<uint32_t> d_sched_ids, d_prop_data_off, d_prop_data_len, d_isp_off, d_lat_count, d_lat_round;
    DevBuf<uint32_t> d_lat_own_off, d_lat_own;
    DevBuf<int32_t> d_lat_origin, d_prop_pid;
    DevBuf<uint64_t> d_lat_out, d_lat_obs;
    uint32_t* d_xcd = nullptr;  // RLO_PART_ONE_XCD: the placement check word (uncached)
    DevBuf<uint32_t> d_tl;  // RLO_FLAG_TIMELINE rows
    uint32_t tl_rows = 0;
    DevBuf<uint8_t> d_mask, d_prop_data, d_log_payload;
    DevBuf<char> d_isp;
    DevBuf<rlo::LogRec> d_log;
    uint32_t lat_rounds = 0;
    // host-service program (pinned host memory)
    uint8_t* h_cmd = nullptr;       // [nl][cmd_cap][stride]     uncached VRAM, CPU writes through the BAR
    uint8_t* h_llc = nullptr;       // [nl][cmd_cap] x kLLCmdSlot command doorbells (pinned host, not in a segment)
    uint64_t* h_ctl = nullptr;      // [nl][kHctlWords]           pinned host: device-written counters
    uint64_t* d_ctl = nullptr;      // [nl][kHctlWords]           uncached VRAM: host-written counters
    volatile uint32_t* hdp = nullptr;  // the GPU's HDP_MEM_COHERENCY_FLUSH_CNTL register (see hdp_flush)
    bool cmd_host = false;          // the command ring + host counters in pinned host memory (default)
    rlo::LogRec* h_ev = nullptr;    // [nl][pk_cap]
    uint8_t* h_evp = nullptr;       // [nl][pk_cap][pk_stride]
    uint32_t pk_stride = 0;         // pickup payload stride (rlo_device.hpp pk_payload_stride)
    uint32_t pk_epoch = 0;          // pickup-tag epoch of the latest host-mode launch (pk_tag)
    bool pk_dirty = false;          // a host-mode launch may have written pickup records / payloads since the last reset
    bool last_hop = false;          // the latest launch ran the hop kernel (rlo_hop.hip), not the progress kernel
    uint32_t cmd_cap = 0, pk_cap = 0;
    std::vector<uint64_t> cmd_tail, pk_head;  // host-side copies of the counters it owns
    // shared host service (rlo_host_share): h_ctl / h_ev / h_evp live in a POSIX shared-memory
    // segment registered with HIP; d_hctl / d_ev / d_evp are the kernel's addresses of them
    uint8_t* shm = nullptr;
    uint64_t shm_bytes = 0;
    std::string shm_name;
    bool shm_linked = false;
    rlo::ShmLayout SL{};
    std::vector<uint64_t> cli_req;  // last bulk request served per local rank
    uint64_t share_stage = 0;       // rlo_host_share called: rlo_program_host builds the segment
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    size_t dyn_lds = 0;
    uint32_t nsmall = 8, stage2 = 1024;
    bool ll_ok = false;  // the doorbell instantiation of the kernel is co-resident at this world's size
    bool pend_hbm = false;  // the pending-proposal tables in HBM (plan_lds), nl x N x pool x 16 B, uncached
    uint64_t nonce = 0;     // this part's creation nonce (PartBlob.nonce)
    uint8_t* pend_mem = nullptr;
    int waves = 4;    // rank-workgroup width: 8 (512 candidates per iteration) when each rank has a CU
    int variant = 4;  // kernel instantiation: 8 / 4 waves, 5 = 4 waves with bulk messages
    // bulk messages (rlo_device.hpp): this part's heap, flag region and job rings (all uncached),
    // every part's heap / flag region as mapped here, and the device tables the kernel indexes
    uint8_t* heap = nullptr;
    uint8_t* bflag = nullptr;
    uint8_t* jmem = nullptr;
    uint64_t jmem_bytes = 0;
    uint32_t nmov = 0, jslots = 0, bpend_off = 0;
    std::vector<uint8_t*> ph, pbf;
    DevBuf<uint64_t> d_bheap, d_bflag;
    DevBuf<int32_t> d_part_of, d_part_begin;
    std::vector<uint32_t> host_bulk_q;     // host mode: next bulk sequence of each local rank
};

namespace {

constexpr uint64_t kNonceTail = 256;  // bytes past a region that hold its creation nonce (rlo_part_create)
// the word region r (0 control, 1 vote, 2 heap, 3 forward, 4 bulk flags) of a part carries: different per region, so
// an import that maps ANOTHER region of the same part fails the check too (one nonce for all five passed it)
uint64_t region_nonce(uint64_t nonce, int r) { return nonce ^ (0x9E3779B97F4A7C15ull * (uint64_t)(r + 1)); }
// ---- the region pool and the import cache.  A world's regions -- the memory its peers map --
// are never handed back to HIP: a destroyed world's regions wait here, by (device, memory type, size class), for the
// next world of this process, and a peer's import of a region stays open here for that peer's next world.  Freeing
// exported memory and importing new handles world after world (bench.py's legs, the test suite's worlds) was seen on
// MI355X / ROCm 7.2 to give importers mappings of OTHER memory for fresh handles (another part's heap, zeros) and
// to make hipIpcGetMemHandle fail for fresh allocations; with the pool, a region a peer imported once is the same
// memory at the same address in every later world (its handle names the same allocation), so no mapping goes stale.
struct PoolEnt {
    void* p;
    uint64_t bytes;
    int device;
    bool uncached;
    bool exported;  // a handle of it went out (rlo_part_export): a peer process may hold an import of it
};
std::mutex g_pool_mu;
std::vector<PoolEnt> g_pool;       // free regions
std::vector<PoolEnt> g_pool_live;  // regions some world of this process holds
std::vector<PoolEnt> g_retired;    // free exported regions beyond the cap: freed only by rlo_pool_trim(RLO_TRIM_RETIRED)
// free bytes kept per process (RLO_POOL_CAP_BYTES, default 8 GiB).  Beyond it a region nobody else ever mapped goes
// back to HIP at once; an EXPORTED one is only retired -- never hipFree'd while a peer process may still hold an import
// of it (freeing exported memory a peer still imported is the failure the pool exists to prevent), until
// the application runs the world-wide close (every process rlo_pool_trim(RLO_TRIM_IMPORTS), a barrier, then
// rlo_pool_trim(RLO_TRIM_RETIRED)); bench.py's sharded legs and the drop-in's RLO_device_memory_release do
uint64_t pool_cap() {
    static const uint64_t cap = [] {
        const char* e = std::getenv("RLO_POOL_CAP_BYTES");
        return e && *e ? std::strtoull(e, nullptr, 10) : (8ull << 30);
    }();
    return cap;
}
// sizes rounded up to a class (>= 2 MiB: its own allocation, not a sub-allocation another region shares; then eighths
// of the next power of two), so that worlds of similar sizes share regions
uint64_t pool_class(uint64_t b) {
    if (b <= (2ull << 20)) return 2ull << 20;
    uint64_t p2 = 1;
    while (p2 < b) p2 <<= 1;
    const uint64_t step = p2 / 8;
    return (b + step - 1) / step * step;
}

int alloc_region(rlo_world* w, void** p, uint64_t bytes) {
    const bool unc = (w->flags & RLO_PART_UNCACHED) != 0;
    const uint64_t cls = pool_class(bytes ? bytes : 256);
    bool reused = false;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); i++)
            if (g_pool[i].device == w->device && g_pool[i].uncached == unc && g_pool[i].bytes == cls) {
                *p = g_pool[i].p;
                g_pool_live.push_back(g_pool[i]);
                g_pool.erase(g_pool.begin() + (long)i);
                reused = true;
                break;
            }
        for (size_t i = 0; !reused && i < g_retired.size(); i++)  // a retired region is still good memory to reuse
            if (g_retired[i].device == w->device && g_retired[i].uncached == unc && g_retired[i].bytes == cls) {
                *p = g_retired[i].p;
                g_pool_live.push_back(g_retired[i]);
                g_retired.erase(g_retired.begin() + (long)i);
                reused = true;
            }
    }
    if (reused) {
        // a region another world used: zeroed, as hipMalloc'd memory was, so no byte of that world is ever read
        // as this one's (the heap and vote regions rely on write-before-read alone otherwise)
        hipError_t e = hipMemset(*p, 0, cls);
        if (e != hipSuccess) { g_last_hip = (int)e; return RLO_E_HIP; }
        return RLO_OK;
    }
    hipError_t e = unc ? hipExtMallocWithFlags(p, cls, hipDeviceMallocUncached) : hipMalloc(p, cls);
    if (e != hipSuccess) { g_last_hip = (int)e; *p = nullptr; return RLO_E_HIP; }
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool_live.push_back(PoolEnt{*p, cls, w->device, unc, false});
    return RLO_OK;
}

// a handle of region p is about to leave this process
void mark_exported(void* p) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (PoolEnt& q : g_pool_live)
        if (q.p == p) q.exported = true;
}

// a destroyed world's region back to the pool; beyond the cap the oldest free ones leave it (never-exported: freed;
// exported: retired, see pool_cap)
void release_region(void* p) {
    if (!p) return;
    std::vector<void*> drop;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool_live.size(); i++)
            if (g_pool_live[i].p == p) {
                g_pool.push_back(g_pool_live[i]);
                g_pool_live.erase(g_pool_live.begin() + (long)i);
                break;
            }
        uint64_t tot = 0;
        for (const PoolEnt& q : g_pool) tot += q.bytes;
        while (tot > pool_cap() && !g_pool.empty()) {
            tot -= g_pool.front().bytes;
            if (g_pool.front().exported) g_retired.push_back(g_pool.front());
            else drop.push_back(g_pool.front().p);
            g_pool.erase(g_pool.begin());
        }
    }
    for (void* d : drop) (void)hipFree(d);
}

// imports of peers' regions, by the handle words that name the allocation (exporter address and pid, the
// allocation's id, its size: the first 13 words; the handle's last words are not initialised)
struct ImpEnt {
    uint32_t key[13];
    void* p;
    int device;
    int refs;
};
std::vector<ImpEnt> g_imports;  // [g_pool_mu]
constexpr size_t kImportCap = 512;  // idle imports kept open (beyond: the idle ones are closed)

hipError_t open_import(void** p, const hipIpcMemHandle_t& h, int device) {
    uint32_t key[13];
    std::memcpy(key, &h, sizeof key);
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (ImpEnt& e : g_imports)
            if (e.device == device && std::memcmp(e.key, key, sizeof key) == 0) {
                e.refs++;
                *p = e.p;
                return hipSuccess;
            }
    }
    const hipError_t r = hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
    if (r != hipSuccess) return r;
    ImpEnt e;
    std::memcpy(e.key, key, sizeof key);
    e.p = *p;
    e.device = device;
    e.refs = 1;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_imports.push_back(e);
    return hipSuccess;
}

void close_import(void* p) {
    std::vector<void*> drop;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (ImpEnt& e : g_imports)
            if (e.p == p && e.refs > 0) { e.refs--; break; }
        if (g_imports.size() > kImportCap) {
            for (size_t i = 0; i < g_imports.size();) {
                if (g_imports[i].refs == 0 && g_imports.size() > kImportCap / 2) {
                    drop.push_back(g_imports[i].p);
                    g_imports.erase(g_imports.begin() + (long)i);
                } else {
                    i++;
                }
            }
        }
    }
    for (void* d : drop) (void)hipIpcCloseMemHandle(d);
}

// job-ring memory of a part (uncached, part-local): [jobs 2J x 64 B][jctl][jclaim 2J][jfree 2J][jdone 2J][jsum 2J]
struct JobMem {
    uint64_t jobs, jctl, jclaim, jfree, jdone, jsum, bytes;
};
JobMem job_mem(uint32_t J, uint32_t nl) {
    (void)nl;
    JobMem m;
    m.jobs = 0;
    m.jctl = m.jobs + 2ull * J * sizeof(rlo::BulkJob);
    m.jclaim = m.jctl + (uint64_t)rlo::kJctlWords * 8;
    m.jfree = m.jclaim + 2ull * J * 8;
    m.jdone = m.jfree + 2ull * J * 8;
    m.jsum = (m.jdone + 2ull * J * 4 + 127) & ~127ull;
    m.bytes = m.jsum + 2ull * J * 8;
    return m;
}

// ---- LDS layout of a part: (kernel variant, staged chunks per message, large-message stage, where the
// pending-proposal table lives, doorbells).  A pure function of the world layout, the local rank count and
// an occupancy oracle: the HIP runtime's answer when the part is created on a GPU, the build's register
// guarantees (Makefile guard) when rlo_layout_plan asks on a host without one.
//
// The small copy path needs every chunk of a small / medium slot staged (nsmall = slot chunks, <= 24), and
// large slots stage 5 chunks (header + 64 B: a 64-B message and a proposal stay on the small path).  That
// count is never lowered to make a layout fit: a world that cannot stage it in LDS moves its
// pending-proposal table (N x pool x 16 B per rank, the one per-rank LDS array that grows with the WORLD
// size) to HBM, then drops to 4 waves -- instead of silently moving every message onto the large path, as
// the 8-GPU world (N = 2048: a 64-KiB table) did up to round 3.
struct LdsPlan {
    int variant = 4, waves = 4, blocks_per_cu = 1;
    uint32_t nsmall = 0, stage2 = 0, bpend_off = 0;
    size_t dyn_lds = 0;
    bool ll_ok = false, pend_hbm = false;
};
// occupancy oracle: blocks of `variant` (| kVariantPH: its PH instantiation; ll: its doorbell form) per CU
// at `dyn_lds` bytes of dynamic LDS
typedef int (*OccFn)(int variant, bool ll, size_t dyn_lds);
constexpr int kVariantPH = 16;  // rlo_kernel.hip rlo_occupancy: variant | 16 = the PH instantiation
constexpr size_t kLdsPerCU = 163840;  // 160 KiB per CU (MI355X_MICROARCH.md)

int occ_device(int variant, bool ll, size_t dyn_lds) {
    int b = 0;
    if ((ll ? rlo_occupancy_ll(&b, dyn_lds, variant) : rlo_occupancy(&b, dyn_lds, variant)) != hipSuccess) return 0;
    return b;
}
// no GPU: LDS (512-B allocation granules), 32 waves per CU, and the waves per SIMD every instantiation is
// built to (the Makefile's register guard fails the build of an 8-wave one, or a 4-wave one without
// doorbells, that drops below 2 per SIMD; the 4-wave doorbell and bulk ones may take one)
int occ_model(int variant, bool ll, size_t dyn_lds) {
    const int v = variant & ~kVariantPH;
    const int W = v == 8 ? 8 : 4;
    const size_t lds = ((rlo_kernel_static_lds(v) + dyn_lds + 511) & ~(size_t)511);
    const int by_lds = lds ? (int)(kLdsPerCU / lds) : 8;
    const int per_simd = (v == 8 || (v == 4 && !ll)) ? 2 : 1;
    const int by_regs = per_simd * 4 / W;
    return std::min(by_lds, std::min(by_regs, 32 / W));
}

// one variant (8 / 4 / 5), the pending table in LDS or HBM
int plan_variant(const Layout& L, int nl, int nmov, int cus, int variant, bool pend_hbm, OccFn occ, uint32_t ns_force,
                 LdsPlan* out) {
    const int waves = variant == 8 ? 8 : 4;
    const int nblk = nl + (variant == 5 ? nmov : 0);
    const int need_bpc = (nblk + cus - 1) / cus;
    const size_t per_block = kLdsPerCU / need_bpc;
    const size_t cand = (size_t)64 * waves, stat = rlo_kernel_static_lds(variant);
    const size_t bpend = variant == 5 ? (size_t)L.n * L.bslots * 32 : 0;  // pending bulk receptions
    const size_t ptab = pend_hbm ? 0 : (size_t)16 * L.n * L.pend_slots;
    // every message of a medium slot (<= 24 chunks: payload <= 368 B) takes the small copy path (packed
    // (message, chunk) copies; the large-message path moves one message per LDS block: 256 B storm 2.0M
    // bcast/s, profiles/r2s2_diag_sizes.log); large slots stage 5 chunks -- header + 64 B -- and leave the
    // LDS to the large-message rounds (4 KiB storm 109 -> 104 ms, 1 KiB 40.4 -> 38.4, r2s4_nsmall_ab.txt)
    const uint32_t ns = ns_force ? ns_force : (L.stride / 16u <= 24u ? L.stride / 16u : 5u);
    // [pending proposals N x pend_slots x 16 B][olist 2 maxfan x cand x 2 B][stage cand x ns x 16 B][stage2][bulk pending]
    const size_t fixed = stat + ptab + (size_t)2 * L.max_fan * cand * 2 + cand * ns * 16 + bpend;
    if (per_block < fixed + 1024 + 512) return RLO_E_OCCUPANCY;
    size_t s2 = std::min<size_t>(128 * 1024, (per_block - fixed - 512) & ~(size_t)1023);  // two halves of <= 64 blocks
    const int vph = variant | (pend_hbm && variant != 5 ? kVariantPH : 0);
    int api = 0;
    for (;;) {
        const size_t dyn = fixed - stat + s2;
        api = occ(variant, false, dyn);
        if (api >= need_bpc && vph != variant) api = std::min(api, occ(vph, false, dyn));
        if (api >= need_bpc) break;
        if (s2 <= 1024) return RLO_E_OCCUPANCY;
        s2 -= 1024;
    }
    LdsPlan p;
    p.variant = variant;
    p.waves = waves;
    p.nsmall = ns;
    p.stage2 = (uint32_t)s2;
    p.dyn_lds = fixed - stat + s2;
    p.bpend_off = (uint32_t)(fixed - stat - bpend + s2);
    p.blocks_per_cu = std::max(1, api);
    p.pend_hbm = pend_hbm;
    {  // the doorbell instantiation co-resident too? (else its programs run without bells)
        int ll = occ(variant, true, p.dyn_lds);
        if (vph != variant) ll = std::min(ll, occ(vph, true, p.dyn_lds));
        p.ll_ok = ll >= need_bpc;
    }
    if (nblk > p.blocks_per_cu * cus) return RLO_E_OCCUPANCY;
    *out = p;
    return RLO_OK;
}

// 8-wave rank-workgroups (512 candidates per iteration) when every local rank gets a CU of its own and
// every message fits the small copy path (slot <= 8 chunks: payloads <= 112 B); else 4 waves (larger slots
// need the LDS for the large-message stage: 64 B storm 12.1 -> 16.0 M bcast/s with 8 waves, but 256 B ..
// 4 KiB 30-40 % slower).  Per variant: the pending table in LDS, else in HBM (RLO_PART_PEND_HBM: always
// HBM, the tests' way to run the 8-GPU layout's proposal path on one GPU).  Bulk worlds: the 4-wave
// kernel with movers, table in LDS (N x B <= kMaxPend keeps them small).  RLO_WAVES / RLO_NSMALL: A/B
int plan_lds(const Layout& L, int nl, int nmov, int cus, uint32_t flags, OccFn occ, LdsPlan* out) {
    uint32_t ns_force = 0;
    if (const char* e = diag_env("RLO_NSMALL"))  // A/B: staged chunks per candidate in large-slot worlds
        if (L.stride / 16u > 24u) ns_force = std::max(2u, std::min(8u, (uint32_t)std::atoi(e)));
    if (L.bulk_max) return plan_variant(L, nl, nmov, cus, 5, false, occ, ns_force, out);
    const char* env = diag_env("RLO_WAVES");
    const int force = env ? std::atoi(env) : 0;
    const bool small = L.stride <= 8u * 16u;
    const bool hbm_only = (flags & RLO_PART_PEND_HBM) != 0;
    if (force != 4 && (small || force == 8) && nl <= cus) {
        if (!hbm_only && plan_variant(L, nl, nmov, cus, 8, false, occ, ns_force, out) == RLO_OK) return RLO_OK;
        if (plan_variant(L, nl, nmov, cus, 8, true, occ, ns_force, out) == RLO_OK) return RLO_OK;
    }
    if (force == 8) return RLO_E_OCCUPANCY;
    // 4 waves (two rank-workgroups per CU beyond 256 local ranks): a full stage first, with the table in LDS
    // or HBM; only then fewer staged chunks (the 4-wave kernel's large-message path takes the rest)
    const uint32_t ns0 = ns_force ? ns_force : (L.stride / 16u <= 24u ? L.stride / 16u : 5u);
    for (uint32_t ns = ns0; ns >= 1; ns--) {
        if (!hbm_only && plan_variant(L, nl, nmov, cus, 4, false, occ, ns, out) == RLO_OK) return RLO_OK;
        if (plan_variant(L, nl, nmov, cus, 4, true, occ, ns, out) == RLO_OK) return RLO_OK;
    }
    return RLO_E_OCCUPANCY;
}

int size_lds(rlo_world* w) {
    LdsPlan p;
    const int rc = plan_lds(w->L, w->nl, (int)w->nmov, w->cus, w->flags, occ_device, &p);
    if (rc) return rc;
    w->variant = p.variant;
    w->waves = p.waves;
    w->nsmall = p.nsmall;
    w->stage2 = p.stage2;
    w->dyn_lds = p.dyn_lds;
    w->bpend_off = p.bpend_off;
    w->blocks_per_cu = p.blocks_per_cu;
    w->ll_ok = p.ll_ok;
    w->pend_hbm = p.pend_hbm;
    return RLO_OK;
}

// RankTopo of every local rank, with remote ends resolved to addresses in this process
void build_topo(rlo_world* w) {
    const Layout& L = w->L;
    const uint64_t ring_bytes = (uint64_t)L.cap * L.stride;
    w->topo.assign(w->nl, rlo::RankTopo{});
    for (int r = w->rb; r < w->rb + w->nl; r++) {
        rlo::RankTopo& t = w->topo[r - w->rb];
        t.level = L.T[r].level;
        t.last_wall = L.T[r].last_wall;
        t.scc = L.T[r].scc;
        t.sll = L.T[r].sll;
        for (int j = 0; j < L.T[r].sll; j++) t.send_list[j] = L.T[r].send_list[j];
        t.n_in = (int)L.in_edges[r].size();
        t.inbox_ctrl = L.inbox[r];
        t.n_inbox = 2 * t.n_in + t.sll;
        t.outbox_ctrl = L.outbox[r];
        t.n_outbox = 2 * t.sll + t.n_in;
        t.orig_data = (uint32_t)L.orig_off[r];
        t.in_bell = L.fbell[r];
        t.vin_bell = L.vbell[r];
    }
    for (size_t e = 0; e < L.E.size(); e++) {
        const Edge& ed = L.E[e];
        const int ps = L.part_of[ed.src], pd = L.part_of[ed.dst];
        if (ps == w->part) {  // I produce its forward rings, consume its votes
            rlo::RankTopo& t = w->topo[ed.src - w->rb];
            for (int vc = 0; vc < 2; vc++) {
                t.out_ring[ed.j][vc] = (uint64_t)(uintptr_t)(w->pf[pd] + L.fwd_off[e] + vc * ring_bytes);
                t.out_tail[ed.j][vc] = (uint64_t)(uintptr_t)(w->pc[pd] + L.inbox[ed.dst] + 2 * ed.k + vc);
            }
            t.vin_data[ed.j] = (uint32_t)L.vote_off[e];
            t.vin_head[ed.j] = (uint64_t)(uintptr_t)(w->pc[pd] + L.outbox[ed.dst] + 2 * L.T[ed.dst].sll + ed.k);
            t.out_bell[ed.j] = (uint64_t)(uintptr_t)(w->pc[pd] + L.fbell[ed.dst] + (uint64_t)rlo::kBellWords * ed.k);
        }
        if (pd == w->part) {  // I consume its forward rings, produce its votes
            rlo::RankTopo& t = w->topo[ed.dst - w->rb];
            for (int vc = 0; vc < 2; vc++) {
                t.in_data[ed.k][vc] = (uint32_t)(L.fwd_off[e] + vc * ring_bytes);
                t.in_head[ed.k][vc] = (uint64_t)(uintptr_t)(w->pc[ps] + L.outbox[ed.src] + 2 * ed.j + vc);
            }
            t.in_src[ed.k] = ed.src;
            t.in_base[ed.k] = (uint64_t)(uintptr_t)w->pf[ps];  // the producer's slots (pulled payloads)
            t.vout_ring[ed.k] = (uint64_t)(uintptr_t)(w->pv[ps] + L.vote_off[e]);
            t.vout_tail[ed.k] = (uint64_t)(uintptr_t)(w->pc[ps] + L.inbox[ed.src] + 2 * L.in_edges[ed.src].size() + ed.j);
            t.vout_bell[ed.k] = (uint64_t)(uintptr_t)(w->pc[ps] + L.vbell[ed.src] + 2 * ed.j);
        }
    }
}

}  // namespace

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
        case RLO_E_NOTCONNECTED: return "part not connected";
        case RLO_E_AGAIN: return "ring full, retry";
        case RLO_E_TIMEOUT: return "shared host service: no answer in time";
        case RLO_E_STALE: return "a peer part's mapped memory is not that part's current memory (stale IPC mapping)";
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

int rlo_part_create(const rlo_part_cfg_t* cfg, rlo_world_t** out) {
    if (!cfg || !out || cfg->n_parts < 1 || cfg->part < 0 || cfg->part >= cfg->n_parts) return RLO_E_INVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return RLO_E_NODEVICE;
    rlo_world* w = new rlo_world();
    w->max_payload = (std::max<uint32_t>(cfg->max_payload ? cfg->max_payload : 4096u, 16u) + 15u) & ~15u;
    if (w->max_payload > 65520u) { delete w; return RLO_E_INVAL; }  // slot header: 16-bit length (rlo_device.hpp)
    w->flags = cfg->flags;
    // RLO_PART_ONE_XCD: one part, no bulk, <= 256 ranks (as many as one XCD's CUs hold: checked at launch), and only
    // hop-kernel programs (rlo_launch_ex)
    const bool one_xcd = (cfg->flags & RLO_PART_ONE_XCD) != 0;
    if (one_xcd && (cfg->n_parts != 1 || cfg->bulk_max || cfg->n_ranks > 256)) { delete w; return RLO_E_INVAL; }
    // rings and counters in uncached memory for every world, not only for parts on other GPUs: a
    // line of ring memory left in some XCD's L2 by an earlier kernel (the creation / reset fill) is
    // not invalidated by another XCD's write-through stores, and a consumer on that XCD read the
    // zeros (seen as unmarked slot headers that never became visible).  A ONE_XCD world's rings are
    // cached: every producer and consumer is on one XCD, so its L2 is the one copy.  RLO_CACHED_RINGS=1: A/B only
    if (!diag_env("RLO_CACHED_RINGS") && !one_xcd) w->flags |= RLO_PART_UNCACHED;
    {
        const uint32_t pp = cfg->proposal_pool ? cfg->proposal_pool : 2u;
        if ((pp & (pp - 1u)) || pp > (uint32_t)rlo::kPoolMax) { delete w; return RLO_E_INVAL; }
        w->L.pend_slots = pp;  // before the layout: it sizes the vote rings
    }
    int rc = build_layout(cfg->n_ranks, cfg->n_parts, cfg->part_begin, w->max_payload, cfg->ring_slots, cfg->bulk_max,
                          cfg->bulk_slots, w->L);
    if (rc) { delete w; return rc; }
    w->part = cfg->part;
    w->rb = w->L.pb[w->part];
    w->nl = w->L.pb[w->part + 1] - w->rb;
    if (cfg->device >= 0 && hipSetDevice(cfg->device) != hipSuccess) { delete w; return RLO_E_HIP; }
    (void)hipGetDevice(&w->device);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, w->device) != hipSuccess) { delete w; return RLO_E_HIP; }
    w->cus = prop.multiProcessorCount;
    if (w->L.bulk_max) {
        // movers: half scatter / verify (never wait), half gather (wait only for scatters).  Auto:
        // every CU the rank-workgroups leave (>= 16): a bulk copy is HBM bound only with hundreds of
        // workgroups storing (8 ranks, 64 MiB: 12.8 GB/s algbw with 32 movers); idle movers sleep
        int mv = (int)cfg->movers;
        if (mv == 0) mv = std::max(16, w->cus - w->nl) & ~1;
        if (mv < 2) { delete w; return RLO_E_OCCUPANCY; }
        w->nmov = (uint32_t)mv;
        // every sub-job that can be unfinished at once: per local rank B originations (SCATTER) and
        // N x B receptions (GATHER + VERIFY), each cut into min(kMaxSub, its tiles) sub-jobs (tile
        // counts grow with the length: bounded at bulk_max)
        {
            const uint32_t bm = (uint32_t)std::min<uint64_t>(w->L.bulk_max, 0xFFF00000ull);
            const rlo::BulkPlan pl = rlo::bulk_plan(w->L.n, bm, true);
            const rlo::BulkPlan p1 = rlo::bulk_plan(w->L.n, bm, false);
            const uint64_t ts = std::max(rlo::bulk_total_tiles(pl, bm), rlo::bulk_total_tiles(p1, bm));
            const uint64_t tg = std::max(rlo::bulk_stripe_tiles(pl, bm, 0), rlo::bulk_stripe_tiles(p1, bm, 0));
            const uint64_t tv = (bm + rlo::kVerifyTile - 1) / rlo::kVerifyTile;
            const uint64_t K = rlo::kMaxSub;
            const uint64_t nl = (uint64_t)w->nl, B = w->L.bslots, N = (uint64_t)w->L.n;
            const uint64_t need = nl * B * std::min<uint64_t>(rlo::kMaxSubScatter, ts) + nl * N * B * (std::min(K, tg) + std::min(K, tv)) + 64;
            if (need > (1ull << 26)) { delete w; return RLO_E_INVAL; }
            w->jslots = pow2_ceil((uint32_t)need);
        }
    }
    rc = size_lds(w);
    if (rc) { delete w; return rc; }
    const int me = w->part;
    // (forward rings and bulk flags: + kNonceTail bytes past the region for the creation nonce, which no reset clears)
    if (alloc_region(w, (void**)&w->fwd, w->L.fwd_bytes[me] + kNonceTail) || alloc_region(w, (void**)&w->vote, w->L.vote_bytes[me]) ||
        alloc_region(w, (void**)&w->ctrl, w->L.ctrl_words[me] * 8)) {
        rlo_world_destroy(w);
        return RLO_E_HIP;
    }
    if (one_xcd) {
        const hipError_t e = hipExtMallocWithFlags((void**)&w->d_xcd, 256, hipDeviceMallocUncached);
        if (e != hipSuccess) { g_last_hip = (int)e; w->d_xcd = nullptr; rlo_world_destroy(w); return RLO_E_HIP; }
    }
    if (w->pend_hbm) {  // uncached: a launch's workgroup may sit on another XCD than the previous launch's
        const uint32_t keep = w->flags;
        w->flags |= RLO_PART_UNCACHED;
        const int e = alloc_region(w, (void**)&w->pend_mem, (uint64_t)w->nl * w->L.n * w->L.pend_slots * 16u);
        w->flags = keep;
        if (e) { rlo_world_destroy(w); return RLO_E_HIP; }
    }
    if (w->L.bulk_max) {  // heap, flags and job rings: uncached (peers and other XCDs write them)
        w->jmem_bytes = job_mem(w->jslots, (uint32_t)w->nl).bytes;
        const uint32_t keep = w->flags;
        w->flags |= RLO_PART_UNCACHED;
        const int e = alloc_region(w, (void**)&w->heap, w->L.heap_bytes[me]) ||
                      alloc_region(w, (void**)&w->bflag, w->L.bflag_bytes[me] + kNonceTail) || alloc_region(w, (void**)&w->jmem, w->jmem_bytes);
        w->flags = keep;
        if (e) { rlo_world_destroy(w); return RLO_E_HIP; }
        (void)hipMemset(w->bflag, 0, w->L.bflag_bytes[me]);
        w->host_bulk_q.assign(w->nl, 0);
    }
    (void)hipMemset(w->fwd, 0, std::max<uint64_t>(w->L.fwd_bytes[me], 1));
    (void)hipMemset(w->vote, 0, std::max<uint64_t>(w->L.vote_bytes[me], 1));
    (void)hipMemset(w->ctrl, 0, w->L.ctrl_words[me] * 8);
    if (w->d_stats.alloc(w->nl)) { rlo_world_destroy(w); return RLO_E_HIP; }
    {  // the creation nonce, in every region a peer's rlo_part_connect reads it back from through its mapping
       // (control header word kCtrlNonceWord, which rlo_reset keeps; the first word of the vote and heap
       // regions, which no reset clears and only a launch -- after every part connected -- writes; past the
       // end of the forward rings and the bulk flags): a mapping that shows an earlier allocation fails the
       // connection loudly instead of carrying messages into memory that is not this part's any more
        static std::atomic<uint64_t> seq{0};
        w->nonce = splitmix64(process_token() ^ (++seq * 0x9E3779B97F4A7C15ull) ^
                              (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count());
        if (!w->nonce) w->nonce = 1;
        void* regs[5] = {w->ctrl + rlo::kCtrlNonceWord, w->vote, w->heap, w->fwd + w->L.fwd_bytes[me],
                         w->bflag ? w->bflag + w->L.bflag_bytes[me] : nullptr};
        for (int i = 0; i < 5; i++) {
            const uint64_t rn = region_nonce(w->nonce, i);
            if (regs[i] && hipMemcpy(regs[i], &rn, 8, hipMemcpyHostToDevice) != hipSuccess) { rlo_world_destroy(w); return RLO_E_HIP; }
        }
    }
    // the null stream only: another part's persistent kernel may already run on this device
    // (a second engine in the process), and a device-wide sync would wait for it forever
    (void)hipStreamSynchronize(nullptr);
    (void)hipEventCreate(&w->ev0);
    (void)hipEventCreate(&w->ev1);
    *out = w;
    return RLO_OK;
}

int rlo_part_export(rlo_world_t* w, void* blob, uint32_t cap) {
    if (!w || !blob || cap < RLO_PART_BLOB_BYTES) return RLO_E_INVAL;
    if (std::getenv("RLO_DEBUG_REGIONS"))  // (which addresses a part exports, world after world)
        std::fprintf(stderr, "rlo: part %d exports ctrl %p vote %p fwd %p heap %p (%llu B) bflag %p nonce %016llx\n", w->part,
                     (void*)w->ctrl, (void*)w->vote, (void*)w->fwd, (void*)w->heap,
                     (unsigned long long)w->L.heap_bytes[w->part], (void*)w->bflag, (unsigned long long)w->nonce);
    PartBlob b;
    std::memset(&b, 0, sizeof b);
    b.magic = kBlobMagic;
    b.version = 1;
    b.part = w->part;
    b.nparts = w->L.nparts;
    b.n = w->L.n;
    b.device = w->device;
    b.cap = w->L.cap;
    b.stride = w->L.stride;
    b.vote_cap = w->L.vote_cap;
    b.token = process_token();
    b.nonce = w->nonce;
    b.fwd_ptr = (uint64_t)(uintptr_t)w->fwd;
    b.vote_ptr = (uint64_t)(uintptr_t)w->vote;
    b.ctrl_ptr = (uint64_t)(uintptr_t)w->ctrl;
    b.fwd_bytes = w->L.fwd_bytes[w->part];
    b.vote_bytes = w->L.vote_bytes[w->part];
    b.ctrl_bytes = w->L.ctrl_words[w->part] * 8;
    HIPCHK(hipDeviceGetPCIBusId(b.bus, sizeof b.bus, w->device));
    if (w->L.bulk_max) {
        b.heap_ptr = (uint64_t)(uintptr_t)w->heap;
        b.bflag_ptr = (uint64_t)(uintptr_t)w->bflag;
        b.heap_bytes = w->L.heap_bytes[w->part];
        b.bflag_bytes = w->L.bflag_bytes[w->part];
    }
    if (w->L.nparts > 1) {  // handles only where another process may map the regions (a one-part world needs none)
        for (void* r : {(void*)w->fwd, (void*)w->vote, (void*)w->ctrl, (void*)w->heap, (void*)w->bflag})
            if (r) mark_exported(r);
        HIPCHK(hipIpcGetMemHandle(&b.hf, w->fwd));
        HIPCHK(hipIpcGetMemHandle(&b.hv, w->vote));
        HIPCHK(hipIpcGetMemHandle(&b.hc, w->ctrl));
        if (w->L.bulk_max) {
            HIPCHK(hipIpcGetMemHandle(&b.hh, w->heap));
            HIPCHK(hipIpcGetMemHandle(&b.hb, w->bflag));
        }
    }
    std::memset(blob, 0, RLO_PART_BLOB_BYTES);
    std::memcpy(blob, &b, sizeof b);
    return (int)RLO_PART_BLOB_BYTES;
}

// the peer tables of a part (sized once per connection attempt: rlo_part_import may fill some of them first)
static void peer_tables(rlo_world* w, int n_parts) {
    if ((int)w->pf.size() == n_parts) return;
    w->pf.assign(n_parts, nullptr);
    w->pv.assign(n_parts, nullptr);
    w->pc.assign(n_parts, nullptr);
    w->ph.assign(n_parts, nullptr);
    w->pbf.assign(n_parts, nullptr);
    w->peer_done.assign(n_parts, 0);
    w->sys_scope = 0;
    w->peers = 0;
}

// part q's blob: checked against this part's layout
static bool blob_ok(const rlo_world* w, const PartBlob& b, int q, int n_parts) {
    const Layout& L = w->L;
    return b.magic == kBlobMagic && b.part == q && b.nparts == n_parts && b.n == L.n && b.cap == L.cap &&
           b.stride == L.stride && b.vote_cap == L.vote_cap && b.fwd_bytes == L.fwd_bytes[q] &&
           b.vote_bytes == L.vote_bytes[q] && b.ctrl_bytes == L.ctrl_words[q] * 8 && b.heap_bytes == L.heap_bytes[q] &&
           b.bflag_bytes == L.bflag_bytes[q];
}

// map part q's regions (my own: check them; same process: take the addresses; another process: hipIpc imports,
// every one checked against the peer's creation nonce)
static int import_peer(rlo_world* w, const PartBlob& b, int q) {
    const Layout& L = w->L;
    char mybus[32] = {0};
    HIPCHK(hipDeviceGetPCIBusId(mybus, sizeof mybus, w->device));
    const uint64_t tok = process_token();
    if (std::strncmp(b.bus, mybus, sizeof mybus) != 0) w->peers |= RLO_PEER_OTHER_GPU;
    // A peer in another process (its regions imported through hipIpc, on this GPU or another) gets the
    // hand-off the 8-GPU world runs: system-scope (sc0 sc1) stores, system-scope counter publishes and
    // flag adds, system-scope releases before the bulk flags (the round-4 churn
    // failures).  Only the bulk PLAN follows the GPU layout (RLO_PEER_OTHER_GPU -> chunked).
    if (q != w->part && b.token != tok) w->peers |= RLO_PEER_IMPORTED;
    w->sys_scope = w->peers ? 1 : 0;
    // parts on other GPUs store into this part's rings and heaps over xGMI: a cached part's L2
    // could hold lines those system-scope stores do not invalidate (rlo_hip.h RLO_PART_UNCACHED)
    if (w->sys_scope && !(w->flags & RLO_PART_UNCACHED)) return RLO_E_INVAL;
    if (q == w->part) {
        w->pf[q] = w->fwd; w->pv[q] = w->vote; w->pc[q] = w->ctrl;
        w->ph[q] = w->heap; w->pbf[q] = w->bflag;
        // my own regions must still show the nonce rlo_part_create wrote (memory that changes under a part
        // between its creation and its connection is not this part's to hand out)
        const void* own[5] = {w->ctrl + rlo::kCtrlNonceWord, w->vote, L.bulk_max ? w->heap : nullptr,
                              w->fwd + L.fwd_bytes[q], L.bulk_max ? w->bflag + L.bflag_bytes[q] : nullptr};
        for (int i = 0; i < 5; i++) {
            if (!own[i]) continue;
            uint64_t got = 0;
            HIPCHK(hipMemcpy(&got, own[i], 8, hipMemcpyDeviceToHost));
            if (got != region_nonce(w->nonce, i)) {
                static const char* const names[5] = {"control", "vote", "heap", "forward", "bulk-flag"};
                std::fprintf(stderr, "rlo: part %d: its own %s region at %p (%llu bytes) shows %016llx since creation, "
                             "not its nonce %016llx\n", q, names[i], own[i],
                             (unsigned long long)(i == 2 ? L.heap_bytes[q] : 0), (unsigned long long)got,
                             (unsigned long long)region_nonce(w->nonce, i));
                return RLO_E_STALE;
            }
        }
    } else if (b.token == tok) {  // same process: the addresses are usable as they are
        if (b.device != w->device) {
            hipError_t e = hipDeviceEnablePeerAccess(b.device, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) { g_last_hip = (int)e; return RLO_E_HIP; }
            (void)hipGetLastError();
        }
        w->pf[q] = (uint8_t*)(uintptr_t)b.fwd_ptr;
        w->pv[q] = (uint8_t*)(uintptr_t)b.vote_ptr;
        w->pc[q] = (uint64_t*)(uintptr_t)b.ctrl_ptr;
        w->ph[q] = (uint8_t*)(uintptr_t)b.heap_ptr;
        w->pbf[q] = (uint8_t*)(uintptr_t)b.bflag_ptr;
    } else {  // another process: map its regions (dmabuf IPC; xGMI when on another GPU)
        void* p = nullptr;
        HIPCHK(open_import(&p, b.hf, w->device));
        w->opened.push_back(p);
        w->pf[q] = (uint8_t*)p;
        HIPCHK(open_import(&p, b.hv, w->device));
        w->opened.push_back(p);
        w->pv[q] = (uint8_t*)p;
        HIPCHK(open_import(&p, b.hc, w->device));
        w->opened.push_back(p);
        w->pc[q] = (uint64_t*)p;
        if (L.bulk_max) {
            HIPCHK(open_import(&p, b.hh, w->device));
            w->opened.push_back(p);
            w->ph[q] = (uint8_t*)p;
            HIPCHK(open_import(&p, b.hb, w->device));
            w->opened.push_back(p);
            w->pbf[q] = (uint8_t*)p;
        }
        // every mapped region must show the peer's creation nonce (rlo_part_create)
        const void* regs[5] = {w->pc[q] + rlo::kCtrlNonceWord, w->pv[q], L.bulk_max ? w->ph[q] : nullptr,
                               w->pf[q] + L.fwd_bytes[q], L.bulk_max ? w->pbf[q] + L.bflag_bytes[q] : nullptr};
        for (int i = 0; i < 5; i++) {
            if (!regs[i]) continue;
            uint64_t got = 0;
            HIPCHK(hipMemcpy(&got, regs[i], 8, hipMemcpyDeviceToHost));
            if (got != region_nonce(b.nonce, i)) {
                static const char* const names[5] = {"control", "vote", "heap", "forward", "bulk-flag"};
                // (what the mapping shows: 0 = never written, another nonce = an earlier allocation of that part)
                const uint64_t eva[5] = {b.ctrl_ptr, b.vote_ptr, b.heap_ptr, b.fwd_ptr, b.bflag_ptr};
                std::fprintf(stderr, "rlo: part %d: the %s region of part %d (at %#llx there), as mapped here at %p, shows "
                             "%016llx, not its nonce %016llx (its other regions' words:",
                             w->part, names[i], q, (unsigned long long)eva[i], regs[i], (unsigned long long)got,
                             (unsigned long long)region_nonce(b.nonce, i));
                for (int k = 0; k < 5; k++) {
                    uint64_t g2 = 0;
                    if (regs[k] && hipMemcpy(&g2, regs[k], 8, hipMemcpyDeviceToHost) == hipSuccess)
                        std::fprintf(stderr, " %s %016llx", names[k], (unsigned long long)g2);
                }
                std::fprintf(stderr, ")\n");
                return RLO_E_STALE;
            }
        }
    }
    w->peer_done[q] = 1;
    return RLO_OK;
}

int rlo_part_import(rlo_world_t* w, const void* blob, int q) {
    if (!w || !blob || q < 0 || q >= w->L.nparts || w->connected) return RLO_E_INVAL;
    HIPCHK(hipSetDevice(w->device));
    peer_tables(w, w->L.nparts);
    PartBlob b;
    std::memcpy(&b, blob, sizeof b);
    if (!blob_ok(w, b, q, w->L.nparts)) return RLO_E_INVAL;
    if (w->peer_done[q]) return RLO_OK;
    return import_peer(w, b, q);
}

int rlo_part_connect(rlo_world_t* w, const void* blobs, int n_parts) {
    if (!w || !blobs || n_parts != w->L.nparts || w->connected) return RLO_E_INVAL;
    HIPCHK(hipSetDevice(w->device));
    const Layout& L = w->L;
    peer_tables(w, n_parts);
    for (int q = 0; q < n_parts; q++) {
        PartBlob b;
        std::memcpy(&b, (const uint8_t*)blobs + (size_t)q * RLO_PART_BLOB_BYTES, sizeof b);
        if (!blob_ok(w, b, q, n_parts)) return RLO_E_INVAL;
        if (w->peer_done[q]) continue;  // (rlo_part_import did it)
        const int rc = import_peer(w, b, q);
        if (rc) return rc;
    }
    build_topo(w);
    if (w->d_topo.upload(w->topo)) return RLO_E_HIP;
    if (L.bulk_max) {  // the tables the movers and progress workgroups address the heaps with
        std::vector<uint64_t> hb(n_parts), fb(n_parts);
        for (int q = 0; q < n_parts; q++) {
            hb[q] = (uint64_t)(uintptr_t)w->ph[q];
            fb[q] = (uint64_t)(uintptr_t)w->pbf[q];
        }
        std::vector<int32_t> po(L.part_of.begin(), L.part_of.end()), pbv(L.pb.begin(), L.pb.end());
        if (w->d_bheap.upload(hb) || w->d_bflag.upload(fb) || w->d_part_of.upload(po) || w->d_part_begin.upload(pbv))
            return RLO_E_HIP;
    }
    w->connected = true;
    return RLO_OK;
}

int rlo_world_create(const rlo_world_cfg_t* cfg, rlo_world_t** out) {
    if (!cfg || !out || cfg->n_ranks < 2 || cfg->n_ranks > 4096) return RLO_E_INVAL;
    rlo_part_cfg_t pc;
    std::memset(&pc, 0, sizeof pc);
    pc.n_ranks = cfg->n_ranks;
    pc.n_parts = 1;
    pc.part = 0;
    pc.max_payload = cfg->max_payload;
    pc.ring_slots = cfg->ring_slots;
    pc.device = cfg->device;
    pc.bulk_max = cfg->bulk_max;
    pc.bulk_slots = cfg->bulk_slots;
    pc.movers = cfg->movers;
    pc.proposal_pool = cfg->proposal_pool;
    pc.flags = cfg->flags & (RLO_PART_PEND_HBM | RLO_PART_CHUNKED | RLO_PART_ONE_XCD);
    rlo_world* w = nullptr;
    int rc = rlo_part_create(&pc, &w);
    if (rc) return rc;
    uint8_t blob[RLO_PART_BLOB_BYTES];
    rc = rlo_part_export(w, blob, sizeof blob);
    if (rc >= 0) rc = rlo_part_connect(w, blob, 1);
    if (rc) { rlo_world_destroy(w); return rc; }
    *out = w;
    return RLO_OK;
}

static void host_free(rlo_world* w);

int rlo_pool_trim(uint32_t what, uint64_t* freed_bytes) {
    std::vector<void*> regions, imports;
    uint64_t freed = 0;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (what & RLO_TRIM_IMPORTS) {
            for (size_t i = 0; i < g_imports.size();) {
                if (g_imports[i].refs == 0) {
                    imports.push_back(g_imports[i].p);
                    g_imports.erase(g_imports.begin() + (long)i);
                } else {
                    i++;
                }
            }
        }
        if (what & (RLO_TRIM_FREE | RLO_TRIM_EXPORTED)) {
            for (size_t i = 0; i < g_pool.size();) {
                const PoolEnt q = g_pool[i];
                if (!q.exported && (what & RLO_TRIM_FREE)) {
                    regions.push_back(q.p);
                    freed += q.bytes;
                } else if (q.exported && (what & RLO_TRIM_EXPORTED)) {
                    g_retired.push_back(q);
                } else {
                    i++;
                    continue;
                }
                g_pool.erase(g_pool.begin() + (long)i);
            }
        }
        if (what & RLO_TRIM_RETIRED) {
            for (const PoolEnt& q : g_retired) {
                regions.push_back(q.p);
                freed += q.bytes;
            }
            g_retired.clear();
        }
    }
    for (void* d : imports) (void)hipIpcCloseMemHandle(d);
    for (void* d : regions) (void)hipFree(d);
    if (freed_bytes) *freed_bytes = freed;
    return RLO_OK;
}

int rlo_pool_stats(uint64_t* out, uint32_t cap) {
    if (!out || cap < 6) return RLO_E_INVAL;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    uint64_t v[6] = {0, 0, 0, 0, 0, 0};
    for (const PoolEnt& q : g_pool_live) v[0] += q.bytes;
    for (const PoolEnt& q : g_pool) v[q.exported ? 2 : 1] += q.bytes;
    for (const PoolEnt& q : g_retired) v[3] += q.bytes;
    for (const ImpEnt& e : g_imports) v[e.refs ? 4 : 5]++;
    for (int i = 0; i < 6; i++) out[i] = v[i];
    return RLO_OK;
}

int rlo_part_close_imports(rlo_world_t* w) {
    if (!w) return RLO_E_INVAL;
    HIPCHK(hipSetDevice(w->device));
    for (void* p : w->opened) close_import(p);
    w->opened.clear();
    w->connected = false;
    w->pf.clear();  // (a new connection maps the peers again)
    return RLO_OK;
}

int rlo_world_destroy(rlo_world_t* w) {
    if (!w) return RLO_E_INVAL;
    (void)hipSetDevice(w->device);
    for (void* p : w->opened) close_import(p);
    w->opened.clear();
    for (void* r : {(void*)w->fwd, (void*)w->vote, (void*)w->ctrl, (void*)w->heap, (void*)w->bflag, (void*)w->jmem,
                    (void*)w->pend_mem})
        release_region(r);
    w->d_bheap.release(); w->d_bflag.release(); w->d_part_of.release(); w->d_part_begin.release();
    w->d_topo.release(); w->d_stats.release();
    w->d_sched_off.release(); w->d_expect_bcast.release(); w->d_prop_off.release(); w->d_expect_dec.release();
    w->d_sched_ids.release(); w->d_prop_data_off.release(); w->d_prop_data_len.release(); w->d_isp_off.release();
    w->d_lat_count.release(); w->d_lat_round.release(); w->d_lat_origin.release(); w->d_prop_pid.release();
    w->d_lat_out.release(); w->d_lat_own_off.release(); w->d_lat_own.release(); w->d_mask.release(); w->d_prop_data.release(); w->d_log_payload.release();
    w->d_isp.release(); w->d_log.release();
    if (w->d_xcd) (void)hipFree(w->d_xcd);
    host_free(w);
    if (w->ev0) (void)hipEventDestroy(w->ev0);
    if (w->ev1) (void)hipEventDestroy(w->ev1);
    delete w;
    return RLO_OK;
}

int rlo_world_query(const rlo_world_t* w, rlo_world_info_t* o) {
    if (!w || !o) return RLO_E_INVAL;
    std::memset(o, 0, sizeof *o);
    o->n_ranks = w->L.n;
    o->max_in_degree = w->L.max_in;
    o->max_fanout = w->L.max_fan;
    o->edges = (int)w->L.E.size();
    o->ring_slots = w->L.cap;
    o->slot_stride = w->L.stride;
    o->vote_slots = w->L.vote_cap;
    o->fwd_bytes = w->L.fwd_bytes[w->part];
    o->vote_bytes = w->L.vote_bytes[w->part];
    o->ctrl_bytes = w->L.ctrl_words[w->part] * 8;
    o->cus = w->cus;
    o->blocks_per_cu = w->blocks_per_cu;
    o->part = w->part;
    o->n_parts = w->L.nparts;
    o->rank_begin = w->rb;
    o->rank_end = w->rb + w->nl;
    o->sys_scope = w->sys_scope;
    o->peers = w->peers;
    o->waves = w->waves;
    o->bulk_slots = w->L.bslots;
    o->movers = w->nmov;
    o->bulk_max = w->L.bulk_max;
    o->heap_bytes = w->L.heap_bytes[w->part];
    o->proposal_pool = w->L.pend_slots;
    o->pull = w->L.pull && w->nsmall >= 2 ? 1u : 0u;  // as Params.pull
    o->nsmall = w->nsmall;
    o->stage2_bytes = w->stage2;
    o->ll_ok = w->ll_ok ? 1u : 0u;
    o->pend_hbm = w->pend_hbm ? 1u : 0u;
    o->dyn_lds = (uint32_t)w->dyn_lds;
    o->last_kernel = w->last_hop ? 1u : 0u;
    o->static_lds = (uint32_t)rlo_kernel_static_lds(w->variant);
    return RLO_OK;
}

// doorbells (rlo_device.hpp) for the latency / IAR / host programs: their lone messages are what a
// bell carries.  Where the doorbell instantiation of the world's kernel is co-resident (its 4-wave forms
// may take one wave per SIMD: worlds whose ranks have a CU each); the 8-wave one has no large-message
// path, so there the program's longest message (max_msg payload bytes) must take the small copy path.
// RLO_NO_LL (diagnostics build) turns bells off
static uint32_t ll_mode(const rlo_world* w, uint32_t max_msg) {
    if (!w->ll_ok || diag_env("RLO_NO_LL")) return 0u;
    if (w->variant == 8 && (rlo::kHdr + max_msg + 15u) / 16u > w->nsmall) return 0u;
    return rlo::MODE_LL;
}

static void base_params(rlo_world* w) {
    // the previous program is gone from here on: a setup that fails below leaves no half-set program a later
    // rlo_launch could run
    w->have_program = false;
    rlo::Params& P = w->P;
    std::memset(&P, 0, sizeof P);
    P.n = w->L.n;
    P.rank_begin = w->rb;
    P.rank_end = w->rb + w->nl;
    P.topo = w->d_topo.p;
    P.fwd_region = w->fwd;
    P.fwd_region_bytes = (uint32_t)std::max<uint64_t>(w->L.fwd_bytes[w->part], 1);
    P.fwd_cap = w->L.cap;
    P.fwd_stride = w->L.stride;
    P.vote_region = w->vote;
    P.vote_region_bytes = (uint32_t)std::max<uint64_t>(w->L.vote_bytes[w->part], 1);
    P.vote_cap = w->L.vote_cap;
    P.ctrl = w->ctrl;
    P.ctrl_bytes = (uint32_t)(w->L.ctrl_words[w->part] * 8);
    P.sys_scope = (uint32_t)w->sys_scope;
    P.n_parts = (uint32_t)w->L.nparts;
    for (int q = 0; q < w->L.nparts; q++) P.err_flag[q] = reinterpret_cast<uint32_t*>(w->pc[q]);
    P.error_flag = reinterpret_cast<uint32_t*>(w->ctrl);
    P.stats = w->d_stats.p;
    P.nsmall = w->nsmall;
    P.nout_max = 2u * (uint32_t)w->L.max_fan;
    P.stage2_bytes = w->stage2;
    P.timeout_ticks = 100000000ull * 10;   // 10 s without progress on a rank
    P.deadline_ticks = 100000000ull * 120; // 120 s per launch
    P.window = 32;
    P.n_local = (uint32_t)w->nl;
    P.ring_cap = w->L.stride - rlo::kHdr;
    P.pend_slots = w->L.pend_slots;
    P.pend_hbm = reinterpret_cast<rlo::PendState*>(w->pend_mem);
    P.pull = w->L.pull && w->nsmall >= 2 ? 1u : 0u;  // the reference chunk is staged as chunk 1
    P.relay_cap = w->L.relay_cap;
    P.own_pool = 1;  // one own proposal per engine (rootless_ops.c:241) unless a program asks for more
    if (w->L.bulk_max) {
        const JobMem m = job_mem(w->jslots, (uint32_t)w->nl);
        P.bulk_slots = w->L.bslots;
        P.bulk_cap = w->L.bcap;
        P.nmov = w->nmov;
        P.bulk_cross = ((w->peers & RLO_PEER_OTHER_GPU) || (w->flags & RLO_PART_CHUNKED)) ? 1u : 0u;  // the chunked plan (rlo_device.hpp)
        P.bheap = w->d_bheap.p;
        P.bflag = w->d_bflag.p;
        P.part_of = w->d_part_of.p;
        P.part_begin = w->d_part_begin.p;
        P.jslots = w->jslots;
        P.bpend_off = w->bpend_off;
        P.jobs = reinterpret_cast<rlo::BulkJob*>(w->jmem + m.jobs);
        P.jctl = reinterpret_cast<uint64_t*>(w->jmem + m.jctl);
        P.jclaim = reinterpret_cast<uint64_t*>(w->jmem + m.jclaim);
        P.jfree = reinterpret_cast<uint64_t*>(w->jmem + m.jfree);
        P.jdone = reinterpret_cast<uint32_t*>(w->jmem + m.jdone);
        P.jsum = reinterpret_cast<uint64_t*>(w->jmem + m.jsum);
    }
}

static int setup_log(rlo_world* w, uint32_t flags, uint32_t log_cap, bool payload) {
    rlo::Params& P = w->P;
    if (!(flags & RLO_FLAG_LOG)) return RLO_OK;
    if (log_cap == 0) log_cap = 1024;
    if (w->d_log.alloc((size_t)w->nl * log_cap)) return RLO_E_HIP;
    P.log = w->d_log.p;
    P.log_cap = log_cap;
    P.mode |= rlo::MODE_LOG;
    if (payload) {
        P.log_stride = w->max_payload;
        if (w->d_log_payload.alloc((size_t)w->nl * log_cap * P.log_stride)) return RLO_E_HIP;
        P.log_payload = w->d_log_payload.p;
    }
    return RLO_OK;
}

int rlo_program_storm(rlo_world_t* w, const rlo_storm_cfg_t* cfg) {
    if (!w || !cfg || cfg->k < 0 || cfg->k > 0xFFFFFFFFll || cfg->order > RLO_ORDER_SLOTS) return RLO_E_INVAL;
    const uint32_t hi = std::max(cfg->len, cfg->len_max);
    // longer than a slot: a bulk message (bulk worlds only); mixed lengths: the bulk kernel only
    if (hi > (w->L.bulk_max ? w->L.bulk_max : w->max_payload)) return RLO_E_INVAL;
    if (cfg->len_max > cfg->len && !w->L.bulk_max) return RLO_E_INVAL;
    if (!w->connected) return RLO_E_NOTCONNECTED;
    base_params(w);
    rlo::Params& P = w->P;
    const int n = w->L.n, nl = w->nl, rb = w->rb;
    // the whole world's schedule is a pure function of (seed, k): each part keeps its own ranks'
    std::vector<int64_t> off(nl + 1, 0), expect(nl, 0), per(n, 0);
    std::vector<uint32_t> org((size_t)std::max<int64_t>(cfg->k, 1));
    for (int64_t b = 0; b < cfg->k; b++) {
        org[b] = cfg->order == RLO_ORDER_SLOTS ? (uint32_t)(b % n)
                                               : (uint32_t)(splitmix64(cfg->seed + (uint64_t)b) % (uint64_t)n);
        per[org[b]]++;
        if ((int)org[b] >= rb && (int)org[b] < rb + nl) off[org[b] - rb + 1]++;
    }
    for (int r = 0; r < nl; r++) off[r + 1] += off[r];
    std::vector<uint32_t> ids((size_t)std::max<int64_t>(off[nl], 1));
    std::vector<int64_t> fill(off.begin(), off.end() - 1);
    for (int64_t b = 0; b < cfg->k; b++)
        if ((int)org[b] >= rb && (int)org[b] < rb + nl) ids[fill[org[b] - rb]++] = (uint32_t)b;
    for (int r = 0; r < nl; r++) expect[r] = cfg->k - per[rb + r];
    if (w->d_sched_off.upload(off) || w->d_sched_ids.upload(ids) || w->d_expect_bcast.upload(expect)) return RLO_E_HIP;
    P.mode = rlo::MODE_STORM | ((cfg->flags & RLO_FLAG_HIST) ? rlo::MODE_HIST : 0u) |
             ((cfg->flags & RLO_FLAG_PROF) ? rlo::MODE_PROF : 0u);
    P.seed = cfg->seed;
    P.len = cfg->len;
    P.len_lo = cfg->len;
    P.len_hi = hi;
    P.storm_order = cfg->order;
    P.window = std::min<uint32_t>(cfg->window ? cfg->window : 64, 64u);  // one wave prefetches the ids
    P.sched_off = w->d_sched_off.p;
    P.sched_ids = w->d_sched_ids.p;
    P.expect_bcast = w->d_expect_bcast.p;
    int rc = setup_log(w, cfg->flags, cfg->log_cap, true);
    if (rc) return rc;
    w->have_program = true;
    return RLO_OK;
}

int rlo_program_latency(rlo_world_t* w, uint32_t rounds, uint32_t len, uint64_t seed, uint32_t flags) {
    if (!w || rounds == 0 || len > (w->L.bulk_max ? w->L.bulk_max : w->max_payload)) return RLO_E_INVAL;
    if (!w->connected) return RLO_E_NOTCONNECTED;
    // sharded: the round word and counts are part 0's copy, peer-mapped (rlo_device.hpp kLatWords)
    if (w->L.nparts != 1 && rounds > (uint32_t)rlo::kLatCap) return RLO_E_INVAL;
#ifndef RLO_DIAG
    if (flags & RLO_FLAG_TIMELINE) return RLO_E_INVAL;  // (the diagnostics build's: make DIAG=1)
#endif
    base_params(w);
    rlo::Params& P = w->P;
    const int n = w->L.n;
    std::vector<int32_t> org(rounds);
    std::vector<int64_t> expect(w->nl, 0);  // per LOCAL rank (the kernel indexes by workgroup)
    for (uint32_t i = 0; i < rounds; i++) org[i] = (int32_t)(splitmix64(seed + i) % (uint64_t)n);
    for (int lr = 0; lr < w->nl; lr++)
        for (uint32_t i = 0; i < rounds; i++) expect[lr] += org[i] != w->rb + lr;
    // per local rank the rounds it originates, in order (the kernel prefetches the next one)
    std::vector<uint32_t> own_off(w->nl + 1, 0), own;
    for (int lr = 0; lr < w->nl; lr++) {
        for (uint32_t i = 0; i < rounds; i++)
            if (org[i] == w->rb + lr) own.push_back(i);
        own_off[lr + 1] = (uint32_t)own.size();
    }
    if (own.empty()) own.push_back(0);
    if (w->d_lat_own_off.upload(own_off) || w->d_lat_own.upload(own)) return RLO_E_HIP;
    if (w->d_lat_origin.upload(org) || w->d_expect_bcast.upload(expect) || w->d_lat_count.alloc(rounds) ||
        w->d_lat_out.alloc(rounds) || w->d_lat_round.alloc(1) || w->d_lat_obs.alloc(rounds))
        return RLO_E_HIP;
    P.mode = rlo::MODE_LAT | ((flags & RLO_FLAG_HIST) ? rlo::MODE_HIST : 0u) | ((flags & RLO_FLAG_PROF) ? rlo::MODE_PROF : 0u) |
             ll_mode(w, len);
    P.len = len;
    P.seed = seed;
    P.lat_rounds = rounds;
    P.hop_chunks = (rlo::kHdr + len + 15u) / 16u;
    P.lat_origin = w->d_lat_origin.p;
    P.lat_count = w->d_lat_count.p;
    P.lat_out = w->d_lat_out.p;
    P.lat_round = w->d_lat_round.p;
    P.lat_obs = w->d_lat_obs.p;
    if (w->L.nparts != 1) {
        uint64_t* blk = w->pc[0] + w->L.lat_base[0];
        P.lat_round = reinterpret_cast<uint32_t*>(blk);
        P.lat_count = reinterpret_cast<uint32_t*>(blk + 16);
    }
    P.lat_own_off = w->d_lat_own_off.p;
    P.lat_own = w->d_lat_own.p;
    P.expect_bcast = w->d_expect_bcast.p;
    w->lat_rounds = rounds;
    w->tl_rows = 0;
    P.tl = nullptr;
    P.tl_rounds = 0;
    if (flags & RLO_FLAG_TIMELINE) {
        w->tl_rows = std::min<uint32_t>(rounds, rlo::kTlRoundsMax);
        if (w->d_tl.alloc((size_t)w->tl_rows * (rlo::kTlGlobal + rlo::kTlCols * (uint32_t)w->nl))) return RLO_E_HIP;
        P.tl = w->d_tl.p;
        P.tl_rounds = w->tl_rows;
        P.mode |= rlo::MODE_TL;
    }
    int rc = setup_log(w, flags, 0, true);
    if (rc) return rc;
    w->have_program = true;
    return RLO_OK;
}

// the device judge registry (rlo_kernel.hip judge_eval) and its per-rank tables, for every world
// rank (a part uses its own ranks' entries)
static int set_judge(rlo_world* w, const rlo_iar_cfg_t* cfg) {
    const int n = w->L.n;
    rlo::Params& P = w->P;
    if (cfg->judge_kind > RLO_JUDGE_HASH) return RLO_E_INVAL;
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
    return RLO_OK;
}

int rlo_program_iar(rlo_world_t* w, const rlo_iar_cfg_t* cfg, int64_t nprop, const int32_t* origin, const int32_t* pid,
                    const uint8_t* data, const uint32_t* data_off, const uint32_t* data_len) {
    if (!w || !cfg || nprop < 0 || (nprop && (!origin || !pid || !data_off || !data_len))) return RLO_E_INVAL;
    if (!w->connected) return RLO_E_NOTCONNECTED;
    const uint32_t pool = cfg->pool ? cfg->pool : 1u;
    if (pool > w->L.pend_slots) return RLO_E_INVAL;  // the world's proposal_pool bounds it
    base_params(w);
    rlo::Params& P = w->P;
    P.own_pool = pool;
    const int n = w->L.n, nl = w->nl, rb = w->rb;
    std::vector<int64_t> off(nl + 1, 0), expect(nl, 0), per(n, 0);
    for (int64_t i = 0; i < nprop; i++) {
        if (origin[i] < 0 || origin[i] >= n) return RLO_E_INVAL;
        if (16ull + data_len[i] > w->max_payload) return RLO_E_INVAL;
        per[origin[i]]++;
        if (origin[i] >= rb && origin[i] < rb + nl) off[origin[i] - rb + 1]++;
    }
    for (int r = 0; r < nl; r++) off[r + 1] += off[r];
    std::vector<int64_t> fill(off.begin(), off.end() - 1);
    const size_t nown = (size_t)std::max<int64_t>(off[nl], 1);
    std::vector<int32_t> ppid(nown);
    std::vector<uint32_t> pdo(nown), pdl(nown);
    std::vector<uint8_t> blob;
    for (int64_t i = 0; i < nprop; i++) {
        if (origin[i] < rb || origin[i] >= rb + nl) continue;
        int64_t at = fill[origin[i] - rb]++;
        ppid[at] = pid[i];
        pdo[at] = (uint32_t)blob.size();
        pdl[at] = data_len[i];
        blob.insert(blob.end(), data + data_off[i], data + data_off[i] + data_len[i]);
    }
    if (blob.empty()) blob.push_back(0);
    for (int r = 0; r < nl; r++) expect[r] = nprop - per[rb + r];
    if (w->d_prop_off.upload(off) || w->d_prop_pid.upload(ppid) || w->d_prop_data_off.upload(pdo) ||
        w->d_prop_data_len.upload(pdl) || w->d_prop_data.upload(blob) || w->d_expect_dec.upload(expect))
        return RLO_E_HIP;
    uint32_t max_msg = 23;  // a decision's PBuf (:908-917); a proposal's is 16 B + its data
    for (int64_t i = 0; i < nprop; i++) max_msg = std::max<uint32_t>(max_msg, 16u + data_len[i]);
    P.mode = rlo::MODE_IAR | ((cfg->flags & RLO_FLAG_PROF) ? rlo::MODE_PROF : 0u) | ll_mode(w, max_msg);
    P.hop_chunks = (rlo::kHdr + max_msg + 15u) / 16u;
    {
        const int jrc = set_judge(w, cfg);
        if (jrc) return jrc;
    }
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

static void host_free(rlo_world* w) {
    if (w->cmd_host) {
        if (w->h_cmd) (void)hipHostFree(w->h_cmd);
        if (w->d_ctl) (void)hipHostFree(w->d_ctl);
    } else {
        if (w->h_cmd) (void)hipFree(w->h_cmd);
        if (w->d_ctl) (void)hipFree(w->d_ctl);
    }
    if (w->h_llc) (void)hipHostFree(w->h_llc);
    w->h_llc = nullptr;
    if (w->shm) {  // h_ctl / h_ev / h_evp point into the segment
        (void)hipHostUnregister(w->shm);
        munmap(w->shm, (size_t)w->shm_bytes);
        if (w->shm_linked) shm_unlink(w->shm_name.c_str());
        w->shm = nullptr;
        w->shm_linked = false;
    } else {
        if (w->h_ctl) (void)hipHostFree(w->h_ctl);
        if (w->h_ev) (void)hipHostFree(w->h_ev);
        if (w->h_evp) (void)hipHostFree(w->h_evp);
    }
    w->h_cmd = nullptr; w->d_ctl = nullptr; w->h_ctl = nullptr; w->h_ev = nullptr; w->h_evp = nullptr;
}

// uncached VRAM the CPU writes through the (large) BAR: the kernel polls it locally instead of
// paying a PCIe round trip per poll (tools/probe/bar_write.hip: 0.10 vs 1.2 us per poll).
// Uncached, not merely fine-grained: a fine-grained line can stay in the XCD's L2 and hide
// the CPU's store until it is evicted (ms-long stalls measured at 8 ranks).
static int bar_alloc(void** p, size_t bytes) {
    hipError_t e = hipExtMallocWithFlags(p, std::max<size_t>(bytes, 256), hipDeviceMallocUncached);
    if (e != hipSuccess) { g_last_hip = (int)e; *p = nullptr; return RLO_E_HIP; }
    std::memset(*p, 0, std::max<size_t>(bytes, 256));  // through the BAR: also checks CPU access
    return RLO_OK;
}

// CPU stores through the BAR pass the GPU's host data path (HDP), which can hold them for up to ~1 ms
// before a polling kernel sees them, uncached VRAM or not: drop-in IAR rounds at 8 ranks were
// bimodal, 110 us or 1.1 ms (profiles/r2_dropin_hdp.txt).  Writing the HDP flush register after a
// batch of BAR stores pushes them to memory at once (what RCCL's host proxy does for its flags)
static void hdp_flush(const rlo_world* w) {
    if (!w->hdp) return;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // the BAR stores (write-combined) before the flush
    *w->hdp = 1u;
}

static int host_alloc(void** p, size_t bytes) {
    // coherent (fine-grained) pinned memory: the kernel polls words the CPU writes and vice versa
    hipError_t e = hipHostMalloc(p, std::max<size_t>(bytes, 256), hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) { g_last_hip = (int)e; *p = nullptr; return RLO_E_HIP; }
    std::memset(*p, 0, std::max<size_t>(bytes, 256));
    return RLO_OK;
}

// rlo_host_share's segment (rlo_shm.hpp), built by rlo_program_host once the ring sizes are known:
// created, mapped, registered with HIP (fine-grained: the kernel's counter / event stores reach the
// clients' polls directly) and described in its header for the clients
static int shm_build(rlo_world* w, const uint64_t** dev_hctl, const rlo::LogRec** dev_ev, const uint8_t** dev_evp,
                     uint8_t** dev_cmd, uint64_t** dev_cli, uint8_t** dev_llc) {
    const uint32_t nl = (uint32_t)w->nl;
    const uint64_t stage = w->L.bulk_max ? w->share_stage : 0;
    const rlo::ShmLayout L = rlo::shm_layout(nl, w->cmd_cap, w->pk_cap, w->L.stride, w->pk_stride, stage);
    const char* name = w->shm_name.c_str();
    const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return RLO_E_INVAL;
    if (ftruncate(fd, (off_t)L.total) != 0) { close(fd); shm_unlink(name); return RLO_E_INVAL; }
    void* p = mmap(nullptr, (size_t)L.total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) { shm_unlink(name); return RLO_E_INVAL; }
    // MTYPE_UC (hipExtHostRegisterUncached), as hipHostMallocCoherent: the kernel's counter / event stores
    // must not linger in its L2 (a default registration showed ms-long delays per pickup)
    hipError_t e = hipHostRegister(p, (size_t)L.total, hipHostRegisterMapped | hipExtHostRegisterUncached);
    void* dp = nullptr;
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, p, 0);
    if (e != hipSuccess) {
        g_last_hip = (int)e;
        munmap(p, (size_t)L.total);
        shm_unlink(name);
        return RLO_E_HIP;
    }
    uint8_t* b = (uint8_t*)p;
    uint8_t* db = (uint8_t*)dp;
    w->shm = b;
    w->shm_bytes = L.total;
    w->shm_linked = true;
    w->SL = L;
    w->h_ctl = (uint64_t*)(b + L.hctl);
    w->h_ev = (rlo::LogRec*)(b + L.ev);
    w->h_evp = b + L.evp;
    w->cli_req.assign(nl, 0);
    *dev_hctl = (const uint64_t*)(db + L.hctl);
    *dev_ev = (const rlo::LogRec*)(db + L.ev);
    *dev_evp = db + L.evp;
    *dev_cmd = db + L.cmd;
    *dev_cli = (uint64_t*)(db + L.cli);
    *dev_llc = db + L.llc;
    rlo::ShmHdr* h = (rlo::ShmHdr*)b;
    h->version = rlo::kShmVersion;
    h->nl = nl;
    h->rb = (uint32_t)w->rb;
    h->n = (uint32_t)w->L.n;
    h->bslots = w->L.bslots;
    h->cmd_cap = w->cmd_cap;
    h->pk_cap = w->pk_cap;
    h->stride = w->L.stride;
    h->max_payload = w->pk_stride;  // (the pickup payload stride)
    h->bulk_max = w->L.bulk_max;
    h->stage_bytes = stage;
    h->off_hctl = L.hctl; h->off_ev = L.ev; h->off_evp = L.evp; h->off_cli = L.cli; h->off_cmd = L.cmd;
    h->off_stage = L.stage; h->total = L.total; h->off_llc = L.llc;
    __atomic_store_n(&h->magic, rlo::kShmMagic, __ATOMIC_RELEASE);  // clients check it last
    return RLO_OK;
}

int rlo_program_host(rlo_world_t* w, const rlo_host_cfg_t* cfg) {
    if (!w) return RLO_E_INVAL;
    if (!w->connected) return RLO_E_NOTCONNECTED;
    const uint32_t cc = cfg && cfg->cmd_slots ? pow2_ceil(cfg->cmd_slots) : 256u;
    const uint32_t pc = cfg && cfg->pickup_slots ? pow2_ceil(cfg->pickup_slots) : 1024u;
    if (pc < 64 || pc > rlo::kPkMaxSlots || cc < 4 || (uint64_t)cc * w->L.stride > 0xFFFF0000ull) return RLO_E_INVAL;
    const uint32_t pool = cfg && cfg->pool ? cfg->pool : 1u;
    if (pool > w->L.pend_slots) return RLO_E_INVAL;
    HIPCHK(hipSetDevice(w->device));
    host_free(w);
    w->cmd_cap = cc;
    w->pk_cap = pc;
    const size_t nl = (size_t)w->nl;
    // Where the host's commands and counters live.  Default: pinned host memory, polled by the
    // kernel over PCIe (wave 0's poll of them runs beside its ring polls).  RLO_BAR_CMDS=1: uncached
    // VRAM written by the CPU through the BAR -- a local poll, but in some runs such a store stayed
    // invisible to the polling kernel for 0.5-2 ms, every round (profiles/r2_dropin_split_legs.txt:
    // forwarded -> consumed; the kernel itself drained each command within 20 us of seeing it)
    w->cmd_host = diag_env("RLO_BAR_CMDS") == nullptr;
    const int arc = w->cmd_host ? (host_alloc((void**)&w->h_cmd, nl * cc * w->L.stride) ||
                                   host_alloc((void**)&w->d_ctl, nl * rlo::kHctlWords * 8))
                                : (bar_alloc((void**)&w->h_cmd, nl * cc * w->L.stride) ||
                                   bar_alloc((void**)&w->d_ctl, nl * rlo::kHctlWords * 8));
    if (arc) {
        host_free(w);
        return RLO_E_HIP;
    }
    w->hdp = nullptr;
    if (!w->cmd_host && !diag_env("RLO_NO_HDP_FLUSH")) {  // A/B switch; the attribute returns the register's mapped address
        uint32_t* reg = nullptr;
        if (hipDeviceGetAttribute(reinterpret_cast<int*>(&reg), hipDeviceAttributeHdpMemFlushCntl, w->device) == hipSuccess)
            w->hdp = reg;
    }
    const uint64_t* dev_hctl = nullptr;
    const rlo::LogRec* dev_ev = nullptr;
    const uint8_t* dev_evp = nullptr;
    uint8_t* dev_cmd = nullptr;
    uint64_t* dev_cli = nullptr;
    uint8_t* dev_llc = nullptr;
    w->pk_stride = rlo::pk_payload_stride(w->max_payload);
    if (!w->shm_name.empty()) {  // rlo_host_share: the host-side rings in the shared segment
        int rc = shm_build(w, &dev_hctl, &dev_ev, &dev_evp, &dev_cmd, &dev_cli, &dev_llc);
        if (rc) { host_free(w); return rc; }
    } else if (host_alloc((void**)&w->h_ctl, nl * rlo::kHctlWords * 8) ||
               host_alloc((void**)&w->h_ev, nl * pc * rlo::kPkRecBytes) ||
               host_alloc((void**)&w->h_evp, nl * pc * w->pk_stride) ||
               (w->cmd_host && host_alloc((void**)&w->h_llc, nl * cc * rlo::kLLCmdSlot))) {
        host_free(w);
        return RLO_E_HIP;
    }
    w->cmd_tail.assign(nl, 0);
    w->pk_head.assign(nl, 0);
    base_params(w);
    rlo::Params& P = w->P;
    P.mode = rlo::MODE_HOST | rlo::MODE_IAR | ll_mode(w, w->L.stride - rlo::kHdr);  // a command fills up to a slot
    P.own_pool = pool;
    P.host_judge = 1;  // judge(data) / judge(NULL) are the host's callbacks (rlo_host_device_judge: the device's)
    P.log = dev_ev ? const_cast<rlo::LogRec*>(dev_ev) : w->h_ev;
    P.log_cap = pc;
    P.log_payload = dev_evp ? const_cast<uint8_t*>(dev_evp) : w->h_evp;
    P.log_stride = w->pk_stride;
    // shared service, commands in host memory: the kernel reads the clients' own rings and counters in
    // the segment (the proxy then only serves bulk requests)
    const bool direct = w->cmd_host && dev_cmd;
    P.hin = direct ? dev_cmd : w->h_cmd;
    P.hin_cap = cc;
    P.hctl = dev_hctl ? const_cast<uint64_t*>(dev_hctl) : w->h_ctl;
    P.hctl_dev = direct ? dev_cli : w->d_ctl;
    // command doorbells (rlo_shm.hpp): wherever the commands are in host memory
    P.hll = direct ? dev_llc : (w->cmd_host && !dev_cmd ? w->h_llc : nullptr);
    const uint64_t idle = cfg ? cfg->idle_timeout_s : 0;
    P.timeout_ticks = idle ? 100000000ull * idle : ~0ull >> 2;
    P.deadline_ticks = ~0ull >> 2;  // serves until RLO_CMD_QUIT
    w->have_program = true;
    return RLO_OK;
}

int rlo_host_post(rlo_world_t* w, int rank, const rlo_cmd_t* c, const void* payload, uint32_t len) {
    if (!w || !c || !w->h_cmd || rank < w->rb || rank >= w->rb + w->nl) return RLO_E_INVAL;
    if (len + rlo::kHdr > w->L.stride || len > 0xffffffu || (len && !payload)) return RLO_E_INVAL;
    const int lr = rank - w->rb;
    uint64_t* ctl = w->h_ctl + (size_t)lr * rlo::kHctlWords;
    uint64_t* dctl = w->d_ctl + (size_t)lr * rlo::kHctlWords;
    // shared service with commands in host memory (rlo_program_host "direct"): the kernel reads the
    // rank's own command ring and counter in the segment, so a command the leader posts itself (the
    // QUIT of a failed engine setup) goes there, behind whatever the rank's client posted
    const bool direct = w->shm && w->cmd_host;
    rlo::ClientBox* box = direct ? (rlo::ClientBox*)(w->shm + w->SL.cli) + lr : nullptr;
    const uint64_t tail = direct ? __atomic_load_n(&box->mtail, __ATOMIC_ACQUIRE) : w->cmd_tail[lr];
    const uint64_t head = __atomic_load_n(&ctl[rlo::kHctlInjHead], __ATOMIC_ACQUIRE);
    if (tail - head >= w->cmd_cap) return RLO_E_AGAIN;
    uint8_t* slot = (direct ? w->shm + w->SL.cmd : w->h_cmd) + ((size_t)lr * w->cmd_cap + (tail & (w->cmd_cap - 1))) * w->L.stride;
    uint32_t hdr[4];
    hdr[0] = (uint32_t)(c->origin & 0xffff) | ((c->kind & 0xffu) << 16) | ((uint32_t)(c->vote & 0xff) << 24);
    hdr[1] = (uint32_t)c->id;
    hdr[2] = (len & 0xffffffu) | ((c->pseq & 0xffu) << 24);
    hdr[3] = 0;
    std::memcpy(slot, hdr, sizeof hdr);
    if (len) std::memcpy(slot + rlo::kHdr, payload, len);
    uint8_t* llc = direct ? w->shm + w->SL.llc : w->h_llc;
    if (llc) rlo::ll_cmd_put(llc + ((size_t)lr * w->cmd_cap + (tail & (w->cmd_cap - 1))) * rlo::kLLCmdSlot, tail, hdr, payload, len);
    if (direct) {
        __atomic_store_n(&box->mtail, tail + 1, __ATOMIC_RELEASE);
        return RLO_OK;
    }
    w->cmd_tail[lr] = tail + 1;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // BAR stores may be write-combined: slot before tail
    __atomic_store_n(&dctl[rlo::kHctlInjTail], tail + 1, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // push the tail out now
    hdp_flush(w);
    return RLO_OK;
}

int rlo_host_poll(rlo_world_t* w, int rank, rlo_log_rec_t* ev, void* payload, uint32_t cap) {
    if (!w || !ev || !w->h_ev || rank < w->rb || rank >= w->rb + w->nl) return RLO_E_INVAL;
    const int lr = rank - w->rb;
    uint64_t* ctl = w->h_ctl + (size_t)lr * rlo::kHctlWords;
    const uint64_t head = w->pk_head[lr];
    // the next event as soon as its tagged units landed (rlo_shm.hpp pk_take)
    if (!rlo::pk_take(reinterpret_cast<const uint8_t*>(w->h_ev) + (size_t)lr * w->pk_cap * rlo::kPkRecBytes,
                      w->h_evp + (size_t)lr * w->pk_cap * w->pk_stride, w->pk_cap, w->pk_stride, w->pk_epoch, head,
                      &ctl[rlo::kHctlPkTail], reinterpret_cast<rlo::LogRec*>(ev), payload, cap))
        return 0;
    w->pk_head[lr] = head + 1;
    if (w->shm && w->cmd_host) {  // direct mode: the kernel polls the pickup head in the rank's ClientBox
        __atomic_store_n(&((rlo::ClientBox*)(w->shm + w->SL.cli) + lr)->mpk, head + 1, __ATOMIC_RELEASE);
        return 1;
    }
    __atomic_store_n(&w->d_ctl[(size_t)lr * rlo::kHctlWords + rlo::kHctlPkHead], head + 1, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // a write-combined BAR store would otherwise linger
    hdp_flush(w);
    return 1;
}

int rlo_host_cmd_count(rlo_world_t* w, int rank, uint64_t* consumed, uint64_t* posted) {
    if (!w || !w->h_ctl || rank < w->rb || rank >= w->rb + w->nl) return RLO_E_INVAL;
    const int lr = rank - w->rb;
    if (consumed) *consumed = __atomic_load_n(&w->h_ctl[(size_t)lr * rlo::kHctlWords + rlo::kHctlInjHead], __ATOMIC_ACQUIRE);
    if (posted) *posted = w->cmd_tail[lr];
    return RLO_OK;
}

int rlo_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rlo_device_numa_node(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return -1;
    for (char* c = bus; *c; c++) *c = (char)std::tolower((unsigned char)*c);
    char path[160];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE* f = std::fopen(path, "r");
    if (!f) return -1;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    return node;
}

int rlo_host_running(rlo_world_t* w) {
    if (!w) return RLO_E_INVAL;
    hipError_t e = hipEventQuery(w->ev1);
    if (e == hipErrorNotReady) return 1;
    if (e != hipSuccess) { g_last_hip = (int)e; return RLO_E_HIP; }
    return 0;
}

int rlo_reset(rlo_world_t* w, void* stream) {
    if (!w) return RLO_E_INVAL;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(w->device));
    if (w->have_program && (w->P.mode & rlo::MODE_HOST)) {  // the kernel is not running: rings restart at 0
        std::memset(w->h_ctl, 0, (size_t)w->nl * rlo::kHctlWords * 8);
        std::memset(w->d_ctl, 0, (size_t)w->nl * rlo::kHctlWords * 8);
        // the command doorbells restart too: the kernel takes a doorbell whose tag is the sequence it expects
        // next (ll_cmd_put), without the tail, so a relaunch that left the previous launch's tags in place
        // would replay that launch's first commands before the host posts anything
        if (w->h_llc) std::memset(w->h_llc, 0, (size_t)w->nl * w->cmd_cap * rlo::kLLCmdSlot);
        if (w->shm) {  // shared service: the clients' boxes restart too
            std::memset(w->shm + w->SL.llc, 0, (size_t)w->nl * w->cmd_cap * rlo::kLLCmdSlot);
            std::memset(w->shm + w->SL.cli, 0, (size_t)w->nl * sizeof(rlo::ClientBox));
            std::fill(w->cli_req.begin(), w->cli_req.end(), 0);
            __atomic_store_n(&((rlo::ShmHdr*)w->shm)->leader_failed, 0u, __ATOMIC_RELEASE);
        }
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        // the pickup ring restarts at sequence 0: records and tagged payload units a previous launch left behind are
        // cleared, so none can pass for this launch's event whatever the epochs (with 16-bit record tags and
        // a per-launch epoch step, the record of the launch 16 (pk_cap 64) .. 256 (pk_cap 1024) back in the same slot
        // could carry the expected tag).  A fresh world's memory is already zero
        if (w->pk_dirty) {
            if (w->h_ev) std::memset((void*)w->h_ev, 0, (size_t)w->nl * w->pk_cap * rlo::kPkRecBytes);
            if (w->h_evp) std::memset(w->h_evp, 0, (size_t)w->nl * w->pk_cap * w->pk_stride);
            w->pk_dirty = false;
        }
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        std::fill(w->cmd_tail.begin(), w->cmd_tail.end(), 0);
        std::fill(w->pk_head.begin(), w->pk_head.end(), 0);
    }
    // every control word but the creation nonce (a peer still connecting may read it)
    HIPCHK(hipMemsetAsync(w->ctrl, 0, rlo::kCtrlNonceWord * 8, s));
    HIPCHK(hipMemsetAsync(w->ctrl + rlo::kCtrlHdrWords, 0, (w->L.ctrl_words[w->part] - rlo::kCtrlHdrWords) * 8, s));
    // zeroed rings: a slot whose bytes are not visible yet reads without the header's slot mark
    // (rlo_device.hpp) and is reloaded, in every launch, not only in a fresh world
    HIPCHK(hipMemsetAsync(w->fwd, 0, w->L.fwd_bytes[w->part], s));
    HIPCHK(hipMemsetAsync(w->d_stats.p, 0, sizeof(rlo::RankStats) * w->nl, s));
    if (w->L.bulk_max) {  // bulk flags / release counts, job rings (generation 0: a slot takes its first sub-job)
        HIPCHK(hipMemsetAsync(w->bflag, 0, w->L.bflag_bytes[w->part], s));
        HIPCHK(hipMemsetAsync(w->jmem, 0, w->jmem_bytes, s));
        std::fill(w->host_bulk_q.begin(), w->host_bulk_q.end(), 0u);
    }
    if (w->have_program && (w->P.mode & rlo::MODE_LAT)) {
        HIPCHK(hipMemsetAsync(w->d_lat_count.p, 0, sizeof(uint32_t) * w->lat_rounds, s));
        HIPCHK(hipMemsetAsync(w->d_lat_out.p, 0, sizeof(uint64_t) * w->lat_rounds, s));
        HIPCHK(hipMemsetAsync(w->d_lat_round.p, 0, sizeof(uint32_t), s));
        HIPCHK(hipMemsetAsync(w->d_lat_obs.p, 0, sizeof(uint64_t) * w->lat_rounds, s));
        if (w->tl_rows)
            HIPCHK(hipMemsetAsync(w->d_tl.p, 0, sizeof(uint32_t) * w->tl_rows * (rlo::kTlGlobal + rlo::kTlCols * (uint32_t)w->nl), s));
        // sharded: part 0's control memset above clears the shared round word and counts
    }
    HIPCHK(hipStreamSynchronize(s));
    return RLO_OK;
}

// The hop kernel (rlo_hop.hip: one wave per rank, one message at a time) runs the latency and iar programs with
// doorbells (device judges, no host service, no bulk messages) whenever every rank-wave of the part is co-resident;
// the diagnostics modes that instrument the progress kernel's doorbell pass (phase profile, hop profile, the no-fast-path
// A/B) keep that kernel, and so does RLO_NO_HOP (diagnostics build: A/B of the two kernels)
static size_t hop_lds(const rlo_world* w) {
    // the pending-proposal table (iar only: the latency program launches without it, so more rank-waves share a CU)
    if (!(w->P.mode & rlo::MODE_IAR)) return 0;
    return w->P.pend_hbm ? 0 : (size_t)16u * (uint32_t)w->L.n * w->P.pend_slots;
}
static bool hop_eligible(rlo_world* w) {
    const rlo::Params& P = w->P;
    if (!(P.mode & rlo::MODE_LL) || !(P.mode & (rlo::MODE_LAT | rlo::MODE_IAR))) return false;
    if (P.mode & (rlo::MODE_HOST | rlo::MODE_STORM | rlo::MODE_PROF | rlo::MODE_HOPPROF | rlo::MODE_NOFAST)) return false;
    // the timeline (diagnostics build) is the hop kernel's too unless RLO_TL_FULL asks for the progress kernel's
    static const bool tl_full = diag_env("RLO_TL_FULL") != nullptr;
    if ((P.mode & rlo::MODE_TL) && tl_full) return false;
    if (w->L.bulk_max || P.hop_chunks == 0 || P.hop_chunks > 64u) return false;
    // iar: one own proposal in flight per rank in small worlds only.  The hop kernel takes one message at a time per
    // rank; with many proposals in flight per rank (the pool, or N of them reaching every rank of a large world) the
    // progress kernel's batches win: decisions/s 4 / 8 ranks 153 K / 148 K vs 113 K / 118 K, but 64 / 256 ranks 158 K /
    // 140 K vs 254 K / 618 K and pool 16 at 8 ranks 186 K vs 686 K (profiles/r6_hop_ab.txt)
    if ((P.mode & rlo::MODE_IAR) && (P.own_pool > 1 || w->L.n > 16)) return false;
    static const bool off = diag_env("RLO_NO_HOP") != nullptr;
    if (off) return false;
    const size_t lds = hop_lds(w);
    if (lds > 64u * 1024u) return false;
    int b = 0;
    if (rlo_occupancy_hop(&b, lds, P.pend_hbm ? 1 : 0) != hipSuccess) { (void)hipGetLastError(); return false; }
    // (RLO_PART_ONE_XCD: every rank-wave on the CUs of one XCD, an eighth of the GPU's)
    return b > 0 && (int64_t)b * (w->d_xcd ? w->cus / 8 : w->cus) >= (int64_t)w->nl;
}

int rlo_launch_ex(rlo_world_t* w, void* stream, uint32_t flags) {
    if (!w) return RLO_E_INVAL;
    if (!w->connected) return RLO_E_NOTCONNECTED;
    if (!w->have_program) return RLO_E_NOPROGRAM;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(w->device));
    if (!(flags & RLO_LAUNCH_NO_RESET)) {
        int rc = rlo_reset(w, stream);
        if (rc) return rc;
        if (w->P.mode & rlo::MODE_HOST) {
            // a new pickup-tag epoch: the rings restart at sequence 0, and a record or payload unit an earlier
            // launch left in a slot carries another epoch's tag, so it never passes for this launch's event
            // (even: tags stay odd, never the 0 of fresh memory).  Diagnostics build: RLO_PK_EPOCH_SAME keeps the
            // epoch, the worst case for stale records (tests/test_gpu_timeline.py: rlo_reset must clear them)
            static const bool same = diag_env("RLO_PK_EPOCH_SAME") != nullptr;
            if (!same) w->pk_epoch += 0x9E3779B8u;
            w->P.pk_epoch = w->pk_epoch;
            if (w->shm) __atomic_store_n(&((rlo::ShmHdr*)w->shm)->pk_epoch, w->pk_epoch, __ATOMIC_RELEASE);
        }
    }
    if (w->P.mode & rlo::MODE_HOST) w->pk_dirty = true;  // rlo_reset clears what this launch writes
    HIPCHK(hipEventRecord(w->ev0, s));
    // diagnostic A/B switch: publish producer counters after the next poll instead of at the end
    // of the iteration that drained the stores
    static const bool lazy = diag_env("RLO_LAZY_PUB") != nullptr;
    if (lazy) w->P.mode |= rlo::MODE_LAZYPUB;
    else w->P.mode &= ~rlo::MODE_LAZYPUB;
    static const bool nospin = diag_env("RLO_NO_IDLE_SPIN") != nullptr;  // diagnostic
    if (nospin) w->P.mode |= rlo::MODE_NOSPIN;
    else w->P.mode &= ~rlo::MODE_NOSPIN;
    static const bool noacq = diag_env("RLO_NO_ACQUIRE") != nullptr;  // diagnostic A/B, unsafe
    if (noacq) w->P.mode |= rlo::MODE_NOACQ;
    else w->P.mode &= ~rlo::MODE_NOACQ;
    static const bool nofast = diag_env("RLO_NO_FAST") != nullptr;  // A/B: no lone-message fast path
    if (nofast) w->P.mode |= rlo::MODE_NOFAST;
    else w->P.mode &= ~rlo::MODE_NOFAST;
    // A/B: large-message staging rounds pipelined over two halves of stage2 (measured slower than whole
    // rounds: 4 KiB storm 122 vs 109 ms, profiles/r2s4_pipe_ab.txt)
    static const bool pipe = [] {
        const char* e = diag_env("RLO_BIG_PIPE");
        return e && std::atoi(e) != 0;
    }();
    if (pipe) w->P.mode |= rlo::MODE_PIPE;
    else w->P.mode &= ~rlo::MODE_PIPE;
    static const bool hopprof = diag_env("RLO_HOP_PROF") != nullptr;  // diagnostic: clocks along a doorbell hop
    if (hopprof) w->P.mode |= rlo::MODE_HOPPROF;
    else w->P.mode &= ~rlo::MODE_HOPPROF;
    static const bool corrupt = diag_env("RLO_BULK_CORRUPT") != nullptr;  // test: VERIFY must catch a zeroed granule
    if (corrupt) w->P.mode |= rlo::MODE_CORRUPT;
    else w->P.mode &= ~rlo::MODE_CORRUPT;
    static const bool nohpw = diag_env("RLO_NO_HPOLLER") != nullptr;  // A/B: no wave-1 host poller
    if (nohpw) w->P.mode |= rlo::MODE_NOHPW;
    else w->P.mode &= ~rlo::MODE_NOHPW;
    static const bool hdiag = diag_env("RLO_HOST_DIAG") != nullptr;  // diagnostic: command-wait counters
    if (hdiag) w->P.mode |= rlo::MODE_HDIAG;
    else w->P.mode &= ~rlo::MODE_HDIAG;
    hipError_t e;
    if (w->d_xcd) {  // RLO_PART_ONE_XCD: the hop kernel on one XCD, or nothing
        if (!hop_eligible(w)) return RLO_E_INVAL;
        w->P.mode |= rlo::MODE_XCD1;
        w->P.xcd_word = w->d_xcd;  // (every program's base_params clears Params)
        HIPCHK(hipMemsetAsync(w->d_xcd, 0, 8, s));  // the placement rendezvous (rlo_hop.hip)
    }
    if (hop_eligible(w)) {
        w->last_hop = true;
        e = rlo_launch_hop(&w->P, w->nl, hop_lds(w), s);
    } else {
        w->last_hop = false;
        e = rlo_launch_progress(&w->P, w->nl + (w->L.bulk_max ? (int)w->nmov : 0), w->dyn_lds, s, w->variant);
    }
    if (e != hipSuccess) { g_last_hip = (int)e; return RLO_E_HIP; }
    HIPCHK(hipEventRecord(w->ev1, s));
    return RLO_OK;
}

int rlo_launch(rlo_world_t* w, void* stream) { return rlo_launch_ex(w, stream, 0); }

int rlo_stream_create(int device, void** stream) {
    if (!stream) return RLO_E_INVAL;
    if (device >= 0) HIPCHK(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void*)s;
    return RLO_OK;
}

int rlo_stream_destroy(void* stream) {
    if (!stream) return RLO_E_INVAL;
    HIPCHK(hipStreamDestroy((hipStream_t)stream));
    return RLO_OK;
}

int rlo_wait(rlo_world_t* w) {
    if (!w) return RLO_E_INVAL;
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipEventSynchronize(w->ev1));
    HIPCHK(hipEventElapsedTime(&w->last_ms, w->ev0, w->ev1));
    uint32_t err = 0;
    HIPCHK(hipMemcpy(&err, w->ctrl, sizeof err, hipMemcpyDeviceToHost));
    return err ? RLO_E_DEVICE : RLO_OK;
}

int rlo_bulk_debug(rlo_world_t* w, uint64_t* out, uint32_t cap) {
    if (!w || !out || !w->jmem) return RLO_E_INVAL;
    const JobMem m = job_mem(w->jslots, (uint32_t)w->nl);
    const uint32_t n = std::min<uint32_t>(cap, rlo::kJctlWords);
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipMemcpy(out, w->jmem + m.jctl, n * 8, hipMemcpyDeviceToHost));
    return (int)n;
}

int rlo_device_error(rlo_world_t* w, uint32_t* code, uint32_t* aux) {
    if (!w) return RLO_E_INVAL;
    uint32_t v[2] = {0, 0};
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipMemcpy(v, w->ctrl, sizeof v, hipMemcpyDeviceToHost));
    if (code) *code = v[0];
    if (aux) *aux = v[1];
    return RLO_OK;
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
    if (!w || !out || n < 0 || n > w->nl) return RLO_E_INVAL;
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipMemcpy(out, w->d_stats.p, sizeof(rlo::RankStats) * n, hipMemcpyDeviceToHost));
    return RLO_OK;
}

int rlo_log(rlo_world_t* w, int rank, rlo_log_rec_t* out, uint32_t cap, uint8_t* payload, uint32_t payload_stride) {
    if (!w || rank < w->rb || rank >= w->rb + w->nl || !out) return RLO_E_INVAL;
    if (!w->d_log.p) return RLO_E_NOPROGRAM;
    HIPCHK(hipSetDevice(w->device));
    const int lr = rank - w->rb;
    rlo::RankStats st;
    HIPCHK(hipMemcpy(&st, w->d_stats.p + lr, sizeof st, hipMemcpyDeviceToHost));
    uint32_t cnt = (uint32_t)std::min<uint64_t>(st.log_count, w->P.log_cap);
    cnt = std::min(cnt, cap);
    if (cnt) HIPCHK(hipMemcpy(out, w->d_log.p + (size_t)lr * w->P.log_cap, sizeof(rlo::LogRec) * cnt, hipMemcpyDeviceToHost));
    if (payload && w->d_log_payload.p && cnt) {
        const uint32_t ls = w->P.log_stride;
        std::vector<uint8_t> tmp((size_t)cnt * ls);
        HIPCHK(hipMemcpy(tmp.data(), w->d_log_payload.p + (size_t)lr * w->P.log_cap * ls, tmp.size(), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < cnt; i++)
            std::memcpy(payload + (size_t)i * payload_stride, tmp.data() + (size_t)i * ls, std::min(ls, payload_stride));
    }
    return (int)cnt;
}

int rlo_latencies(rlo_world_t* w, uint64_t* ticks, uint32_t cap) {
    if (!w || !ticks || !w->d_lat_out.p) return RLO_E_INVAL;
    uint32_t n = std::min(cap, w->lat_rounds);
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipMemcpy(ticks, w->d_lat_out.p, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
    return (int)n;
}

int rlo_timeline(rlo_world_t* w, uint32_t* out, uint64_t cap, uint32_t* stride) {
    if (!w || !out) return RLO_E_INVAL;
    const uint32_t st = rlo::kTlGlobal + rlo::kTlCols * (uint32_t)w->nl;
    if (stride) *stride = st;
    if (!w->tl_rows || !w->d_tl.p) return 0;
    const uint32_t rows = (uint32_t)std::min<uint64_t>(w->tl_rows, cap / st);
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipMemcpy(out, w->d_tl.p, sizeof(uint32_t) * rows * st, hipMemcpyDeviceToHost));
    return (int)rows;
}

int rlo_round_ticks(rlo_world_t* w, uint64_t* ticks, uint32_t cap) {
    if (!w || !ticks || !w->d_lat_obs.p) return RLO_E_INVAL;
    if (w->rb != 0) return RLO_E_INVAL;  // the observer is world rank 0
    uint32_t n = std::min(cap, w->lat_rounds);
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipMemcpy(ticks, w->d_lat_obs.p, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
    return (int)n;
}

}  // extern "C"

// ====================================================================== bulk messages, host side

extern "C" {

int rlo_bulk_plan(int n, uint64_t len, int cross, rlo_bulk_plan_t* out) {
    if (n < 2 || !out || len == 0 || len > 0xFFF00000ull) return RLO_E_INVAL;
    const rlo::BulkPlan p = rlo::bulk_plan(n, (uint32_t)len, cross != 0);
    out->nchunks = p.nchunks;
    out->stripe = p.stripe;
    out->chunk = p.chunk;
    out->tile = p.tile;
    out->total_tiles = rlo::bulk_total_tiles(p, (uint32_t)len);
    out->direct = p.direct;
    return RLO_OK;
}

int rlo_layout_plan(const rlo_plan_cfg_t* cfg, rlo_world_info_t* o) {
    if (!cfg || !o || cfg->n_parts < 1 || cfg->part < 0 || cfg->part >= cfg->n_parts) return RLO_E_INVAL;
    Layout L;
    const uint32_t mp = (std::max<uint32_t>(cfg->max_payload ? cfg->max_payload : 4096u, 16u) + 15u) & ~15u;
    if (mp > 65520u) return RLO_E_INVAL;
    const uint32_t pp = cfg->proposal_pool ? cfg->proposal_pool : 2u;
    if ((pp & (pp - 1u)) || pp > (uint32_t)rlo::kPoolMax) return RLO_E_INVAL;
    L.pend_slots = pp;
    int rc = build_layout(cfg->n_ranks, cfg->n_parts, nullptr, mp, cfg->ring_slots, cfg->bulk_max, cfg->bulk_slots, L);
    if (rc) return rc;
    const int cus = cfg->cus > 0 ? cfg->cus : 256;
    const int nl = L.pb[cfg->part + 1] - L.pb[cfg->part];
    int nmov = 0;
    if (L.bulk_max) nmov = cfg->movers ? (int)cfg->movers : (std::max(16, cus - nl) & ~1);
    LdsPlan p;
    rc = plan_lds(L, nl, nmov, cus, cfg->flags, occ_model, &p);
    if (rc) return rc;
    std::memset(o, 0, sizeof *o);
    o->n_ranks = L.n;
    o->max_in_degree = L.max_in;
    o->max_fanout = L.max_fan;
    o->edges = (int)L.E.size();
    o->ring_slots = L.cap;
    o->slot_stride = L.stride;
    o->vote_slots = L.vote_cap;
    o->fwd_bytes = L.fwd_bytes[cfg->part];
    o->vote_bytes = L.vote_bytes[cfg->part];
    o->ctrl_bytes = L.ctrl_words[cfg->part] * 8;
    o->cus = cus;
    o->blocks_per_cu = p.blocks_per_cu;
    o->part = cfg->part;
    o->n_parts = L.nparts;
    o->rank_begin = L.pb[cfg->part];
    o->rank_end = L.pb[cfg->part + 1];
    o->waves = p.waves;
    o->bulk_slots = L.bslots;
    o->movers = (uint32_t)nmov;
    o->bulk_max = L.bulk_max;
    o->heap_bytes = L.heap_bytes[cfg->part];
    o->proposal_pool = L.pend_slots;
    o->pull = L.pull && p.nsmall >= 2 ? 1u : 0u;
    o->nsmall = p.nsmall;
    o->stage2_bytes = p.stage2;
    o->ll_ok = p.ll_ok ? 1u : 0u;
    o->pend_hbm = p.pend_hbm ? 1u : 0u;
    o->dyn_lds = (uint32_t)p.dyn_lds;
    o->static_lds = (uint32_t)rlo_kernel_static_lds(p.variant);
    return RLO_OK;
}

int rlo_storm_lengths(uint64_t seed, uint64_t k, uint32_t len, uint32_t len_max, uint32_t* out) {
    if (!out && k) return RLO_E_INVAL;
    const uint32_t hi = len_max > len ? len_max : len;
    for (uint64_t b = 0; b < k; b++) out[b] = hi > len ? rlo::storm_len_of(seed, b, len, hi) : len;
    return RLO_OK;
}

int rlo_host_bulk_stage(rlo_world_t* w, int rank, const void* data, uint64_t len, uint32_t timeout_us, uint32_t* q_out) {
    if (!w || !w->h_cmd || !w->L.bulk_max || rank < w->rb || rank >= w->rb + w->nl || !q_out) return RLO_E_INVAL;
    if (len == 0 || len > w->L.bulk_max || (len && !data)) return RLO_E_INVAL;
    const int lr = rank - w->rb;
    const uint32_t B = w->L.bslots, q = w->host_bulk_q[lr], s = q & (B - 1u);
    const uint64_t need = (uint64_t)(q / B) * (uint64_t)(w->L.n - 1);
    // done(rank, s): every receiver released the slot's previous message (read through the BAR)
    const volatile uint64_t* done = reinterpret_cast<const volatile uint64_t*>(
        w->bflag + ((uint64_t)w->nl * w->L.n * B + (uint64_t)lr * B + s) * rlo::kBulkLine);
    const auto t0 = std::chrono::steady_clock::now();
    while (*done < need) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(timeout_us)) return RLO_E_AGAIN;
    }
    HIPCHK(hipSetDevice(w->device));
    uint8_t* dst = w->heap + (((uint64_t)lr * w->L.n + (uint64_t)rank) * B + s) * w->L.bcap;
    HIPCHK(hipMemcpy(dst, data, len, hipMemcpyHostToDevice));
    w->host_bulk_q[lr] = q + 1;
    *q_out = q;
    return RLO_OK;
}

int rlo_host_bulk_copy(rlo_world_t* w, int rank, const rlo_log_rec_t* ev, void* dst) {
    if (!w || !ev || !w->L.bulk_max || rank < w->rb || rank >= w->rb + w->nl || !dst) return RLO_E_INVAL;
    if (ev->kind != RLO_EV_DELIVER_BULK || ev->origin < 0 || ev->origin >= w->L.n || ev->aux >= w->L.bslots ||
        ev->len > w->L.bulk_max)
        return RLO_E_INVAL;
    const int lr = rank - w->rb;
    HIPCHK(hipSetDevice(w->device));
    const uint8_t* src = w->heap + (((uint64_t)lr * w->L.n + (uint64_t)ev->origin) * w->L.bslots + ev->aux) * w->L.bcap;
    HIPCHK(hipMemcpy(dst, src, ev->len, hipMemcpyDeviceToHost));
    return RLO_OK;
}

// ====================================================================== shared host service

int rlo_host_share(rlo_world_t* w, const char* name, uint64_t stage_bytes) {
    // before rlo_program_host: that call builds the segment.  (Replacing pinned rings afterwards
    // would mean a hipHostFree, which waits for the whole device -- i.e. for the persistent kernel
    // of another engine of this process.)
    if (!w || !name || name[0] != '/' || std::strlen(name) > 200 || w->have_program || w->shm) return RLO_E_INVAL;
    if (stage_bytes == 0) stage_bytes = 4ull << 20;
    w->share_stage = (stage_bytes + 4095u) & ~uint64_t(4095);
    w->shm_name = name;
    return RLO_OK;
}

int rlo_host_unlink(rlo_world_t* w) {
    if (!w || !w->shm) return RLO_E_INVAL;
    if (w->shm_linked) shm_unlink(w->shm_name.c_str());
    w->shm_linked = false;
    return RLO_OK;
}

int rlo_host_fail(rlo_world_t* w) {
    if (!w || !w->shm) return RLO_E_INVAL;
    __atomic_store_n(&((rlo::ShmHdr*)w->shm)->leader_failed, 1u, __ATOMIC_RELEASE);
    return RLO_OK;
}

int rlo_host_device_judge(rlo_world_t* w, const rlo_iar_cfg_t* cfg) {
    if (!w || !cfg || !w->have_program || !(w->P.mode & rlo::MODE_HOST)) return RLO_E_INVAL;
    HIPCHK(hipSetDevice(w->device));
    const int rc = set_judge(w, cfg);
    if (rc) return rc;
    w->P.host_judge = 0;
    return RLO_OK;
}

int rlo_host_wait_started(rlo_world_t* w, uint32_t timeout_ms) {
    if (!w || !w->h_ctl) return RLO_E_INVAL;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        int up = 0;
        for (int lr = 0; lr < w->nl; lr++)
            up += __atomic_load_n(&w->h_ctl[(size_t)lr * rlo::kHctlWords + rlo::kHctlState], __ATOMIC_ACQUIRE) != 0;
        if (up == w->nl) return RLO_OK;
        const int r = rlo_host_running(w);
        if (r != 1) return RLO_E_DEVICE;  // the kernel already ended (or the launch failed)
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return RLO_E_TIMEOUT;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

// One pass of the leader's proxy over its clients (rlo_shm.hpp).
int rlo_host_proxy(rlo_world_t* w) {
    if (!w || !w->shm) return RLO_E_INVAL;
    int acted = 0;
    bool bar = false;  // BAR stores this pass: one HDP flush after them
    const uint32_t cc = w->cmd_cap, stride = w->L.stride;
    for (int lr = 0; lr < w->nl; lr++) {
        rlo::ClientBox* box = (rlo::ClientBox*)(w->shm + w->SL.cli) + lr;
        uint64_t* dctl = w->d_ctl + (size_t)lr * rlo::kHctlWords;
        // commands: the client's shared ring -> the VRAM ring the kernel polls locally.  The client
        // admitted each one only with room in its ring (mtail - device head < cmd_cap), which is
        // room in the VRAM ring too (it holds [device head, copied) of the same sequence)
        const uint64_t mt = w->cmd_host ? 0 : __atomic_load_n(&box->mtail, __ATOMIC_ACQUIRE);
        uint64_t c = w->cmd_tail[lr];
        if (!w->cmd_host && mt != c) {
            const uint8_t* src = w->shm + w->SL.cmd + (size_t)lr * cc * stride;
            uint8_t* dst = w->h_cmd + (size_t)lr * cc * stride;
            for (; c != mt; c++) {
                const size_t off = (size_t)(c & (cc - 1)) * stride;
                uint32_t hdr2;
                std::memcpy(&hdr2, src + off + 8, 4);
                const size_t nb = std::min<size_t>(stride, ((rlo::kHdr + (hdr2 & 0xffffffu)) + 15) & ~(size_t)15);
                std::memcpy(dst + off, src + off, nb);
            }
            w->cmd_tail[lr] = mt;
            box->fwd_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now().time_since_epoch()).count();
            box->fwd = mt;
            __atomic_thread_fence(__ATOMIC_SEQ_CST);  // BAR stores may be write-combined: slots before tail
            __atomic_store_n(&dctl[rlo::kHctlInjTail], mt, __ATOMIC_RELEASE);
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            bar = true;
            acted++;
        }
        const uint64_t pk = w->cmd_host ? 0 : __atomic_load_n(&box->mpk, __ATOMIC_ACQUIRE);
        if (!w->cmd_host && pk != w->pk_head[lr]) {  // pickup events the client consumed: room for the kernel
            w->pk_head[lr] = pk;
            __atomic_store_n(&dctl[rlo::kHctlPkHead], pk, __ATOMIC_RELEASE);
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            bar = true;
            acted++;
        }
        if (bar) {  // this rank's command / pickup head: visible to its kernel now, not after the pass
            hdp_flush(w);
            bar = false;
        }
        const uint64_t rq = __atomic_load_n(&box->req, __ATOMIC_ACQUIRE);
        if (rq == w->cli_req[lr]) continue;
        w->cli_req[lr] = rq;  // one bulk request: ACQUIRE a heap slot, or move bytes through stage
        int64_t rc = RLO_OK;
        const int rank = w->rb + lr;
        uint8_t* stage = w->shm + w->SL.stage + (size_t)lr * ((rlo::ShmHdr*)w->shm)->stage_bytes;
        const uint32_t B = w->L.bslots;
        if (!w->L.bulk_max) {
            rc = RLO_E_INVAL;
        } else if (box->op == rlo::SHM_OP_ACQUIRE) {
            const uint32_t q = w->host_bulk_q[lr], s = q & (B - 1u);
            const uint64_t need = (uint64_t)(q / B) * (uint64_t)(w->L.n - 1);
            const volatile uint64_t* done = reinterpret_cast<const volatile uint64_t*>(
                w->bflag + ((uint64_t)w->nl * w->L.n * B + (uint64_t)lr * B + s) * rlo::kBulkLine);
            if (*done >= need) box->q = q;  // taken only by COMMIT, once the bytes are staged
            else rc = RLO_E_AGAIN;          // receivers still hold the slot's previous message
        } else if (box->op == rlo::SHM_OP_COMMIT) {
            if (box->arg == w->host_bulk_q[lr]) w->host_bulk_q[lr]++;
            else rc = RLO_E_INVAL;
        } else if (box->op == rlo::SHM_OP_PUT || box->op == rlo::SHM_OP_GET) {
            const bool put = box->op == rlo::SHM_OP_PUT;
            const uint32_t origin = put ? (uint32_t)rank : box->arg >> 8;
            const uint32_t s = put ? (box->arg & (B - 1u)) : (box->arg & 0xffu);
            const uint64_t off = box->off, len = box->len;
            if (origin >= (uint32_t)w->L.n || s >= B || len > ((rlo::ShmHdr*)w->shm)->stage_bytes || off + len > w->L.bulk_max) {
                rc = RLO_E_INVAL;
            } else {
                uint8_t* slot = w->heap + (((uint64_t)lr * w->L.n + origin) * B + s) * w->L.bcap + off;
                hipError_t e = hipSetDevice(w->device);
                if (e == hipSuccess)
                    e = put ? hipMemcpy(slot, stage, len, hipMemcpyHostToDevice) : hipMemcpy(stage, slot, len, hipMemcpyDeviceToHost);
                if (e != hipSuccess) { g_last_hip = (int)e; rc = RLO_E_HIP; }
            }
        } else {
            rc = RLO_E_INVAL;
        }
        box->rc = rc;
        __atomic_store_n(&box->ack, rq, __ATOMIC_RELEASE);
        acted++;
    }
    return acted;
}

}  // extern "C"
