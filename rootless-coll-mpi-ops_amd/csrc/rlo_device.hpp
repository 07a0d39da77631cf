// rlo_device.hpp -- plain-old-data shared by the host world builder (rlo_world.cpp)
// and the persistent progress kernel (rlo_kernel.hip).
//
// One "world" = N ranks, partitioned into parts (contiguous rank ranges).  A part is
// hosted by one process on one GPU; every rank of a part is one 4-wave (256-thread)
// workgroup of that part's persistent kernel.  Every directed overlay edge
// (r -> send_list(r)[j]) owns
//   * two forward rings (virtual channels vc = 0/1, vc = child < origin; the
//     "dateline" split that makes the ring channel-dependency graph acyclic),
//   * one reverse vote ring (child -> parent).
// A ring's bytes and its producer count (tail) live in the CONSUMER's part; the
// consumer count (head, = credits) lives in the PRODUCER's part.  So every poll is
// local, and every remote access is a store (payload, tail, head) into a peer part's
// HBM -- through a hipIpc mapping when the peer is another process / GPU (xGMI).
#pragma once
#include <stdint.h>

namespace rlo {

// the 4-wave rank-workgroup; the kernel is templated on the wave count (4 or 8: 256 or 512
// messages per iteration, rlo_kernel.hip) and the host picks the width per world (rlo_world.cpp)
constexpr int kBlock = 256;       // threads per rank-workgroup: 4 waves, one 64-message pass each
constexpr int kWaves = kBlock / 64;
constexpr int kMaxFanout = 16;    // send_list_len <= ceil(log2 N) <= 16  (N <= 65536)
constexpr int kMaxIn = 32;        // forward in-edges per rank
constexpr int kMaxOut = 2 * kMaxFanout;
constexpr int kHdr = 16;          // slot header bytes
constexpr int kVoteSlot = 16;     // vote ring slot bytes
constexpr int kMaxCand = 256;     // messages handled per rank per progress iteration (4 passes of 64)
constexpr int kStagePasses = 4;  // 4 x 64 messages per progress iteration
constexpr int kHistBins = 128;    // latency histogram: 4 sub-bins per octave of 10 ns ticks
constexpr int kMaxParts = 64;     // parts (processes x GPUs) of one world
constexpr int kCtrlHdrWords = 16; // per-part control words before the rank blocks: [0] error flag
// latency program of a world split over parts: the round word and the per-round delivery counts are
// one world-wide copy in part 0's control region (peer-mapped like the ring counters), after its rank
// blocks: [round word, own 128-B line][counts: kLatCap x u32]
constexpr int kLatCap = 8192;
constexpr int kLatWords = 16 + kLatCap / 2;

// message classes == enum RLO_COMM_TAGS (rootless_ops.h:50-61)
enum Tag : uint32_t { TAG_BCAST = 0, TAG_PROPOSAL = 2, TAG_VOTE = 3, TAG_DECISION = 4 };

enum Mode : uint32_t {
    MODE_STORM = 1u,   // every rank originates its share of K bcasts (random originators)
    MODE_LAT = 2u,     // one bcast at a time, completion latency per round
    MODE_IAR = 4u,     // every rank runs its proposal list (proposal / vote / decision)
    MODE_LOG = 16u,    // record every event (+ delivered payload bytes) for parity tests
    MODE_HIST = 32u,   // per-delivery latency histogram
    MODE_PROF = 64u,   // per-phase shader-clock accounting (diagnostic build of the same kernel)
    MODE_LAZYPUB = 256u,  // diagnostic: publish counters after the next poll (the pre-eager scheme)
    MODE_NOSPIN = 512u,   // diagnostic: no tight re-poll after an idle iteration
    MODE_NOACQ = 1024u,   // diagnostic (UNSAFE): no agent acquire between iterations (A/B of its cost)
    MODE_HOST = 128u,  // host-service: originations / judge verdicts come from a host command ring,
                       //   deliveries / judge requests / results go to a host pickup ring (rootless_ops.h)
};

// host-service command kinds (tag field of a command slot); tags < 16 are originations
// (TAG_BCAST: RLO_bcast_gen :1581, TAG_PROPOSAL: RLO_submit_proposal :876)
enum HostCmd : uint32_t { CMD_JUDGE = 16, CMD_OWN_JUDGE = 17, CMD_QUIT = 18 };
// per local rank, 64 host words (one 128-B line per counter)
constexpr int kHctlWords = 64;
constexpr int kHctlInjTail = 0, kHctlInjHead = 16, kHctlPkTail = 32, kHctlPkHead = 48;

enum Judge : uint32_t { JUDGE_APPROVE = 0, JUDGE_MASK = 1, JUDGE_ISP = 2, JUDGE_HASH = 3 };

enum LogKind : uint32_t { LOG_DELIVER = 1, LOG_JUDGE = 2, LOG_ACTION = 3, LOG_RESULT = 4, LOG_ERROR = 5,
                          LOG_JREQ = 6,      // host mode: judge(data) request for a received proposal (:698)
                          LOG_OWN_JREQ = 7 };// host mode: the originator's final judge(NULL) request (:773)

enum Err : uint32_t { ERR_NONE = 0, ERR_TIMEOUT = 1, ERR_VOTE_RING = 2, ERR_PID_COLLISION = 3, ERR_VOTE_ORPHAN = 4,
                      ERR_LOG_FULL = 5, ERR_BAD_SLOT = 6, ERR_HOST_CMD = 7 };

// Slot header, 16 bytes:
//   w0 = origin (16 b) | tag (8 b) << 16 | vote (8 b) << 24
//   w1 = id   (bcast id / proposal pid)
//   w2 = len (16 b, payload bytes) | mark 0xA5 (8 b) << 16 | pseq (8 b) << 24 (pseq: per-origin
//        proposal sequence; the mark, set at origination, tells a written slot from zeroed ring memory)
//   w3 = t0   (low 32 bits of s_memrealtime at origination, 100 MHz)
// Vote slot, 16 bytes: w0 = origin | vote << 24, w1 = pid, w2 = pseq, w3 = voter

struct RankTopo {
    int32_t level, last_wall, scc, sll;   // rootless_ops.c:86-112 fields, restated
    int32_t send_list[kMaxFanout];
    int32_t n_in;                          // forward in-edges
    int32_t in_src[kMaxIn];                // sender rank of in-edge k
    // rings I consume (local part): byte offsets in my part's forward / vote regions
    uint32_t in_data[kMaxIn][2];           // forward in-ring (k, vc)
    uint32_t vin_data[kMaxFanout];         // vote ring from child j
    uint32_t inbox_ctrl, n_inbox;          // my tails in my part's ctrl: fwd in 2*n_in, then votes-in sll
    uint32_t outbox_ctrl, n_outbox;        // my heads in my part's ctrl: fwd out 2*sll, then votes-out n_in
    // remote ends, as addresses valid in the hosting process (peer HBM via hipIpc / P2P)
    uint64_t out_ring[kMaxFanout][2];      // forward ring (j, vc) data, in the child's part
    uint64_t out_tail[kMaxFanout][2];      // its tail word, in the child's ctrl
    uint64_t in_head[kMaxIn][2];           // head word of in-ring (k, vc), in the parent's ctrl
    uint64_t vout_ring[kMaxIn];            // vote ring to the parent of in-edge k, in the parent's part
    uint64_t vout_tail[kMaxIn];            // its tail word, in the parent's ctrl
    uint64_t vin_head[kMaxFanout];         // head word of the vote ring from child j, in the child's ctrl
};

struct RankStats {
    uint64_t bcast_delivered, bcast_sum, originated;
    uint64_t dec_delivered, dec_approved, actions, judge_calls;
    uint64_t own_decided, own_approved, proposals_recv;
    uint64_t iterations, busy_iterations, stalls, log_count;
    uint64_t t_start, t_end;              // s_memrealtime
    uint32_t error, error_aux;
    uint64_t prof[8];                     // MODE_PROF: s_memtime cycles per phase A..H
    uint64_t dbg[8];                      // MODE_PROF: ring cands, admitted, storm-allowed iters, storm offered,
                                          //   shallow-blocked, backlog-blocked, child copies, max out-ring fill
    uint32_t hist[kHistBins];
    uint64_t unmarked_slots;               // staged ring slots whose header lacked the slot mark (an error)
};

struct LogRec {            // 32 bytes
    uint32_t kind;         // LogKind | tag << 8
    int32_t origin;
    int32_t from;          // parent rank (deliveries) / -1
    uint32_t id;           // bid / pid
    uint32_t len;
    int32_t vote;          // decision / judge return / -1
    uint32_t aux;          // judge: arg==NULL ; action: data_len
    uint32_t payload_idx;  // index into log payload area, 0xffffffff if none
};

struct Params {
    int32_t n, rank_begin, rank_end;
    uint32_t mode;
    const RankTopo* topo;         // [rank_end - rank_begin]
    uint8_t* fwd_region;          // this part's forward in-rings (<= 4 GiB, one buffer rsrc)
    uint32_t fwd_region_bytes;
    uint32_t fwd_cap, fwd_stride; // slots per forward ring (pow2), slot stride bytes
    uint8_t* vote_region;         // this part's vote in-rings
    uint32_t vote_region_bytes;
    uint32_t vote_cap;            // slots per vote ring (pow2), >= 2 * N
    uint64_t* ctrl;               // this part's control words (tails / heads of its ranks)
    uint32_t sys_scope;           // 1: some peer part is on another GPU -> system-scope remote stores
    uint32_t n_parts;
    uint32_t* err_flag[kMaxParts];// every part's error word (ctrl word 0 of each part)
    // storm / latency workload
    uint64_t seed;
    uint32_t len, window;         // payload bytes; max originations per iteration
    const int64_t* sched_off;     // [n_local + 1] CSR of bcast ids originated by each local rank
    const uint32_t* sched_ids;
    const int64_t* expect_bcast;  // [n_local]
    uint32_t lat_rounds;
    const int32_t* lat_origin;    // [lat_rounds]
    uint32_t* lat_count;          // [lat_rounds] deliveries so far
    uint64_t* lat_out;            // [lat_rounds] completion ticks
    uint32_t* lat_round;          // current round (global; part 0's control region when sharded)
    uint64_t* lat_obs;            // [lat_rounds] observer clock (world rank 0) when round i completed
    const uint32_t* lat_own_off;  // [n_local + 1] CSR of the rounds each local rank originates
    const uint32_t* lat_own;
    // IAR workload
    uint32_t judge_kind, judge_ppm;
    uint64_t judge_seed;
    const uint8_t* judge_mask;    // [n]
    const char* judge_isp;        // concatenated NUL-terminated strings
    const uint32_t* judge_isp_off;// [n]
    const int64_t* prop_off;      // [n_local + 1] CSR of own proposals per local rank
    const int32_t* prop_pid;
    const uint32_t* prop_data_off;
    const uint32_t* prop_data_len;
    const uint8_t* prop_data;
    const int64_t* expect_dec;    // [n_local] decisions each rank picks up
    // outputs
    RankStats* stats;             // [n_local]
    LogRec* log;                  // [n_local * log_cap]
    uint8_t* log_payload;         // [n_local * log_cap * log_stride] or null
    uint32_t log_cap, log_stride;
    // control
    uint64_t timeout_ticks;       // no progress for this long -> ERR_TIMEOUT (100 MHz ticks)
    uint64_t deadline_ticks;      // hard cap on one launch (every spin is bounded)
    uint32_t* error_flag;         // this part's error word (polled every iteration)
    // dynamic LDS carve-out: [pend: 2N x 16 B][olist: nout_max x 256 x 2 B]
    //                        [stage: 256 x nsmall x 16 B][stage2: stage2_bytes]
    uint32_t nsmall;              // slot chunks staged per message on the small path (<= 8)
    uint32_t stage2_bytes;        // LDS staging for large messages (multiple of 1 KiB, >= 1 KiB)
    uint32_t nout_max;            // 2 x max send_list_len over the ranks of this launch
    // host-service mode (MODE_HOST): all in pinned host memory.  Pickup records / payloads use
    // log / log_payload above as per-rank rings of log_cap slots.
    uint8_t* hin;                 // command slots [n_local][hin_cap] x fwd_stride (forward-slot layout),
                                  //   uncached VRAM written by the CPU through the BAR
    uint32_t hin_cap;
    uint64_t* hctl;               // [n_local][kHctlWords] counters the DEVICE writes (pinned host memory)
    uint64_t* hctl_dev;           // [n_local][kHctlWords] counters the HOST writes (uncached VRAM:
                                  //   the CPU stores through the BAR, the kernel polls locally)
};

// ---- bulk (large-message) rootless bcast: pipelined scatter + all-gather (rlo_bulk.hip)
constexpr int kMaxBulkRanks = 64;
constexpr uint32_t kBulkBlock = 1024;     // bytes one wave moves per step (64 lanes x 16 B)
constexpr uint32_t kBulkMaxChunks = 4096; // flags per rank and kind

struct BulkParams {
    int32_t n, rank_begin, origin, pad;
    uint64_t bytes;                      // message size
    uint32_t chunk, stripe, nchunks;     // chunk = stripe * (n - 1); stripe multiple of kBulkBlock
    uint32_t buf_bytes;                  // capacity of every rank's buffer (<= 4 GiB, multiple of 1 KiB)
    uint8_t* buf[kMaxBulkRanks];         // every rank's receive buffer (peer HBM mapped)
    uint32_t* sflag[kMaxBulkRanks];      // every rank's scatter flags [kBulkMaxChunks]
    uint32_t* gflag[kMaxBulkRanks];      // every rank's gather flags [kBulkMaxChunks]
    uint64_t deadline_ticks;
    uint32_t* err;                       // this part's error word
};

}  // namespace rlo
