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
constexpr int kPoolMax = 16;      // own proposals in flight per rank (PROPOSAL_POOL_SIZE, rootless_ops.c:30)
constexpr int kCtrlHdrWords = 16; // per-part control words before the rank blocks: [0] error flag
// [15] the part's creation nonce (rlo_part_connect checks it through every peer's mapping; rlo_reset keeps it)
constexpr int kCtrlNonceWord = 15;
// MODE_TL timeline of a latency round: global events (the part where each happens writes it), then per local
// rank the arrival of the round's message (or bulk announcement) and the completion of its bulk copy
constexpr uint32_t kTlRoundsMax = 64, kTlGlobal = 8, kTlCols = 9;
// per-rank columns: arrival, bulk completion (ring-slot messages: forwards issued), tree parent + 1, and for a
// message the doorbell pass took: when the spin's polls that found it were issued, when the pass began
enum TlCol : uint32_t { TLC_ARRIVE = 0, TLC_DONE = 1, TLC_PARENT = 2, TLC_ISSUE = 3, TLC_PASS = 4,
                        TLC_FWD = 5,    // bulk announcement: its forwards issued
                        TLC_NEXT = 6,   // bulk announcement: the next spin of wave 0 began
                        TLC_P1 = 7, TLC_P2 = 8 };  // ring-slot message taken by the doorbell pass: probes in lone()
enum TlEvent : uint32_t { TL_ORIGIN = 0, TL_POSTED = 1, TL_CLAIMED = 2, TL_MOVED = 3, TL_ROUND = 4, TL_VERIFIED = 5,
                          TL_GEN = 6, TL_DRAINED = 7 };  // (the first sub-job's mover: origin copy written, copy drained)
// latency program of a world split over parts: the round word and the per-round delivery counts are
// one world-wide copy in part 0's control region (peer-mapped like the ring counters), after its rank
// blocks: [round word, own 128-B line][counts: kLatCap x u32]
constexpr int kLatCap = 8192;
constexpr int kLatWords = 16 + kLatCap / 2;

// message classes == enum RLO_COMM_TAGS (rootless_ops.h:50-61); TAG_BULK (beyond RLO_ANY_TAG) is
// the announcement of a bulk message (longer than a ring slot): payload = BulkDesc, the bytes move
// through the mover workgroups (below), the user sees an RLO_BCAST
enum Tag : uint32_t { TAG_BCAST = 0, TAG_PROPOSAL = 2, TAG_VOTE = 3, TAG_DECISION = 4, TAG_BULK = 10 };

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
    MODE_NOFAST = 2048u,  // A/B: every iteration takes the full path (no lone-message fast path)
    MODE_HDIAG = 4096u,   // diagnostic, host mode: command-wait counters into hctl[kHctlDiag..] at exit
    MODE_PIPE = 8192u,    // A/B: large-message staging rounds pipelined over two halves of stage2
    MODE_LL = 16384u,     // doorbells (below): lone messages and originations hop without a counter round trip
    MODE_TL = 32768u,     // latency program: per-round event clocks into Params.tl (RLO_FLAG_TIMELINE; no path changes)
    MODE_HOPPROF = 131072u,  // diagnostics build: shader clocks at points of a doorbell hop into stats.prof (tools/hop_prof.py)
    MODE_NOHPW = 262144u,   // diagnostics build, host mode A/B: no wave-1 host poller (wave 0 polls the host words itself)
    MODE_XCD1 = 524288u,    // RLO_PART_ONE_XCD: the hop kernel's rank-waves on one XCD, L2-kept (plain) hand-off stores
    MODE_CORRUPT = 65536u,  // diagnostics build, test of the VERIFY check: a direct scatter zeroes one granule of one copy
    MODE_HOST = 128u,  // host-service: originations / judge verdicts come from a host command ring,
                       //   deliveries / judge requests / results go to a host pickup ring (rootless_ops.h)
};

// host-service command kinds (tag field of a command slot); tags < 16 are originations
// (TAG_BCAST: RLO_bcast_gen :1581, TAG_PROPOSAL: RLO_submit_proposal :876, TAG_BULK: a bulk
// bcast whose bytes the host put in the origin's own heap slot)
enum HostCmd : uint32_t { CMD_JUDGE = 16, CMD_OWN_JUDGE = 17, CMD_QUIT = 18, CMD_BULK_RELEASE = 19 };
// per local rank, 64 host words (one 128-B line per counter)
constexpr int kHctlWords = 64;
constexpr int kHctlInjTail = 0, kHctlInjHead = 16, kHctlPkTail = 32, kHctlPkHead = 48;
constexpr int kHctlState = 40;  // device-written: 1 once the rank's workgroup serves, 2 once it exited
constexpr int kHctlDiag = 20;  // MODE_HDIAG, 8 words: iterations with commands pending, proposals held (own one
                               // active), pickup-ring blocks, host iterations, seen -> drained < 20 / 100 / 500 / >= 500 us
constexpr int kHctlBeat = 41;   // device-written heartbeat: [41] iterations, [42] command tail seen, [43] pickup head seen

enum Judge : uint32_t { JUDGE_APPROVE = 0, JUDGE_MASK = 1, JUDGE_ISP = 2, JUDGE_HASH = 3 };

enum LogKind : uint32_t { LOG_DELIVER = 1, LOG_JUDGE = 2, LOG_ACTION = 3, LOG_RESULT = 4, LOG_ERROR = 5,
                          LOG_JREQ = 6,      // host mode: judge(data) request for a received proposal (:698)
                          LOG_OWN_JREQ = 7,  // host mode: the originator's final judge(NULL) request (:773)
                          LOG_JUDGED = 8 };  // host mode, device judge: a proposal judged here (vote, PBuf)

enum Err : uint32_t { ERR_NONE = 0, ERR_TIMEOUT = 1, ERR_VOTE_RING = 2, ERR_PID_COLLISION = 3, ERR_VOTE_ORPHAN = 4,
                      ERR_LOG_FULL = 5, ERR_BAD_SLOT = 6, ERR_HOST_CMD = 7,
                      ERR_BULK = 8, ERR_XCD = 9 };  // a bulk index / job field out of range (error_aux: site << 24 | value)

// Slot header, 16 bytes:
//   w0 = origin (16 b) | tag (8 b) << 16 | vote (8 b) << 24
//   w1 = id   (bcast id / proposal pid)
//   w2 = len (16 b, payload bytes) | mark 0xA5 (8 b) << 16 | pseq (8 b) << 24 (pseq: the origin's
//        proposal-pool slot of a proposal / its decision, which names the receivers' pending entry
//        (origin, pseq); the mark, set at origination, tells a written slot from zeroed ring memory)
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
    uint64_t in_base[kMaxIn];              // forward region of in-edge k's producer part (pulled payloads)
    uint32_t orig_data, orig_pad;          // pull worlds: my relay ring (byte offset in my part)
    // doorbells (MODE_LL, below): word indices of my forward bells (in-edge k at + kBellWords k) and my
    // vote bells (child j at + 2 j) in my part's ctrl region; the remote bells I ring, as addresses
    uint32_t in_bell, vin_bell;
    uint64_t out_bell[kMaxFanout];         // child j's forward bell for the edge (me -> child j)
    uint64_t vout_bell[kMaxIn];            // the parent of in-edge k: its vote bell for me
};

// Doorbells (MODE_LL: the latency / IAR / host programs of worlds without bulk messages).  A message a
// rank forwards on its own -- a lone ring message, a local origination -- is also written, data-tagged,
// into the child's DOORBELL for the edge: one per directed edge (both virtual channels), kBellChunks
// 16-B chunks (header + 112 B) as 32-B pairs of LL granules {d0, T, d1, T}, {d2, T, d3, T} where
// T = bell_tag(ring sequence) | vc << 31.  Every 8-byte half carries T, so a reader that finds T in all of
// them holds the message, whatever order the halves landed in (MI355X_MICROARCH.md handoff-1to1: the
// data is the flag).  The consumer polls the bell beside its ring counters: a bell tagged with the
// sequence at its ring head IS the head message -- no counter poll, no slot load, no producer drain on
// the hop.  The ring slot and the counter are still written (a bell is overwritten by the next message
// on the edge; whatever the consumer does not take from a bell it takes through the counter), so the
// batched path is unchanged.  A vote bell (child -> parent) is one granule pair {origin | pseq << 16 |
// vote << 24, T, pid, T}, T = bell_tag(vote sequence).  Bells live in the ctrl region: uncached, mapped
// across parts, zeroed at every launch (a tag of a previous launch can never match).
constexpr uint32_t kBellChunks = 8;
// the data tag of the s-th message (0-based) of a forward edge, a vote ring or a command ring: never 0 (a
// zeroed bell matches nothing) and 30 bits wide, so a forward bell's bit 31 carries only the virtual channel
// -- after 2^31 messages on one edge a vc-0 tag could otherwise read as vc 1.  Tags of one bell
// repeat every 2^30 messages, far beyond the <= 4,096 a ring holds in flight
__host__ __device__ inline uint32_t bell_tag(uint64_t s) { return ((uint32_t)s & 0x3fffffffu) + 1u; }
constexpr uint32_t kBellWords = 2 * kBellChunks * 2;  // 8-byte words per forward bell (256 B)

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

// Host mode's pickup ring carries self-validating records (the LL idea): the record's four 8-byte units -- each
// lands whole -- and the units of a payload the doorbell pass writes carry a tag derived from the event's sequence and
// the launch epoch, so the host takes an event as soon as its units have landed instead of after the kernel drained
// its stores and then published the pickup tail (two PCIe crossings later).  The record keeps LogRec's 32 bytes with
// a 16-bit tag in the spare upper half of one word of each unit: kind (16 bits used), from + 1 (a rank or -1),
// vote (-1 / 0 / 1), and the payload slot (< kPkMaxSlots; kPkNoPayload = none, | kPkTaggedPayload = the tagged
// form: payload byte 4k + j in the low half of 8-byte unit k, pk_tag in the high half).  A plain payload (the full
// path's, large messages) is read once the published tail covers the event.
constexpr uint32_t kPkRecBytes = 32, kPkMaxSlots = 16384, kPkNoPayload = 0xffffu, kPkTaggedPayload = 0x8000u;
__host__ __device__ inline uint32_t pk_tag(uint64_t seq, uint32_t epoch) { return (((uint32_t)seq << 1) | 1u) ^ epoch; }
__host__ __device__ inline uint32_t pk_tag16(uint64_t seq, uint32_t epoch) { return pk_tag(seq, epoch) & 0xffffu; }
// the pickup payload stride: room for a doorbell-pass payload (<= 7 chunks, 112 B) in the tagged form (224 B)
__host__ __device__ inline uint32_t pk_payload_stride(uint32_t max_payload) { return max_payload >= 256u ? max_payload : 256u; }

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
    uint64_t* ctrl;               // this part's control words (tails / heads of its ranks, doorbells)
    uint32_t ctrl_bytes;
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
    uint32_t* xcd_word;           // MODE_XCD1: the first rank-wave's XCC id + 1 (uncached; zeroed at every launch)
    uint64_t* lat_obs;            // [lat_rounds] observer clock (world rank 0) when round i completed
    uint32_t* tl;                 // MODE_TL: [tl_rounds][kTlGlobal + kTlCols n_local] low 32 bits of the 100-MHz clock
    uint32_t tl_rounds;
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
    // proposal pool: pend_slots entries per origin in every rank's pending table (a power of two
    // <= kPoolMax, fixed at world creation: the table is dynamic LDS [N x pend_slots] x 16 B); an
    // originator keeps up to own_pool <= pend_slots own proposals in flight, in slots it takes
    // round-robin, and reuses a slot only after that slot's decision went out
    uint32_t pend_slots, own_pool;
    struct PendState* pend_hbm;   // non-null: the pending tables in HBM, [n_local][n][pend_slots] x 16 B (uncached)
    // pulled payloads (slots beyond the small copy path, no bulk): a large bcast travels each edge as
    // its header (mark kRefMark) + a reference chunk {byte offset of the sender's copy in the sender's
    // part}.  The sender's copy sits in its RELAY ring (one per rank, fwd_cap slots): an originator or
    // a forwarding rank writes the message there once, its children load the payload from there (and
    // write it into their own relay ring if they forward it on), and a relay slot is reused only after
    // every child consumed the references written up to it (a release queue on the out-ring heads).
    // A wall rank then stores header + reference per child instead of the whole payload per child.
    uint32_t pull, relay_cap;     // relay slots per rank (power of two)
    // outputs
    RankStats* stats;             // [n_local]
    LogRec* log;                  // [n_local * log_cap]
    uint8_t* log_payload;         // [n_local * log_cap * log_stride] or null
    uint32_t log_cap, log_stride;
    // control
    uint64_t timeout_ticks;       // no progress for this long -> ERR_TIMEOUT (100 MHz ticks)
    uint64_t deadline_ticks;      // hard cap on one launch (every spin is bounded)
    uint32_t* error_flag;         // this part's error word (polled every iteration)
    // dynamic LDS carve-out: [pend: N x pend_slots x 16 B][olist: nout_max x 256 x 2 B]
    //                        [stage: 256 x nsmall x 16 B][stage2: stage2_bytes]
    uint32_t nsmall;              // slot chunks staged per message on the small path (<= 24)
    uint32_t stage2_bytes;        // LDS staging for large messages (multiple of 1 KiB, 1 KiB .. 128 KiB)
    uint32_t nout_max;            // 2 x max send_list_len over the ranks of this launch
    // host-service mode (MODE_HOST): all in pinned host memory.  Pickup records / payloads use
    // log / log_payload above as per-rank rings of log_cap slots.
    uint8_t* hin;                 // command slots [n_local][hin_cap] x fwd_stride (forward-slot layout),
                                  //   uncached VRAM written by the CPU through the BAR
    uint32_t hin_cap;
    uint32_t pk_epoch;            // host mode: this launch's pickup-tag epoch (even; pk_tag), in hin_cap's padding
    uint64_t* hctl;               // [n_local][kHctlWords] counters the DEVICE writes (pinned host memory)
    uint64_t* hctl_dev;           // [n_local][kHctlWords] counters the HOST writes (uncached VRAM:
                                  //   the CPU stores through the BAR, the kernel polls locally)
    uint8_t* hll;                 // [n_local][hin_cap] x (kBellChunks x 32 B) command doorbells (rlo_shm.hpp
                                  //   ll_cmd_put), host memory; null: none (commands in VRAM)
    // bulk messages (the BULK kernel instantiation only; rlo_device.hpp "bulk messages" below)
    uint32_t bulk_slots, bulk_cap;  // B (power of two) heap slots per origin, bytes per slot (x 64 KiB)
    uint32_t n_local, nmov;         // progress workgroups, mover workgroups (blocks [n_local, n_local + nmov))
    uint32_t bulk_cross;            // parts span GPUs: chunked (pipelined) plan
    uint32_t len_lo, len_hi;        // storm payload lengths: len_hi > len_lo -> storm_len_of per bcast
    uint32_t ring_cap;              // payload bytes a ring slot carries (longer -> bulk)
    const uint64_t* bheap;          // [n_parts] heap base of every part, mapped in this process
    const uint64_t* bflag;          // [n_parts] flag-region base of every part, mapped in this process
    const int32_t* part_of;         // [n] part of every rank
    const int32_t* part_begin;      // [n_parts + 1]
    struct BulkJob* jobs;           // [2][jslots] this part's job rings (class A, class B)
    uint32_t jslots, bpend_off;     // job ring slots per class (power of two, >= every job that can be
                                    //   unfinished at once); dynamic-LDS byte offset of the pending table
    uint64_t* jctl;                 // [kJctlWords] posted / head counters, exited progress workgroups
    uint64_t* jclaim;               // (unused)
    uint64_t* jfree;                // [2][jslots] generation: slot j % J takes sub-job j once jfree == j / J
    uint32_t* jdone;                // [2][jslots] finished tiles of the slot's job
    uint64_t* jsum;                 // [2][jslots] VERIFY checksum accumulator
    uint32_t storm_order;           // RLO_ORDER_SLOTS: bcast b originates at b mod N
    uint32_t host_judge;            // host mode: 1 = judges are the host's callbacks, 0 = the device registry
    uint32_t hop_chunks;            // the hop kernel (rlo_hop.hip): 16-B chunks of the program's longest message
};

// ---- bulk messages (longer than a ring slot; SURVEY §8(f)1, BASELINE configs[2], [4]).
// Rootless: the origin's progress workgroup originates a TAG_BULK announcement that travels the
// skip-ring tree like any bcast; the bytes move as a pipelined scatter + all-gather between the
// ranks' heaps, done by MOVER workgroups of the same persistent launch:
//   * heap slot (r, o, s) of rank r holds r's copy of origin o's bulk message with bulk sequence q,
//     s = q mod B; every rank computes every address, so nobody allocates or asks;
//   * the message is cut into chunks, a chunk into N-1 stripes (whole KiB), stripe k owned by
//     rank (o + 1 + k) mod N; SCATTER tiles (origin's movers) store stripe k into its owner's slot
//     and bump the owner's sflag[chunk] and tflag; GATHER tiles (each receiver's movers, posted when
//     the announcement arrives) wait for their own stripe of a chunk, then store it into the other
//     N-2 receivers' slots and bump their tflag;
//   * a receiver's copy is complete when tflag == the message's tile count plus its own gather tiles
//     (it may not be released before its pushes out of it are done; its progress workgroup polls);
//     it is then delivered (device programs: a VERIFY job checksums it; host mode: a pickup
//     event, the host copies it out), the slot's flags are cleared and done(o, s) at the origin is
//     bumped; the origin reuses slot s for sequence q + B only when done(o, s) counts every receiver.
// Mover classes: class A (SCATTER, VERIFY) never waits; class B (GATHER) waits only for class-A
// scatters, so no cycle of waits exists however announcements interleave.
// DIRECT plans (every part on one GPU: no links to balance, the copy is HBM bound): one stripe, the
// whole message; a SCATTER tile is stored straight into EVERY receiver's slot (a fan-out from the
// origin's copy: read once, written N-1 times) and bumps every receiver's tflag; no GATHER jobs; all
// movers are class A (nothing waits).  Per byte: the origin's copy read once and N-1 copies written,
// against a stripe read + a scatter write + N-1 gather writes, and no scatter -> gather hand-off.
constexpr uint32_t kBulkKiB = 1024;     // stripe granularity
constexpr int kBulkMaxChunks = 16;
constexpr uint32_t kBulkLine = 128;     // per (rank, origin, slot): sflag[16] u32 @0, tflag u32 @64
constexpr uint32_t kBulkTflag = 16;     // word index of tflag in the line
constexpr uint64_t kJobTileMask = (1ull << 40) - 1;  // post counter: jobs << 40 | tiles
constexpr int kMaxPend = 1024;          // pending bulk receptions per rank (N * B <= 1024: C5 at 8 GPUs, 512 ranks)
enum JobKind : uint32_t { JOB_SCATTER = 1, JOB_GATHER = 2, JOB_VERIFY = 3 };
enum JobClass : uint32_t { JCLS_A = 0, JCLS_B = 1 };

struct BulkJob {         // 64 B, one slot of a part's job ring: one SUB-job (consecutive tiles of a job)
    uint32_t seq;        // j + 1 once the slot holds sub-job j (written last)
    uint32_t kind;       // JobKind
    int32_t origin, lr;  // message origin, posting (local) rank
    uint32_t slot, bid;  // heap slot s, bcast id
    uint32_t len, ntiles;  // message bytes; tiles of this sub-job
    uint32_t ti0, parent;  // its first tile in the job; the job's first sub-job slot (VERIFY accounting)
    int32_t from;        // VERIFY: tree parent of the announcement (log)
    uint32_t logidx;     // VERIFY: log record to complete with the checksum, ~0u = none
    uint32_t q, gen;     // bulk sequence; SCATTER source: 1 = heap slot (o, o, s) (host), 0 = generated
    uint32_t total;      // tiles of the whole job
    uint32_t pjob;       // VERIFY: the parent sub-job's index, low 32 bits (its slot's generation)
};
static_assert(sizeof(BulkJob) == 64, "job slot");

// part-local job-ring control words (each on its own 128-B line): [cls*16 + 0] jobs posted,
// [cls*16 + 8] head (first job not fully claimed), [32] exited progress workgroups; then diagnostics
// (rlo_bulk_debug): tiles finished per class, gather tiles that waited / passed their wait, the sink
// line an out-of-range flag index is redirected to (posts by job kind follow it), slot releases,
// bulk originations that waited for a slot, the last gather wait, and the first fault record (the
// bulk guards' site-specific detail, written once)
constexpr int kJctlPost = 0, kJctlClaim = 8, kJctlExited = 32;
constexpr int kJctlTilesDone = 36, kJctlGatherWaited = 38, kJctlGatherPassed = 39, kJctlSink = 40,
              kJctlPostsByKind = 40, kJctlReleases = 44, kJctlSlotWaits = 45, kJctlLastGather = 46,
              kJctlFault = 47, kJctlWords = 48;

// stripe / chunk / tile plan of a bulk message: a pure function of (N, len, cross-GPU), so every
// rank derives the same one.  One GPU: the direct plan (one stripe = the message, fanned out).  Across
// GPUs (and RLO_PART_CHUNKED): chunks pipeline the scatter into the all-gather, the gather of chunk c
// running while chunk c + 1 is scattered, ~sqrt(len / 4 MiB) chunks.  A tile (what
// one mover claim moves, then one release + flag add) is the stripe cut to <= 64 KiB, or to <= 16 KiB
// for messages under 8 MiB: a mover workgroup stores ~20 GB/s into uncached HBM, so a message is fast
// only when many movers share it -- short ones are latency bound and want many small tiles, long ones
// large tiles so the per-tile release stays a small share.
constexpr uint32_t kBulkTileMax = 64u << 10, kBulkTileSmall = 16u << 10;
constexpr uint32_t kBulkChunk1 = 4u << 20;  // chunked plan: ~sqrt(len / kBulkChunk1) chunks; 64-KiB tiles from 2x this
// a VERIFY job (a receiver's read of its whole copy) is cut into 64-KiB tiles, independent of the
// stripe plan: many movers read a copy at once (at N = 64 a stripe-sized tile made ~63 tiles per copy)
constexpr uint32_t kVerifyTile = 64u << 10;
// a job is posted as at most kMaxSub sub-jobs of consecutive tiles; a mover draws sub-jobs by ticket
// (one fetch-add, never retried) and moves all of a sub-job's tiles itself.  Enough sub-jobs that every
// mover of a class has one while a single message's scatter or verify runs
constexpr uint32_t kMaxSub = 256;
// ... except a SCATTER job: one tile per sub-job up to 1024 (a direct 64-MiB message's 1024 tiles): with
// 4-tile sub-jobs, 256 of them over 248 movers left 8 movers a second sub-job each -- the round took two
// sub-job times; with single tiles the tail is one tile
constexpr uint32_t kMaxSubScatter = 1024;
// ... and a VERIFY job (reads only) in at most 64: its sub-jobs are cheap to move, so their claim overhead
// (ticket, record, accounting) is what a finer cut would add
constexpr uint32_t kMaxSubVerify = 64;
__host__ __device__ inline uint32_t max_sub(uint32_t kind) {
    return kind == 1u /* JOB_SCATTER */ ? kMaxSubScatter : (kind == 3u /* JOB_VERIFY */ ? kMaxSubVerify : kMaxSub);
}
// granules in flight per mover thread (16 B each): 256 threads x 8 x 16 B = 32 KiB per round trip
constexpr int kMoveDepth = 8;
struct BulkPlan {
    uint32_t nchunks, stripe, chunk, tile;  // chunk = stripe * (N - 1); stripe, tile multiples of 1 KiB
    uint32_t direct;                        // one GPU: one stripe = chunk = the message, fanned out
};
__host__ __device__ inline BulkPlan bulk_plan(int n, uint32_t len, bool cross) {
    if (!cross) {
        BulkPlan p;
        p.direct = 1;
        p.stripe = p.chunk = len ? (len + kBulkKiB - 1) / kBulkKiB * kBulkKiB : kBulkKiB;
        p.nchunks = len ? 1u : 0u;
        // (4-KiB tiles for a 1-MiB message -- 256 sub-jobs instead of 64 -- measured slower: 40 -> 44 us)
        const uint32_t tmax = len >= 2 * kBulkChunk1 ? kBulkTileMax : kBulkTileSmall;
        const uint32_t parts = (p.stripe + tmax - 1) / tmax;
        p.tile = (p.stripe / parts + kBulkKiB - 1) / kBulkKiB * kBulkKiB;
        (void)n;
        return p;
    }
    uint32_t k = 1;
    while ((uint64_t)(k + 1) * (k + 1) * kBulkChunk1 <= len && k < (uint32_t)kBulkMaxChunks) k++;
    const uint32_t m = (uint32_t)(n - 1);
    const uint64_t per = ((uint64_t)len + k - 1) / k;
    uint64_t stripe = ((per + m - 1) / m + kBulkKiB - 1) / kBulkKiB * kBulkKiB;
    if (stripe < kBulkKiB) stripe = kBulkKiB;
    uint64_t chunk = stripe * m;
    while ((len + chunk - 1) / chunk > (uint64_t)kBulkMaxChunks) { stripe *= 2; chunk = stripe * m; }
    BulkPlan p;
    p.direct = 0;
    p.stripe = (uint32_t)stripe;
    p.chunk = (uint32_t)chunk;
    p.nchunks = len ? (uint32_t)((len + chunk - 1) / chunk) : 0u;
    const uint32_t tmax = len >= 2 * kBulkChunk1 ? kBulkTileMax : kBulkTileSmall;
    const uint32_t parts = (p.stripe + tmax - 1) / tmax;
    p.tile = (p.stripe / parts + kBulkKiB - 1) / kBulkKiB * kBulkKiB;
    return p;
}
// bytes of stripe k in chunk c
__host__ __device__ inline uint32_t bulk_stripe_len(const BulkPlan& p, uint32_t len, uint32_t c, uint32_t k) {
    const uint64_t c0 = (uint64_t)c * p.chunk;
    const uint64_t clen = len - c0 < p.chunk ? len - c0 : p.chunk;
    const uint64_t s0 = (uint64_t)k * p.stripe;
    if (s0 >= clen) return 0u;
    return (uint32_t)(clen - s0 < p.stripe ? clen - s0 : p.stripe);
}
__host__ __device__ inline uint32_t bulk_tiles_of(const BulkPlan& p, uint32_t bytes) {
    return (bytes + p.tile - 1) / p.tile;
}
// tiles of chunk c over all its stripes
__host__ __device__ inline uint32_t bulk_chunk_tiles(const BulkPlan& p, uint32_t len, uint32_t c) {
    const uint64_t c0 = (uint64_t)c * p.chunk;
    const uint32_t clen = (uint32_t)(len - c0 < p.chunk ? len - c0 : p.chunk);
    const uint32_t full = clen / p.stripe, rem = clen % p.stripe;
    return full * bulk_tiles_of(p, p.stripe) + bulk_tiles_of(p, rem);
}
// tiles of every stripe of every chunk = what reaches each receiver = its completion count
__host__ __device__ inline uint32_t bulk_total_tiles(const BulkPlan& p, uint32_t len) {
    uint32_t t = 0;
    for (uint32_t c = 0; c < p.nchunks; c++) t += bulk_chunk_tiles(p, len, c);
    return t;
}
// tiles of stripe k over all chunks (one receiver's GATHER job; none in a direct plan)
__host__ __device__ inline uint32_t bulk_stripe_tiles(const BulkPlan& p, uint32_t len, uint32_t k) {
    if (p.direct) return 0u;
    uint32_t t = 0;
    for (uint32_t c = 0; c < p.nchunks; c++) t += bulk_tiles_of(p, bulk_stripe_len(p, len, c, k));
    return t;
}

// storm workload with mixed payload sizes (BASELINE configs[4]): piecewise log-uniform length of
// bcast b in [lo, hi]: an octave e uniform over [log2 lo, log2 hi), then uniform inside the octave
// (integer only, so the device, the host and the oracle (rlo_testvec.h) agree bit for bit)
__host__ __device__ inline uint64_t rlo_mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint32_t storm_len_of(uint64_t seed, uint64_t b, uint32_t lo, uint32_t hi) {
    if (hi <= lo) return lo;
    if (lo == 0) lo = 1;
    const int elo = 31 - __builtin_clz(lo), ehi = 31 - __builtin_clz(hi);
    const uint64_t x = rlo_mix64(seed ^ 0xC5C5C5C5C5C5C5C5ull ^ (b * 0x9E3779B97F4A7C15ull));
    // octaves [2^e, 2^(e+1)) for e in [elo, ehi), plus the partial top one when hi is no power of 2
    const uint32_t noct = (uint32_t)(ehi - elo) + ((hi & (hi - 1u)) ? 1u : 0u);
    if (noct == 0) return lo;
    const uint32_t e = (uint32_t)elo + (uint32_t)(x % noct);
    const uint64_t base = 1ull << e;
    uint64_t v = base + ((x >> 32) % base);
    if (v < lo) v = lo;
    if (v > hi) v = hi;
    return (uint32_t)v;
}

}  // namespace rlo
