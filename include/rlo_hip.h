/*
 * rlo_hip.h -- C ABI of the MI355X rootless collective engine (librlo_hip.so).
 *
 * This is the device-engine layer underneath the drop-in rootless_ops.h API.
 * Plain C types only (no HIP / torch types in signatures): a stream is passed
 * as `void*` (a hipStream_t, NULL = default stream).
 *
 * A world is N ranks.  It is hosted by one or more PARTS (contiguous rank ranges,
 * one per process / GPU); every rank of a part is one 256-thread workgroup of that
 * part's persistent progress kernel.  Each rank's inboxes are SPSC rings in its
 * part's HBM, one per overlay in-edge and virtual channel; producers in other
 * parts store into them through hipIpc mappings (xGMI across GPUs)
 * (DESIGN.md "Data layout").
 * A *program* is the workload the kernel runs until every rank is quiescent:
 *   storm   : K bcasts from random originators          (replaces RLO_bcast_gen +
 *             RLO_make_progress_all + RLO_user_pickup_next loops, rootless_ops.c:1581, :538, :938)
 *   latency : one bcast at a time, completion latency per round
 *   iar     : every rank runs its own proposal list, device judge, vote AND,
 *             decision bcast (RLO_submit_proposal :876 ... _iar_decision_handler :814)
 */
#ifndef RLO_HIP_H
#define RLO_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ errors */
#define RLO_OK 0
#define RLO_E_INVAL (-1)     /* bad argument / unsupported size                          */
#define RLO_E_HIP (-2)       /* a HIP runtime call failed (rlo_last_hip_error)            */
#define RLO_E_OCCUPANCY (-3) /* the ranks cannot all be co-resident on the device         */
#define RLO_E_DEVICE (-4)    /* the kernel reported an error (see rlo_rank_stats_t.error) */
#define RLO_E_NOPROGRAM (-5) /* rlo_launch without a program                              */
#define RLO_E_NODEVICE (-6)  /* no HIP device                                              */
#define RLO_E_NOTCONNECTED (-7) /* part created but rlo_part_connect not called yet          */
#define RLO_E_AGAIN (-8)     /* host-service ring full / nothing to do, retry after progress  */
#define RLO_E_TIMEOUT (-9)   /* shared host service: the leader did not answer in time         */
#define RLO_E_STALE (-10)    /* a peer part's memory, as mapped here, is not what that part holds now (an IPC
                                mapping of an earlier allocation): rlo_part_connect checks every mapped region */

/* device error codes (rlo_rank_stats_t.error) */
#define RLO_DERR_TIMEOUT 1
#define RLO_DERR_VOTE_RING 2
#define RLO_DERR_PID_COLLISION 3 /* proposal carries the receiver's own pid (rootless_ops.c:690) */
#define RLO_DERR_VOTE_ORPHAN 4
#define RLO_DERR_LOG_FULL 5
#define RLO_DERR_BAD_SLOT 6
#define RLO_DERR_HOST_CMD 7      /* malformed / unexpected host-service command                */
#define RLO_DERR_BULK 8          /* a bulk-message index / job field out of range (a bug: reported
                                    instead of touching memory outside the heaps); site 14: a device
                                    program's VERIFY read a granule that is not what the origin wrote
                                    (aux value = receiver rank & 0xff << 16 | 16-KiB block of the message) */
#define RLO_DERR_XCD 9           /* a RLO_PART_ONE_XCD world's rank-waves were not all placed on one XCD
                                    (aux = the first XCC id seen + 1 << 8 | this wave's + 1)     */

/* ------------------------------------------------------------------ topology (host only) */
/* skip-ring overlay, restated from rootless_ops.c:1416-1579; usable without a GPU */
int rlo_topology(int n, int rank, int* level, int* last_wall, int* send_channel_cnt, int* send_list_len,
                 int* send_list /* >= 16 entries */);
int rlo_children(int n, int rank, int origin, int from /* -1: originate */, int* out /* >= 16 */);

/* ------------------------------------------------------------------ world */
typedef struct rlo_world rlo_world_t;

typedef struct {
    int32_t n_ranks;      /* world size, 2 .. 4096                                        */
    uint32_t max_payload; /* payload bytes per slot (rounded up to 16); default 4096       */
    uint32_t ring_slots;  /* forward ring capacity (power of two); 0 = auto               */
    int32_t device;       /* HIP device ordinal; -1 = current                              */
    /* bulk messages (longer than max_payload, up to bulk_max bytes): announced through the
     * rings, moved by mover workgroups of the same launch (DESIGN.md "Bulk messages").
     * bulk_max 0 = no bulk messages */
    uint64_t bulk_max;
    uint32_t bulk_slots;  /* heap slots per origin (power of two <= 8, N * slots <= 1024); 0 = 2 (1 beyond 512 ranks) */
    uint32_t movers;      /* mover workgroups of the part (>= 2, half scatter, half gather); 0 = auto */
    /* proposal pool (PROPOSAL_POOL_SIZE, rootless_ops.c:30): pending-proposal entries per origin
     * in every rank's table (power of two <= 16; N x pool x 16 B per rank, in LDS, or in HBM where it
     * would crowd the small copy path's stage out of LDS: rlo_world_info_t.pend_hbm); 0 = 2.  An iar
     * program keeps up to rlo_iar_cfg_t.pool <= this many own proposals in flight per rank */
    uint32_t proposal_pool;
    uint32_t flags;       /* RLO_PART_* (PEND_HBM, CHUNKED, ONE_XCD); 0 = none                      */
} rlo_world_cfg_t;

typedef struct {
    int32_t n_ranks, max_in_degree, max_fanout, edges;
    uint32_t ring_slots, slot_stride, vote_slots;
    uint32_t peers;       /* RLO_PEER_*: where this part's peer parts are (set by rlo_part_connect)     */
    uint64_t fwd_bytes, vote_bytes, ctrl_bytes; /* this part's regions                    */
    int32_t cus, blocks_per_cu;
    int32_t part, n_parts, rank_begin, rank_end; /* ranks [rank_begin, rank_end) are local */
    int32_t sys_scope;                           /* 1: system-scope remote stores and publishes: a peer part on
                                                    another GPU or in another process (peers)              */
    int32_t waves;                               /* waves per rank-workgroup: 8 (512 messages per
                                                    iteration) or 4 (256), chosen at creation     */
    uint32_t bulk_slots, movers;                 /* bulk: heap slots per origin, mover workgroups   */
    uint64_t bulk_max, heap_bytes;               /* bulk: largest message, this part's heap bytes   */
    uint32_t proposal_pool;                      /* pending entries per origin (own proposals in flight) */
    uint32_t pull;                               /* 1: large bcasts cross edges as header + reference into
                                                    the sender's relay ring (pulled payloads)           */
    /* the part's LDS layout (rlo_layout_plan gives the same answer without a GPU) */
    uint32_t nsmall;       /* 16-B chunks staged per message (the small copy path takes slots of <= nsmall) */
    uint32_t stage2_bytes; /* large-message LDS stage                                                 */
    uint32_t ll_ok;        /* 1: the latency / iar / host programs run with doorbells                 */
    uint32_t pend_hbm;     /* 1: the pending-proposal tables live in HBM, not LDS (large N x pool)     */
    uint32_t dyn_lds, static_lds; /* bytes of LDS per rank-workgroup                                  */
    uint32_t last_kernel;  /* the latest launch ran: 0 the progress kernel, 1 the hop kernel (the latency / iar
                              programs with doorbells: one wave per rank)                  */
    uint32_t info_pad;
} rlo_world_info_t;

/* single-part world: all N ranks on one GPU (replaces RLO_progress_engine_new :467-522
 * + bcomm_init :1454-1522 for every rank of the communicator at once) */
int rlo_world_create(const rlo_world_cfg_t* cfg, rlo_world_t** out);

/* ---- sharded world: one part per process / GPU.
 * create (allocates the rings this part consumes) -> export a fixed-size blob -> exchange
 * blobs out of band (MPI_Allgather, torch.distributed, a file) -> connect (maps every peer
 * part: same process = direct pointer, other process = hipIpc / dmabuf, xGMI across GPUs).
 * Every part must rlo_reset before ANY part launches (host barrier in between), and every part must close its
 * imports (rlo_part_close_imports) before ANY part destroys its world (host barrier in between): a part that frees
 * and re-allocates memory a peer still imports can export, for its NEW allocation, a handle that maps the OLD one
 * (seen on MI355X / ROCm 7.2 in 8-part worlds; rlo_part_connect's nonce check then fails with RLO_E_STALE). */
#define RLO_PART_BLOB_BYTES 512u
#define RLO_PEER_OTHER_GPU 1u  /* rlo_world_info_t.peers: some peer part is on another GPU (xGMI; the chunked bulk plan) */
#define RLO_PEER_IMPORTED 2u   /* ... some peer part is in another process (its regions hipIpc-imported)            */
#define RLO_PART_UNCACHED 1u /* allocate the part's rings uncached (for peer GPUs writing over xGMI) */
#define RLO_PART_PEND_HBM 4u /* the pending-proposal tables in HBM whatever the world size (the layout an 8-GPU
                                 * world takes, rehearsed at smaller N; every part must set it alike) */
#define RLO_PART_ONE_XCD 8u  /* rlo_world_create, no bulk, as many ranks as one XCD's CUs hold (<= 256; checked at
                                 * launch): the rings cached and every rank-wave of the
                                 * hop kernel on ONE XCD, so a hand-off store stays in that XCD's L2 and the
                                 * consumer's load hits it (one hop 0.51 vs 1.11 us, tools/xcd_probe.hip).  Only the
                                 * hop kernel's programs run (latency; iar with pool 1, <= 16 ranks, device judges);
                                 * a launch that needs the progress kernel returns RLO_E_INVAL */
#define RLO_PART_CHUNKED 2u  /* bulk messages take the multi-GPU plan (chunked scatter + all-gather) even when every
                                 * part is on one GPU: the 8-GPU path, rehearsed on one (every part must set it alike) */
typedef struct {
    int32_t n_ranks;           /* world size                                               */
    int32_t n_parts, part;     /* number of parts, this part                                */
    const int32_t* part_begin; /* [n_parts + 1] rank boundaries, NULL = even contiguous split */
    uint32_t max_payload, ring_slots;
    int32_t device;            /* -1 = current                                              */
    uint32_t flags;            /* RLO_PART_*                                                */
    uint64_t bulk_max;         /* as rlo_world_cfg_t (the same on every part)               */
    uint32_t bulk_slots, movers;
    uint32_t proposal_pool, pad; /* as rlo_world_cfg_t (the same on every part)             */
} rlo_part_cfg_t;
int rlo_part_create(const rlo_part_cfg_t* cfg, rlo_world_t** out);
int rlo_part_export(rlo_world_t* w, void* blob, uint32_t cap); /* returns RLO_PART_BLOB_BYTES */
int rlo_part_connect(rlo_world_t* w, const void* blobs /* n_parts x RLO_PART_BLOB_BYTES, by part */, int n_parts);
/* map part q's regions now (rlo_part_connect then skips q).  Parts in several processes import one exporter at a
 * time -- every part imports part k's regions while part k imports nothing, host barrier, next k: a part importing
 * while its peers import its own regions was seen to hand them a mapping of ANOTHER part's region for its handle
 * (8 parts on MI355X / ROCm 7.2) */
int rlo_part_import(rlo_world_t* w, const void* blob /* RLO_PART_BLOB_BYTES */, int q);
int rlo_world_destroy(rlo_world_t* w);
/* close this part's hipIpc imports of its peers' regions (rlo_world_destroy does it too); the part can no longer
 * launch.  Lets every part of a world drop its imports before any part frees the memory they map */
int rlo_part_close_imports(rlo_world_t* w);
int rlo_world_query(const rlo_world_t* w, rlo_world_info_t* out);

/* ---- the per-process region pool.  A destroyed world's device regions stay in a per-process pool for
 * the next world, and imports of peers' regions stay open (idle) for the peer's next world: exported memory freed and
 * re-exported world after world gave importers mappings of OTHER memory on MI355X / ROCm 7.2.  Free bytes beyond
 * RLO_POOL_CAP_BYTES (environment, default 8 GiB) leave the pool: a region no other process ever mapped is freed at
 * once, an exported one is RETIRED and freed only by RLO_TRIM_RETIRED.  To give every byte back, all processes that
 * shared worlds run the world-wide close: each rlo_pool_trim(RLO_TRIM_IMPORTS | RLO_TRIM_FREE | RLO_TRIM_EXPORTED)
 * once none of its worlds is alive, a barrier, then each rlo_pool_trim(RLO_TRIM_RETIRED).  No replacement in the
 * reference (MPI owns its buffers). */
#define RLO_TRIM_IMPORTS 1u  /* close this process's idle imports of peers' regions                            */
#define RLO_TRIM_FREE 2u     /* hipFree the free regions no other process ever mapped                          */
#define RLO_TRIM_RETIRED 4u  /* hipFree the retired exported regions: only after EVERY peer process trimmed its
                                imports (a world-wide close with a barrier)                                     */
#define RLO_TRIM_EXPORTED 8u /* retire every free exported region (RLO_TRIM_RETIRED then frees it)               */
int rlo_pool_trim(uint32_t what, uint64_t* freed_bytes);
/* out[6]: bytes held by live worlds, free never-exported, free exported, retired; imports in use, idle imports */
int rlo_pool_stats(uint64_t* out, uint32_t cap);

/* ------------------------------------------------------------------ programs */
#define RLO_FLAG_LOG 1u  /* record every delivery / judge / action / result (+ payload bytes) */
#define RLO_FLAG_HIST 2u /* per-delivery latency histogram                                  */
#define RLO_FLAG_PROF 4u /* per-phase cycle accounting (diagnostic)                         */
#define RLO_FLAG_TIMELINE 8u /* latency program: per-round event clocks (rlo_timeline); diagnostics build only
                                (make DIAG=1 -> lib_diag/; the product library refuses it with RLO_E_INVAL) */

#define RLO_ORDER_RANDOM 0u /* origin of bcast b = splitmix64(seed + b) % N                      */
#define RLO_ORDER_SLOTS 1u  /* origin of bcast b = b % N: every rank originates in every "slot" of N
                               bcasts (BASELINE configs[4]: collision-heavy simultaneous originators) */
typedef struct {
    uint64_t seed;       /* workload seed                                                  */
    int64_t k;           /* bcasts in the storm                                            */
    uint32_t len;        /* payload bytes (<= max_payload, or <= bulk_max with bulk)        */
    uint32_t window;     /* max originations per rank per progress iteration (0 = 64, max 64) */
    uint32_t flags;      /* RLO_FLAG_*                                                      */
    uint32_t log_cap;    /* log records per rank when RLO_FLAG_LOG                          */
    uint32_t len_max;    /* > len: mixed sizes, bcast b has storm_len(seed, b) in [len, len_max]
                            (piecewise log-uniform, oracle/rlo_testvec.h rlo_tv_len)           */
    uint32_t order;      /* RLO_ORDER_*                                                     */
} rlo_storm_cfg_t;
int rlo_program_storm(rlo_world_t* w, const rlo_storm_cfg_t* cfg);

/* one bcast per round, round i from splitmix64(seed + i) % N; round i+1 starts when every
 * rank has picked up round i.  rlo_latencies() returns per-round completion ticks (10 ns):
 * origination -> last pickup, on one clock only when the world is one part.  The hop kernel
 * (rlo_hop.hip) takes the largest of the receivers' own pickup clocks (the reference harness's
 * t_recv); the progress kernel (bulk rounds) the clock of the rank whose pickup completed the
 * round's delivery count, so it includes that count's round trip.  Worlds split over
 * parts (processes / GPUs, <= 8192 rounds) share the round word through part 0; there
 * rlo_round_ticks() (on the part holding world rank 0) returns the clock of world rank 0 when it
 * saw round i complete: successive differences are closed-loop round times on ONE clock. */
int rlo_program_latency(rlo_world_t* w, uint32_t rounds, uint32_t len, uint64_t seed, uint32_t flags);

/* RLO_FLAG_TIMELINE: the first min(rounds, 64) rounds' event clocks (low 32 bits of the 10-ns clock; 0 =
 * not seen on this part), row r = [8 global events][9 columns x local ranks]: global 0 origination, 1 scatter
 * job posted, 2 claimed by a mover, 3 moved (completion counts added), 4 round complete (last pickup), 5 last
 * receiver's VERIFY done; per rank: arrival, bulk completion (ring-slot messages: their forwards issued),
 * tree parent + 1, and for a message the doorbell pass took, when the polls that found it were issued and
 * when that pass began (bulk: when the poll that found the copy complete began, when its loads were back), and for
 * a bulk announcement when its forwards were issued and when wave 0's next spin began (a ring-slot message the
 * doorbell pass took: two probes inside that pass), two probes inside the lone-message path.  Copies rows * *stride words to out (cap words), returns the rows copied. */
int rlo_timeline(rlo_world_t* w, uint32_t* out, uint64_t cap, uint32_t* stride);

#define RLO_JUDGE_APPROVE 0u /* approve everything                                           */
#define RLO_JUDGE_MASK 1u    /* decline iff mask[rank] != 0 (arg != NULL)                     */
#define RLO_JUDGE_ISP 2u     /* testcases.c:18-37 is_proposal_approved_cb, per-rank string    */
#define RLO_JUDGE_HASH 3u    /* decline iff splitmix64(seed^rank<<32^pid) % 1e6 < ppm         */

typedef struct {
    uint32_t judge_kind, judge_ppm;
    uint64_t judge_seed;
    const uint8_t* judge_mask; /* [N] for RLO_JUDGE_MASK                                   */
    const char* judge_isp;     /* N NUL-terminated strings, concatenated (RLO_JUDGE_ISP)    */
    uint32_t flags, log_cap;
    uint32_t pool;             /* own proposals in flight per rank (<= the world's proposal_pool);
                                  0 = 1: one own proposal per engine (rootless_ops.c:241)     */
    uint32_t pad;
} rlo_iar_cfg_t;
/* proposals in per-origin submission order: origin[i] submits pid[i] with
 * data[data_off[i] .. +data_len[i]); a rank keeps up to cfg->pool of its proposals in flight
 * (the proposal pool, rootless_ops.c:30, :1251-1366) and submits the next one as soon as a pool
 * slot's decision has been broadcast; pool 1 = the reference's one own proposal (:241). */
int rlo_program_iar(rlo_world_t* w, const rlo_iar_cfg_t* cfg, int64_t nprop, const int32_t* origin, const int32_t* pid,
                    const uint8_t* data, const uint32_t* data_off, const uint32_t* data_len);

/* one event record (parity log / host pickup ring).  A bulk delivery (kind 1 | 10 << 8) logs
 * len = message bytes and, once its VERIFY job ran, aux | payload_idx << 32 = the message checksum
 * (the oracle's orc_msg_checksum) */
typedef struct {
    uint32_t kind; /* 1 deliver | 2 judge | 3 action | 4 result | 5 error | 6 judge req | 7 own judge req; | tag << 8 */
    int32_t origin, from;
    uint32_t id, len;
    int32_t vote;
    uint32_t aux, payload_idx;
} rlo_log_rec_t;

/* ---- host-service program: the kernel serves the rootless_ops.h API of this part's ranks.
 * The host posts originations and judge verdicts into a per-rank command ring and drains a
 * per-rank pickup ring of events; both rings live in pinned host memory.  The kernel runs
 * (persistent) from rlo_launch_ex until every local rank has received RLO_CMD_QUIT.
 * Replaces the MPI transport under RLO_bcast_gen :1581, RLO_make_progress_all :538,
 * RLO_user_pickup_next :938, RLO_submit_proposal :876 and the judge / action callbacks
 * (:698, :773, :842), which the host layer (librootless_ops.so) invokes on pickup events. */
typedef struct {
    uint32_t cmd_slots;      /* command ring capacity per rank (power of two), 0 = 256       */
    uint32_t pickup_slots;   /* pickup ring capacity per rank (power of two, 64 .. 16384), 0 = 1024 */
    uint32_t idle_timeout_s; /* kernel stops (RLO_DERR_TIMEOUT) after this long without any
                                progress; 0 = never                                          */
    uint32_t flags;
    uint32_t pool;           /* own proposals a rank may keep in flight (<= the world's proposal_pool):
                                the proposal pool (rootless_ops.c:30); 0 = 1 (my_own_proposal, :241).
                                A proposal command beyond it waits at the head of the command ring
                                and holds up every command behind it (judge verdicts too): keep
                                extra proposals on the host until an RLO_EV_RESULT frees a slot
                                (librootless_ops.so and rlo/host.py do)                           */
    uint32_t pad;
} rlo_host_cfg_t;
int rlo_program_host(rlo_world_t* w, const rlo_host_cfg_t* cfg);

/* command kinds: originations use the reference tags (enum RLO_COMM_TAGS) */
#define RLO_CMD_BCAST 0u      /* payload = user bytes; id = caller's sequence number           */
#define RLO_CMD_PROPOSAL 2u   /* payload = serialized PBuf (pid, vote, data_len, data) :1369   */
#define RLO_CMD_JUDGE 16u     /* verdict for an RLO_EV_JUDGE event: origin, pid, pseq, vote     */
#define RLO_CMD_OWN_JUDGE 17u /* verdict of the originator's final judge(NULL) (:773): id = pid,
                                 pseq = the RLO_EV_OWN_JUDGE event's aux (pool slot), vote       */
#define RLO_CMD_QUIT 18u      /* stop this rank's progress (after everything before it)          */
#define RLO_CMD_BULK 10u      /* bulk origination: payload = {u32 len, u32 q}; use rlo_host_bulk_send */
#define RLO_CMD_BULK_RELEASE 19u /* a bulk delivery was copied out: origin, pseq = heap slot        */
typedef struct {
    uint32_t kind;
    int32_t origin; /* RLO_CMD_JUDGE: origin of the proposal                                  */
    int32_t id;     /* BCAST: sequence number; PROPOSAL / JUDGE: pid                          */
    uint32_t pseq;  /* RLO_CMD_JUDGE: the event's aux (proposal sequence)                     */
    int32_t vote;   /* JUDGE / OWN_JUDGE: 0 or 1                                              */
    uint32_t pad;
} rlo_cmd_t;
/* world rank `rank` must be local; RLO_E_AGAIN when the command ring is full */
int rlo_host_post(rlo_world_t* w, int rank, const rlo_cmd_t* cmd, const void* payload, uint32_t len);

/* pickup events (rlo_log_rec_t.kind) */
#define RLO_EV_DELIVER_BCAST (1u | (0u << 8))    /* origin, from (tree parent), id, len + payload */
#define RLO_EV_DELIVER_DECISION (1u | (4u << 8)) /* origin, id = pid, vote = decision             */
#define RLO_EV_DELIVER_BULK (1u | (10u << 8))   /* origin, from, id, len, aux = heap slot: the bytes
                                                   are in this rank's heap (rlo_host_bulk_recv)   */
#define RLO_EV_ACTION 3u    /* decision 1 for a proposal this rank approved: run action (:842)   */
#define RLO_EV_RESULT 4u    /* my own proposal decided: id = pid, vote = decision                */
#define RLO_EV_JUDGE 6u     /* call judge(data): origin, from, id = pid, aux = pseq,
                               payload = the proposal's PBuf (len bytes)                        */
#define RLO_EV_OWN_JUDGE 7u /* call judge(NULL) for my proposal id (all votes were 1); aux = its
                               proposal-pool slot (echo it in RLO_CMD_OWN_JUDGE.pseq)          */
#define RLO_EV_JUDGED 8u    /* device judge (rlo_host_device_judge): origin, from, id = pid, vote =
                               verdict, aux = pseq, payload = PBuf -- informational, no reply        */
/* next event of local rank `rank`: 1 = got one (payload copied, up to cap bytes), 0 = none */
int rlo_host_poll(rlo_world_t* w, int rank, rlo_log_rec_t* ev, void* payload, uint32_t cap);
/* 1 while this part's kernel runs, 0 once it has ended (rlo_wait then reports its status) */
int rlo_host_running(rlo_world_t* w);
/* commands of local rank `rank` taken by the device so far / posted so far */
int rlo_host_cmd_count(rlo_world_t* w, int rank, uint64_t* consumed, uint64_t* posted);
/* number of HIP devices visible to this process (0 without a GPU) */
int rlo_device_count(void);
/* the NUMA node of HIP device `device` (its PCI function's numa_node in sysfs), -1 if unknown */
int rlo_device_numa_node(int device);

/* ---- bulk messages in the host-service program (the drop-in's RLO_bcast_gen beyond a slot).
 * rlo_host_bulk_stage: takes local rank `rank`'s next bulk sequence q, waits (RLO_E_AGAIN after
 * timeout_us) until every receiver released heap slot q mod B, and copies `len` bytes into the
 * rank's own heap slot; then post RLO_CMD_BULK with payload {u32 len, u32 q}.
 * rlo_host_bulk_copy: copies the message of an RLO_EV_DELIVER_BULK event (ev->len bytes) out of
 * this rank's heap; then post RLO_CMD_BULK_RELEASE with origin = ev->origin, pseq = ev->aux. */
/* the chunk / stripe / tile plan every rank derives for a bulk message of len bytes in an N-rank
 * world (cross: parts span GPUs); pure host arithmetic (rlo_device.hpp bulk_plan) */
/* direct = 1: one GPU -- one stripe (the message), every tile fanned out from the origin's copy */
typedef struct { uint32_t nchunks, stripe, chunk, tile, total_tiles, direct; } rlo_bulk_plan_t;
int rlo_bulk_plan(int n, uint64_t len, int cross, rlo_bulk_plan_t* out);
/* the LDS layout a part of this world would get (rlo_world_query's waves, nsmall, stage2_bytes, ll_ok,
 * pend_hbm, blocks_per_cu, ...), pure host arithmetic: no GPU needed.  The occupancy answers come from the
 * build's register guarantees (rlo_progress_kernel keeps 2 waves per SIMD in its 8-wave and 4-wave
 * non-doorbell forms, Makefile), not from the runtime; a part created on a GPU takes the runtime's */
typedef struct {
    int32_t n_ranks, n_parts, part;  /* even contiguous split, as rlo_part_create with part_begin NULL */
    uint32_t max_payload, ring_slots, flags;
    uint64_t bulk_max;
    uint32_t bulk_slots, movers, proposal_pool;
    int32_t cus;                     /* CUs of the GPU; 0 = 256 (MI355X)                                */
} rlo_plan_cfg_t;
int rlo_layout_plan(const rlo_plan_cfg_t* cfg, rlo_world_info_t* out);
/* the storm program's payload length of bcasts 0..k-1 (rlo_storm_cfg_t len, len_max, seed): the
 * workload generator's host side, for byte accounting (no GPU) */
int rlo_storm_lengths(uint64_t seed, uint64_t k, uint32_t len, uint32_t len_max, uint32_t* out);
int rlo_host_bulk_stage(rlo_world_t* w, int rank, const void* data, uint64_t len, uint32_t timeout_us, uint32_t* q);
int rlo_host_bulk_copy(rlo_world_t* w, int rank, const rlo_log_rec_t* ev, void* dst);

/* ---- the shared host service (rlo_shm.hpp): ONE process per GPU owns a host-service part and
 * its persistent kernel; the other rank processes of that part drive their ranks through a POSIX
 * shared-memory segment and never create GPU queues (a GPU's hardware scheduler time-slices whole
 * processes once more of them hold queues than it maps at once: DESIGN.md "one queue-holding
 * process per GPU").
 * Leader: rlo_host_share(name, stage bytes) BEFORE rlo_program_host (which then builds the host-side
 * rings in the segment and registers it with HIP), rlo_reset, rlo_launch_ex, rlo_host_wait_started;
 * once every client attached, rlo_host_unlink.  While the kernel runs, rlo_host_proxy must be called continuously
 * (a service thread): it moves client commands into the part's VRAM command ring, the clients'
 * pickup heads into the counters the kernel polls, and runs bulk copies for them.
 * Client: rlo_client_attach(name, world rank) and the rlo_client_* calls, which mirror
 * rlo_host_post / rlo_host_poll / rlo_host_cmd_count / rlo_host_bulk_stage / rlo_host_bulk_copy. */
int rlo_host_share(rlo_world_t* w, const char* shm_name, uint64_t stage_bytes);
int rlo_host_unlink(rlo_world_t* w);
int rlo_host_proxy(rlo_world_t* w);  /* one pass; returns the number of actions taken (>= 0) */
/* waits until every local rank's kernel workgroup serves (1), or RLO_E_TIMEOUT / RLO_E_DEVICE */
int rlo_host_wait_started(rlo_world_t* w, uint32_t timeout_ms);
/* marks the segment failed so clients stop waiting (engine setup aborted, kernel gone) */
int rlo_host_fail(rlo_world_t* w);
/* extension: the device judge registry (judge_kind / ppm / seed / mask / isp of cfg, as in
 * rlo_program_iar) judges this host-service part's proposals, and approves every originator's
 * final judge(NULL), instead of RLO_EV_JUDGE / RLO_EV_OWN_JUDGE round trips to the host.  Each
 * judged proposal is reported by a one-way RLO_EV_JUDGED event (vote = verdict, payload = PBuf), so
 * the host can still run action(PBuf) on approval.  Call after rlo_program_host, before launch. */
int rlo_host_device_judge(rlo_world_t* w, const rlo_iar_cfg_t* cfg);

typedef struct rlo_client rlo_client_t;
int rlo_client_attach(const char* shm_name, int rank, rlo_client_t** out);
int rlo_client_detach(rlo_client_t* c);
int rlo_client_state(rlo_client_t* c);  /* 0 not started, 1 serving, 2 exited, RLO_E_DEVICE */
int rlo_client_post(rlo_client_t* c, const rlo_cmd_t* cmd, const void* payload, uint32_t len);
int rlo_client_poll(rlo_client_t* c, rlo_log_rec_t* ev, void* payload, uint32_t cap);
int rlo_client_cmd_count(rlo_client_t* c, uint64_t* consumed, uint64_t* posted);
int rlo_client_bulk_put(rlo_client_t* c, const void* data, uint64_t len, uint32_t timeout_us, uint32_t* q);
int rlo_client_bulk_get(rlo_client_t* c, const rlo_log_rec_t* ev, void* dst);
/* diagnostics, 9 words: posted, forwarded, consumed, tail seen by the kernel, pickups consumed,
 * pickups written, pickup head seen by the kernel, kernel iterations (/4096 beat), state */
int rlo_client_debug(rlo_client_t* c, uint64_t* out);
/* diagnostics (kernel launched with RLO_HOST_DIAG set), 8 words valid once the rank stopped serving:
 * iterations with commands pending, iterations a proposal was held (own proposal active), iterations
 * blocked on pickup-ring room, host iterations, then commands seen -> drained in < 20 / 100 / 500 /
 * >= 500 us (counts) */
int rlo_client_hdiag(rlo_client_t* c, uint64_t* out);
/* diagnostics: commands the leader's proxy forwarded so far, and when (CLOCK_MONOTONIC ns) */
int rlo_client_fwd(rlo_client_t* c, uint64_t* fwd, int64_t* fwd_ns);

/* ------------------------------------------------------------------ run */
int rlo_reset(rlo_world_t* w, void* stream);           /* zero this part's counters (sync) */
#define RLO_LAUNCH_NO_RESET 1u
int rlo_launch_ex(rlo_world_t* w, void* stream, uint32_t flags); /* async launch of this part */
int rlo_launch(rlo_world_t* w, void* stream);          /* rlo_reset + rlo_launch_ex        */
/* a non-blocking HIP stream for one part's launch (parts of one process need one each) */
int rlo_stream_create(int device, void** stream);
int rlo_stream_destroy(void* stream);
int rlo_wait(rlo_world_t* w);                          /* sync; RLO_E_DEVICE on error  */
int rlo_run(rlo_world_t* w, void* stream, float* kernel_ms); /* launch + wait, HIP-event time */
int rlo_last_kernel_ms(rlo_world_t* w, float* ms);

/* ------------------------------------------------------------------ results */
typedef struct {
    uint64_t bcast_delivered, bcast_sum, originated;
    uint64_t dec_delivered, dec_approved, actions, judge_calls;
    uint64_t own_decided, own_approved, proposals_recv;
    uint64_t iterations, busy_iterations, stalls, log_count;
    uint64_t t_start, t_end;
    uint32_t error, error_aux;
    uint64_t prof[8];  /* RLO_FLAG_PROF: shader cycles per phase (poll, votes+select, classify,
                          admit, effects, copy, publish) */
    uint64_t dbg[8];   /* RLO_FLAG_PROF: engine counters (DESIGN.md "Diagnostics") */
    uint32_t hist[128];
    uint64_t unmarked_slots; /* staged ring slots whose header lacked the slot mark (RLO_DERR_BAD_SLOT) */
} rlo_rank_stats_t;


/* results of this part's ranks: stats index = rank - rank_begin; rlo_log takes the world rank */
int rlo_stats(rlo_world_t* w, rlo_rank_stats_t* out, int n);
int rlo_log(rlo_world_t* w, int rank, rlo_log_rec_t* out, uint32_t cap, uint8_t* payload, uint32_t payload_stride);
int rlo_latencies(rlo_world_t* w, uint64_t* ticks, uint32_t cap);
int rlo_round_ticks(rlo_world_t* w, uint64_t* ticks, uint32_t cap);

/* this part's device error word (ctrl word 0): the first RLO_DERR_* code any workgroup of any part
 * raised (0 = none) and, for RLO_DERR_BULK, aux = site << 24 | value */
int rlo_device_error(rlo_world_t* w, uint32_t* code, uint32_t* aux);
/* diagnostics of a bulk world: its part's job-ring control words (rlo_device.hpp kJctl*: posted and
 * head per class, exited progress workgroups, tiles moved per class, gather waits) */
int rlo_bulk_debug(rlo_world_t* w, uint64_t* out, uint32_t cap);
const char* rlo_strerror(int code);
int rlo_last_hip_error(void);

#ifdef __cplusplus
}
#endif
#endif
