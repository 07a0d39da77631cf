/*
 * rlo_oracle.h -- TEST INFRASTRUCTURE ONLY: clean-room CPU restatement of the
 * reference's rootless-bcast / IAR path (mierl/rootless-coll-mpi-ops).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so, and only as the checker / CPU baseline.  The product
 * (librlo_hip.so) never links or calls it.
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks every function here
 * against fixtures captured from the compiled reference (tests/golden/, made by
 * tests/golden/gen_fixtures.py running oracle/_ref/ref_harness under MPICH).
 */
#ifndef RLO_ORACLE_H
#define RLO_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_FANOUT 32

/* message classes = enum RLO_COMM_TAGS values (rootless_ops.h:50-61) */
enum { ORC_BCAST = 0, ORC_PROPOSAL = 2, ORC_VOTE = 3, ORC_DECISION = 4 };

/* ---- overlay topology: rootless_ops.c:1416-1522 (is_powerof2, get_level, last_wall, bcomm_init) */
int orc_topology(int n, int rank, int* level, int* last_wall, int* send_channel_cnt, int* send_list_len, int* send_list);
/* forwarding rule: rootless_ops.c:1104-1225 (_bc_forward) and :1587 (originate, from < 0) */
int orc_children(int n, int rank, int origin, int from, int* out);
/* rootless_ops.c:1559-1579 */
int orc_fwd_send_cnt(int n, int rank, int origin, int from);
/* rootless_ops.c:1534-1556 */
int orc_check_passed_origin(int n, int rank, int origin, int to);
/* single bcast from origin through FIFO mailboxes; parent[r] = sender, -1 at origin; returns #deliveries */
int orc_tree(int n, int origin, int32_t* parent);

/* ---- workload + checksums (DESIGN.md "storm workload") */
void orc_payload(uint32_t origin, uint32_t bid, uint8_t* out, size_t len);
uint32_t orc_origin_of(uint64_t seed, uint64_t bid, uint32_t n);
uint32_t orc_chunk_mix(uint32_t q, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3);
uint64_t orc_msg_checksum(uint32_t origin, uint32_t bid, uint32_t tag, const uint8_t* payload, uint32_t len);
uint64_t orc_region_hash(const uint8_t* payload, size_t len);
uint64_t orc_fnv1a(const uint8_t* p, size_t len); /* FNV-1a 64 of exactly len bytes */

/* ---- storm: every bid b in [0,k) originates at orc_origin_of(seed,b,n) with a len-byte payload.
 * Message-passing simulation: per-rank FIFO inbox, payload copied on every tree edge.
 * Outputs (any may be NULL): parent[b*n + r] (-1 for origin), count[r], sum[r] (checksum of checksums).
 * Returns number of deliveries, or -1 on internal error.                                                */
int64_t orc_storm(int n, uint64_t seed, int64_t k, uint32_t len, int32_t* parent, int64_t* count, uint64_t* sum);
/* same outputs, computed analytically (every non-origin receives every bcast exactly once) */
int64_t orc_storm_expected(int n, uint64_t seed, int64_t k, uint32_t len, int64_t* count, uint64_t* sum);
/* the same with mixed payload sizes (bcast b has rlo_tv_len(seed, b, len_lo, len_hi) bytes) and an
 * origin order (0 random, 1 slots: b % n).  Messages longer than the reference's 32,764-B data region
 * are bulk messages: delivered to every other rank byte for byte like the rest, their
 * bytes are not copied per hop in the simulation (a pure function of origin, bid and len) */
int64_t orc_storm2(int n, uint64_t seed, int64_t k, uint32_t len_lo, uint32_t len_hi, uint32_t order, int32_t* parent,
                   int64_t* count, uint64_t* sum);
int64_t orc_storm_expected2(int n, uint64_t seed, int64_t k, uint32_t len_lo, uint32_t len_hi, uint32_t order,
                            int64_t* count, uint64_t* sum);
uint32_t orc_len_of(uint64_t seed, uint64_t bid, uint32_t lo, uint32_t hi);
/* orc_storm2's workload on `threads` host threads (bench.py's multi-core cpu_baseline leg): the ranks
 * are dealt to the threads, every rank's inbox is a mutex-guarded FIFO, and every tree edge copies
 * the bytes (malloc + memcpy, an MPI send).  Same count / sum outputs (parents are not recorded). */
int64_t orc_storm_mt(int n, uint64_t seed, int64_t k, uint32_t len_lo, uint32_t len_hi, uint32_t order, int threads,
                     int64_t* count, uint64_t* sum);
uint32_t orc_origin_of2(uint64_t seed, uint64_t bid, uint32_t n, uint32_t order);

/* ---- IAR (proposal / vote / decision): rootless_ops.c:668-917, :1036-1070 */
enum { ORC_JUDGE_APPROVE = 0, ORC_JUDGE_MASK = 1, ORC_JUDGE_ISP = 2, ORC_JUDGE_HASH = 3 };
typedef struct {
    int kind;
    const uint8_t* decline; /* MASK: n bytes, decline iff decline[rank] && arg != NULL */
    const char* isp;        /* ISP: n NUL-terminated strings, concatenated (testcases.c:18-37 semantics) */
    uint64_t seed;          /* HASH: decline iff arg != NULL && hash(seed,rank,pid) % 1000000 < ppm */
    uint32_t ppm;
} orc_judge_cfg;

uint32_t orc_judge_hash(uint64_t seed, uint32_t rank, int32_t pid);

/* event records, 6 x int32 each: {ev, rank, pid, a, b, c} */
enum { ORC_EV_JUDGE = 1, ORC_EV_ACTION = 2, ORC_EV_PICKUP = 3, ORC_EV_RESULT = 4, ORC_EV_ERROR = 5 };
/* JUDGE : a = arg is NULL, b = return, c = proposal origin
 * ACTION: a = vote field of the serialized PBuf (always 1), b = data_len, c = origin
 * PICKUP: a = decision, b = origin, c = data_len (7, "IAR_DEC")
 * RESULT: a = decision (originator, RLO_get_vote_my_proposal)
 * ERROR : a = code (1 = proposal carries my own pid: rootless_ops.c:690)                           */

/* All proposals are submitted up front (proposal i from origin[i] with pid[i] and data
 * data + data_off[i], data_len[i] bytes); runs to quiescence.  Returns #events written
 * (or -1 if cap was too small / error).                                                       */
int orc_iar(int n, int nprop, const int32_t* origin, const int32_t* pid, const char* data, const int32_t* data_off,
            const int32_t* data_len, const orc_judge_cfg* judge, int32_t* events, int cap);

/* consensus throughput model: every rank keeps one outstanding proposal (pid = iter*n + rank,
 * 16-byte body) for p iterations.  Outputs totals; returns #decisions or -1.                   */
int64_t orc_iar_bench(int n, int p, const orc_judge_cfg* judge, int64_t* approved, int64_t* judge_calls,
                      int64_t* actions);
/* the same workload with every event recorded (orc_iar's format); returns #events or -1 */
int orc_iar_rounds(int n, int p, const orc_judge_cfg* judge, int32_t* events, int cap);

/* the proposal pool (PROPOSAL_POOL_SIZE, rootless_ops.c:30, :1251-1366): every rank keeps up to
 * `pool` own proposals in flight.  orc_iar_pool: each origin submits its proposals (list order)
 * whenever a pool slot is free; orc_iar_rounds_pool: orc_iar_rounds with `pool` outstanding per
 * rank.  Same event format; returns #events or -1.                                             */
int orc_iar_pool(int n, int nprop, const int32_t* origin, const int32_t* pid, const char* data, const int32_t* data_off,
                 const int32_t* data_len, const orc_judge_cfg* judge, int pool, int32_t* events, int cap);
int orc_iar_rounds_pool(int n, int p, int pool, const orc_judge_cfg* judge, int32_t* events, int cap);

#ifdef __cplusplus
}
#endif
#endif
