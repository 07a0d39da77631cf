/*
 * rootless_ops.h -- drop-in C API of the MI355X rootless collective engine
 * (librootless_ops.so), source-compatible with mierl/rootless-coll-mpi-ops'
 * rootless_ops.h (reference file:line cited per declaration).
 *
 * Same function names, argument meaning, enum values, RLO_user_msg layout and
 * return conventions as the reference.  Underneath, every engine is one rank of a
 * device world: the rank's mailbox rings live in GPU HBM (peer HBM over xGMI when the
 * ranks of the communicator sit on different GPUs of the node), a persistent HIP
 * progress kernel forwards along the skip-ring overlay and merges votes, and this
 * library drains the rank's pickup ring in RLO_make_progress_all, running the
 * judge / action callbacks on the host (DESIGN.md "Host-service mode").
 *
 * Differences a caller can observe (DESIGN.md lists them with reasons):
 *   - RLO_msg_t / RLO_proposal_state are opaque handles (the reference exposes MPI
 *     request fields nobody reads);
 *   - a judge callback returning neither 0 nor 1 counts as 0 (the reference never
 *     votes and the proposal hangs, rootless_ops.c:720-722);
 *   - one communicator must stay inside one node (hipIpc mappings).
 */
#ifndef ROOTLESS_OPS_H_
#define ROOTLESS_OPS_H_

#include <assert.h>
#include <mpi.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <unistd.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rootless_ops.h:44-47: a debug counter the reference tests update (defined once, here in
 * the library, instead of in every translation unit) */
extern int total_pickup;

#define RLO_MSG_SIZE_MAX 32768 /* rootless_ops.h:49 */

enum RLO_COMM_TAGS { /* rootless_ops.h:50-61, values fixed */
    RLO_BCAST,
    RLO_JOB_DONE,
    RLO_IAR_PROPOSAL,
    RLO_IAR_VOTE,
    RLO_IAR_DECISION,
    RLO_BC_TEARDOWN,
    RLO_IAR_TEARDOWN,
    RLO_P2P,
    RLO_SYS,
    RLO_ANY_TAG
};

typedef enum REQ_STATUS { /* rootless_ops.h:63-68 */
    RLO_COMPLETED,
    RLO_IN_PROGRESS,
    RLO_FAILED,
    RLO_INVALID
} RLO_Req_stat;

typedef int RLO_ID;   /* rootless_ops.h:70 */
typedef int RLO_Vote; /* rootless_ops.h:71: 1 yes, 0 no */

typedef struct IAR_Single_Prop_CTX { /* rootless_ops.h:73-75 */
    void* my_proposal;
} ISP;

/* rootless_ops.h:77: judge(proposal data | NULL, ctx) -> 0 / 1;  action(serialized PBuf, ctx) */
typedef int (*iar_cb_func_t)(const void* msg_buf, void* app_ctx);

typedef struct progress_engine RLO_engine_t;
typedef struct RLO_msg_generic RLO_msg_t;
typedef struct Proposal_state RLO_proposal_state;

/* rootless_ops.h:84-91, same layout: buf = [origin int32][data 32768 B]; for decisions
 * pid / vote / data_len / data come from the PBuf (rootless_ops.c:920-932) */
typedef struct user_msg {
    char buf[RLO_MSG_SIZE_MAX + sizeof(int)];
    int type;
    RLO_ID pid;
    RLO_Vote vote;
    size_t data_len;
    char* data;
} RLO_user_msg;

/* rootless_ops.h:151 (declared, never defined by the reference): returns the message's user view */
RLO_user_msg* RLO_user_msg_new(RLO_msg_t* gen_msg_in);

/* rootless_ops.c:289-317: a message whose header carries my rank; _bc copies n bytes */
RLO_msg_t* RLO_msg_new_generic(RLO_engine_t* eng);
RLO_msg_t* RLO_msg_new_bc(RLO_engine_t* eng, void* buf_in, int send_size);
int RLO_msg_free(RLO_msg_t* msg_in); /* :331-340 */

/* :319-325: 1 when the message has left this rank (its command was taken by the device) */
int RLO_msg_test_isends(RLO_engine_t* eng, RLO_msg_t* msg_in);

/* :467-522: collective over mpi_comm (all ranks call it); msg_size_max sizes the device
 * slots (0 = RLO_MSG_SIZE_MAX); callbacks may be NULL for bcast-only engines */
RLO_engine_t* RLO_progress_engine_new(MPI_Comm mpi_comm, size_t msg_size_max, void* approv_cb_func, void* app_ctx,
                                      void* app_proposal_action);
/* :1606-1647: collective quiescence (every bcast and decision delivered), then teardown */
int RLO_progress_engine_cleanup(RLO_engine_t* eng);

/* :538-549: drain every engine's pickup ring (deliveries, judge / action callbacks) */
int RLO_make_progress_all(void);
int RLO_get_engine_id(RLO_engine_t* eng); /* :524-527 */
MPI_Comm RLO_get_my_comm(RLO_engine_t* eng); /* :528-531 */

/* :1581-1604: rootless bcast from this rank; the engine owns msg_in afterwards */
int RLO_bcast_gen(RLO_engine_t* eng, RLO_msg_t* msg_in, enum RLO_COMM_TAGS tag);

/* :938-979: 1 and the next received message (lent until RLO_user_msg_recycle), or 0 */
int RLO_user_pickup_next(RLO_engine_t* eng, RLO_user_msg** msg_out);
int RLO_user_msg_recycle(RLO_engine_t* eng, RLO_user_msg* msg_in); /* :981-992 */

/* :876-906: -1 while the vote runs, else the decision (0 / 1) */
int RLO_submit_proposal(RLO_engine_t* eng, char* proposal, size_t prop_size, RLO_ID my_proposal_id);
int RLO_check_proposal_state(RLO_engine_t* eng, int pid); /* :869-872 (pid ignored, as there) */
int RLO_get_vote_my_proposal(RLO_engine_t* eng);          /* :1666-1673: -1 if not complete */
int RLO_proposal_reset(RLO_proposal_state* ps);           /* :1649-1664 */

/* :128-152 utilities */
unsigned long RLO_get_time_usec(void);
void RLO_get_time_str(char* str_out);
int RLO_get_my_rank(void);
int RLO_get_world_size(void);

/* ---- extensions (not in the reference) */
/* tree parent the message arrived from (the reference's irecv_stat.MPI_SOURCE), -1 if none */
int RLO_user_msg_source(const RLO_user_msg* msg);
/* HIP device ordinal this engine's rank lives on */
int RLO_engine_device(RLO_engine_t* eng);
/* Device memory held between engines.  An engine's device regions go back to a per-process pool
 * at cleanup and are reused by the next engine; the last engine's cleanup in a process frees every region no other
 * process ever mapped and closes the idle imports of peers' regions.  Regions a multi-GPU engine exported to other
 * processes stay pooled (up to RLO_POOL_CAP_BYTES free bytes, default 8 GiB, then retired but kept): freeing memory a
 * peer may still map is unsafe.  RLO_device_memory_release(comm) gives those back too: collective over
 * every process that shared engines with this one, called when none of them has an engine; 0 or -1 */
int RLO_device_memory_release(MPI_Comm comm);

/* Device judges: RLO_progress_engine_new_dj creates an engine whose proposals are judged on the
 * GPU by a registered predicate instead of approv_cb_func -- no host round trip per tree hop, and
 * the originator's final judge(NULL) approves (as every device judge does).  action callbacks still
 * run on this thread with the proposal's PBuf when a decision 1 arrives for a proposal this rank
 * approved (rootless_ops.c:842).  Collective like RLO_progress_engine_new; every rank passes its
 * own judge (kinds must agree):
 *   RLO_DJUDGE_APPROVE  approve every proposal;
 *   RLO_DJUDGE_ISP      testcases.c:18-37 is_proposal_approved_cb with this rank's string isp;
 *   RLO_DJUDGE_HASH     decline iff splitmix64(seed ^ rank << 32 ^ pid) % 1e6 < ppm (testing). */
#define RLO_HAVE_DEVICE_JUDGE 1
enum { RLO_DJUDGE_APPROVE = 0, RLO_DJUDGE_ISP = 2, RLO_DJUDGE_HASH = 3 };
typedef struct {
    int kind;
    const char* isp;
    unsigned int ppm;
    unsigned long long seed;
} RLO_device_judge;
RLO_engine_t* RLO_progress_engine_new_dj(MPI_Comm mpi_comm, size_t msg_size_max, const RLO_device_judge* judge,
                                         void* app_ctx, void* app_proposal_action);

/* Proposal pool (PROPOSAL_POOL_SIZE, rootless_ops.c:30, :159-165, :1251-1366 -- declared but never
 * wired in the reference, which keeps ONE my_own_proposal per engine, :241).  With the environment
 * variable RLO_PROPOSAL_POOL=d (1..16, the largest value over the engine's ranks wins) at
 * RLO_progress_engine_new, a rank may call RLO_submit_proposal again while earlier own proposals are
 * still in flight: up to d run at once (further ones wait, in submission order, for a slot), each
 * decided independently.  RLO_check_proposal_state(eng, pid) then reports the state of THAT pid (the
 * reference ignores pid; an unknown pid still reports the most recent proposal), RLO_get_vote_proposal
 * (eng, pid) returns its vote (-1 while not completed) and forgets it; RLO_get_vote_my_proposal keeps
 * meaning the most recently submitted proposal.
 * d = 1 (the default) is the reference's behaviour. */
#define RLO_HAVE_PROPOSAL_POOL 1
int RLO_proposal_pool_depth(RLO_engine_t* eng);
int RLO_get_vote_proposal(RLO_engine_t* eng, RLO_ID pid);

#ifdef __cplusplus
}
#endif
#endif /* ROOTLESS_OPS_H_ */
