/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Driver that links the *compiled reference* (oracle/_ref/rootless_ops.o, built
 * from /root/reference/rootless_ops.c in place by oracle/Makefile) and runs it
 * under host MPI to capture golden vectors.  Built a second time with -DRLO_DROPIN
 * against include/rootless_ops.h + librootless_ops.so (oracle/_ref/dropin_harness):
 * the same capture modes then drive the MI355X drop-in, and tests/ compare the two.  It only uses the public API of
 * rootless_ops.h, plus the reference's own test callbacks from testcases.c
 * (is_proposal_approved_cb / proposal_action_cb, testcases.c:18-42) and the
 * two exported topology helpers get_level / last_wall (rootless_ops.c:1427,1444).
 *
 * Every rank appends JSON lines to a private buffer; rank 0 gathers and writes
 * them to the output file given on the command line.  Modes:
 *   topo   NMAX                 get_level/last_wall tables (rootless_ops.c:1427-1452)
 *   parents LEN                  one bcast per origin; receivers log parent (MPI_SOURCE)
 *   stream SEED K LEN            random-originator stream (rlo_testvec.h)
 *   iar    ORIGIN MASK           single proposal, decline iff rank in MASK (arg != NULL)
 *   multi  ACTIVE1 MOD AGREE     test_iar_multi_proposal roles (testcases.c:401-486), logging decisions
 *   tests                        the reference's own test wrappers' return values
 *   tests_safe                   the same, hacky-sack rounds run on every rank (see mode_tests_safe)
 *   tests2                       its two-engine IAR tests
 *   bench  K LEN                 storm throughput: every rank originates K bcasts
 *   lat    ROUNDS LEN SEED       unloaded latency: one random originator per round
 *   iarbench P                   every rank keeps one outstanding proposal, approve-all
 *   setupfail LEN, twice O D     drop-in only: engine setup failure, a second submission (see below)
 */
#include "rootless_ops.h"
#include "rlo_testvec.h"
#include <stdarg.h>
#include <stdint.h>

#ifndef RLO_DROPIN
int get_level(int world_size, int rank); /* rootless_ops.c:1427 */
int last_wall(int rank);                 /* rootless_ops.c:1444 */
#endif
int is_proposal_approved_cb(const void* buf, void* app_data); /* testcases.c:18 */
int proposal_action_cb(const void* buf, void* app_data);      /* testcases.c:39 */
int test_wrapper_bcast(int bc_cnt);                            /* testcases.c:699 */
int test_wrapper_hackysacking(int cnt_round, int cnt_msg);     /* testcases.c:726 */
int test_IAllReduce_single_proposal(MPI_Comm comm, int starter, int no_rank, int agree); /* :243 */
int test_iar_multi_proposal(MPI_Comm comm, int active_1, int active_2_mod, int agree);   /* :401 */

static char* g_out = NULL;
static size_t g_len = 0, g_cap = 0;
static int g_rank = 0, g_size = 1;

static void emit(const char* fmt, ...) {
    char tmp[8192];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(tmp, sizeof tmp, fmt, ap);
    va_end(ap);
    if (g_len + n + 2 > g_cap) {
        g_cap = (g_len + n + 2) * 2;
        g_out = realloc(g_out, g_cap);
    }
    memcpy(g_out + g_len, tmp, n);
    g_len += n;
    g_out[g_len++] = '\n';
}

static void gather_write(const char* path) {
    int len = (int)g_len;
    int* lens = NULL;
    int* displs = NULL;
    char* all = NULL;
    if (g_rank == 0) {
        lens = calloc(g_size, sizeof(int));
        displs = calloc(g_size, sizeof(int));
    }
    MPI_Gather(&len, 1, MPI_INT, lens, 1, MPI_INT, 0, MPI_COMM_WORLD);
    int total = 0;
    if (g_rank == 0) {
        for (int i = 0; i < g_size; i++) { displs[i] = total; total += lens[i]; }
        all = malloc(total + 1);
    }
    MPI_Gatherv(g_out, len, MPI_CHAR, all, lens, displs, MPI_CHAR, 0, MPI_COMM_WORLD);
    if (g_rank == 0) {
        FILE* f = fopen(path, "w");
        fwrite(all, 1, total, f);
        fclose(f);
        free(all); free(lens); free(displs);
    }
}

static void json_str(char* dst, size_t cap, const char* s, size_t maxlen) {
    size_t j = 0;
    for (size_t i = 0; i < maxlen && s[i] && j + 8 < cap; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c == '"' || c == '\\') { dst[j++] = '\\'; dst[j++] = c; }
        else if (c < 32 || c > 126) j += snprintf(dst + j, cap - j, "\\u%04x", c);
        else dst[j++] = c;
    }
    dst[j] = 0;
}

/* parent rank of a received message = MPI_SOURCE of its irecv (rootless_ops.h:115) */
#ifdef RLO_DROPIN
/* built against the MI355X drop-in (include/rootless_ops.h): the engine reports the tree
 * parent through its RLO_user_msg_source extension */
static int msg_parent(RLO_user_msg* u) { return RLO_user_msg_source(u); }
#else
static int msg_parent(RLO_user_msg* u) { return ((RLO_msg_t*)u)->irecv_stat.MPI_SOURCE; }
#endif

/* ---------------------------------------------------------------- topo */
#ifdef RLO_DROPIN
static void mode_topo(int nmax) { (void)nmax; } /* reference internals only */
#else
static void mode_topo(int nmax) {
    /* get_level(N, r) depends on N only for r == 0; last_wall(r) never depends on N */
    if (g_rank != 0) return;
    for (int n = 2; n <= nmax; n++) emit("{\"n\":%d,\"level0\":%d}", n, get_level(n, 0));
    for (int r = 1; r < nmax; r++)
        emit("{\"rank\":%d,\"level\":%d,\"last_wall_fn\":%d}", r, get_level(nmax, r), last_wall(r));
}

#endif

/* ---------------------------------------------------------------- parents */
static void mode_parents(int len) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    uint8_t* buf = calloc(1, len + 8);
    for (int o = 0; o < g_size; o++) {
        MPI_Barrier(MPI_COMM_WORLD);
        if (g_rank == o) {
            rlo_tv_payload(o, o, buf, len);
            RLO_msg_t* m = RLO_msg_new_bc(eng, buf, len);
            RLO_bcast_gen(eng, m, RLO_BCAST);
        } else {
            int got = 0;
            while (!got) {
                RLO_make_progress_all();
                RLO_user_msg* u = NULL;
                while (RLO_user_pickup_next(eng, &u)) {
                    uint64_t h = rlo_tv_region_hash((const uint8_t*)u->data, RLO_TV_DATA_REGION);
                    emit("{\"rank\":%d,\"origin\":%d,\"hdr_origin\":%d,\"parent\":%d,\"type\":%d,\"pid\":%d,\"vote\":%d,\"data_len\":%zu,\"hash\":\"%016llx\"}",
                         g_rank, o, *(int*)u->buf, msg_parent(u), u->type, u->pid, u->vote, u->data_len,
                         (unsigned long long)h);
                    RLO_user_msg_recycle(eng, u);
                    got++;
                }
            }
        }
        /* keep progressing until my own sends for this origin complete */
        for (int i = 0; i < 50; i++) RLO_make_progress_all();
    }
    MPI_Barrier(MPI_COMM_WORLD);
    RLO_progress_engine_cleanup(eng);
    free(buf);
}

/* ---------------------------------------------------------------- stream */
static void mode_stream(uint64_t seed, int K, int len) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    uint8_t* buf = calloc(1, len + 8);
    int mine = 0;
    for (int b = 0; b < K; b++) if ((int)rlo_tv_origin(seed, b, g_size) == g_rank) mine++;
    int expect = K - mine, got = 0, next_b = 0;
    MPI_Barrier(MPI_COMM_WORLD);
    while (got < expect || next_b < K) {
        /* originate the next bcast of mine, if any */
        while (next_b < K && (int)rlo_tv_origin(seed, next_b, g_size) != g_rank) next_b++;
        if (next_b < K) {
            rlo_tv_payload(g_rank, next_b, buf, len);
            RLO_msg_t* m = RLO_msg_new_bc(eng, buf, len);
            RLO_bcast_gen(eng, m, RLO_BCAST);
            next_b++;
        }
        RLO_make_progress_all();
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            uint64_t w0;
            memcpy(&w0, u->data, 8);
            uint64_t h = rlo_tv_region_hash((const uint8_t*)u->data, RLO_TV_DATA_REGION);
            emit("{\"rank\":%d,\"bid\":%u,\"origin\":%d,\"parent\":%d,\"type\":%d,\"hash\":\"%016llx\"}", g_rank,
                 (unsigned)(w0 >> 32), *(int*)u->buf, msg_parent(u), u->type, (unsigned long long)h);
            RLO_user_msg_recycle(eng, u);
            got++;
        }
    }
    RLO_progress_engine_cleanup(eng);
    free(buf);
}

/* ---------------------------------------------------------------- bulk stream (drop-in extension)
 * Mixed sizes lo..hi (rlo_tv_len), bcast b from rank b % N (every rank originates in every slot).
 * Bcasts longer than the reference's data region are the drop-in's bulk extension; they arrive with
 * data_len = their size (the reference cannot send them at all).  Per delivery: bid,
 * origin, tree parent, data_len and the FNV-1a of the delivered bytes (the data region for ring
 * bcasts, data_len bytes for bulk ones). */
static void mode_bulkstream(uint64_t seed, int K, int lo, int hi) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    uint8_t* buf = calloc(1, (size_t)hi + 8);
    int mine = 0;
    for (int b = 0; b < K; b++) if (b % g_size == g_rank) mine++;
    int expect = K - mine, got = 0, next_b = g_rank;
    MPI_Barrier(MPI_COMM_WORLD);
    while (got < expect || next_b < K) {
        if (next_b < K) {
            int len = (int)rlo_tv_len(seed, (uint64_t)next_b, (uint32_t)lo, (uint32_t)hi);
            rlo_tv_payload(g_rank, next_b, buf, len);
            RLO_msg_t* m = RLO_msg_new_bc(eng, buf, len);
            if (!m || RLO_bcast_gen(eng, m, RLO_BCAST) != 0) { fprintf(stderr, "bulkstream: send failed\n"); break; }
            next_b += g_size;
        }
        RLO_make_progress_all();
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            uint64_t w0;
            memcpy(&w0, u->data, 8);
            size_t n = u->data_len ? u->data_len : RLO_TV_DATA_REGION;
            uint64_t h = rlo_tv_fnv1a((const uint8_t*)u->data, n, RLO_TV_FNV_INIT);
            emit("{\"rank\":%d,\"bid\":%u,\"origin\":%d,\"parent\":%d,\"type\":%d,\"len\":%zu,\"hash\":\"%016llx\"}",
                 g_rank, (unsigned)(w0 >> 32), *(int*)u->buf, msg_parent(u), u->type, (size_t)u->data_len,
                 (unsigned long long)h);
            RLO_user_msg_recycle(eng, u);
            got++;
        }
    }
    RLO_progress_engine_cleanup(eng);
    free(buf);
}

/* ---------------------------------------------------------------- iar */
typedef struct { unsigned mask; int rank; } MaskCtx;

static int judge_mask_cb(const void* arg, void* ctx) {
    MaskCtx* c = (MaskCtx*)ctx;
    char s[256];
    if (arg) json_str(s, sizeof s, (const char*)arg, 64); else s[0] = 0;
    emit("{\"ev\":\"judge\",\"rank\":%d,\"null\":%d,\"arg\":\"%s\"}", c->rank, arg == NULL, s);
    if (arg && ((c->mask >> c->rank) & 1u)) return 0;
    return 1;
}

static int action_log_cb(const void* buf, void* ctx) {
    MaskCtx* c = (MaskCtx*)ctx;
    const char* b = (const char*)buf;
    int pid, vote;
    size_t dl;
    memcpy(&pid, b, 4);
    memcpy(&vote, b + 4, 4);
    memcpy(&dl, b + 8, 8);
    char s[256];
    json_str(s, sizeof s, b + 16, dl < 64 ? dl : 64);
    emit("{\"ev\":\"action\",\"rank\":%d,\"pid\":%d,\"vote\":%d,\"data_len\":%zu,\"data\":\"%s\"}", c->rank, pid, vote, dl, s);
    return 0;
}

static void mode_iar(int origin, unsigned mask) {
    MaskCtx ctx = {mask, g_rank};
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &judge_mask_cb, &ctx, &action_log_cb);
    char prop[64];
    snprintf(prop, sizeof prop, "proposal-from-%d", origin);
    MPI_Barrier(MPI_COMM_WORLD);
    if (g_rank == origin) {
        int ret = RLO_submit_proposal(eng, prop, strlen(prop), 100 + origin);
        int result;
        if (ret > -1) result = RLO_get_vote_my_proposal(eng);
        else {
            while (RLO_check_proposal_state(eng, 0) != RLO_COMPLETED) RLO_make_progress_all();
            result = RLO_get_vote_my_proposal(eng);
        }
        emit("{\"ev\":\"result\",\"rank\":%d,\"pid\":%d,\"vote\":%d}", g_rank, 100 + origin, result);
    } else {
        int done = 0;
        while (!done) {
            RLO_make_progress_all();
            RLO_user_msg* u = NULL;
            while (RLO_user_pickup_next(eng, &u)) {
                char s[64];
                json_str(s, sizeof s, u->data, u->data_len < 32 ? u->data_len : 32);
                emit("{\"ev\":\"pickup\",\"rank\":%d,\"type\":%d,\"pid\":%d,\"vote\":%d,\"data_len\":%zu,\"data\":\"%s\",\"origin\":%d}",
                     g_rank, u->type, u->pid, u->vote, u->data_len, s, *(int*)u->buf);
                if (u->type == RLO_IAR_DECISION) done = 1;
                RLO_user_msg_recycle(eng, u);
            }
        }
    }
    RLO_progress_engine_cleanup(eng);
}

#ifdef RLO_HAVE_PROPOSAL_POOL
/* the proposal pool (drop-in extension; the reference keeps one own proposal, rootless_ops.c:241):
 * every rank submits `per` proposals (pid 1000 + i * N + rank, data "p<i>-r<rank>") keeping up to
 * RLO_proposal_pool_depth in flight; judge = the decline mask (judge_mask_cb logs every call) */
static void mode_pool(int per, unsigned mask) {
    MaskCtx ctx = {mask, g_rank};
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &judge_mask_cb, &ctx, &action_log_cb);
    const int depth = RLO_proposal_pool_depth(eng);
    int fl[16], nfl = 0, sub = 0, done = 0;
    long got = 0, expect = (long)per * (g_size - 1);
    MPI_Barrier(MPI_COMM_WORLD);
    while (done < per || got < expect) {
        while (nfl < depth && sub < per) {
            char prop[64];
            snprintf(prop, sizeof prop, "p%d-r%d", sub, g_rank);
            const int pid = 1000 + sub * g_size + g_rank;
            RLO_submit_proposal(eng, prop, strlen(prop), pid);
            fl[nfl++] = pid;
            sub++;
        }
        RLO_make_progress_all();
        for (int i = 0; i < nfl;) {
            if (RLO_check_proposal_state(eng, fl[i]) != RLO_COMPLETED) { i++; continue; }
            emit("{\"ev\":\"result\",\"rank\":%d,\"pid\":%d,\"vote\":%d}", g_rank, fl[i], RLO_get_vote_proposal(eng, fl[i]));
            done++;
            fl[i] = fl[--nfl];
        }
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            if (u->type == RLO_IAR_DECISION) {
                emit("{\"ev\":\"decision\",\"rank\":%d,\"pid\":%d,\"vote\":%d,\"origin\":%d}", g_rank, u->pid, u->vote,
                     *(int*)u->buf);
                got++;
            }
            RLO_user_msg_recycle(eng, u);
        }
    }
    emit("{\"ev\":\"depth\",\"rank\":%d,\"depth\":%d}", g_rank, depth);
    RLO_progress_engine_cleanup(eng);
}
#endif

#ifdef RLO_DROPIN
/* drop-in robustness (no reference counterpart).
 * setupfail LEN: the first engine's setup fails after its kernels were launched (RLO_FAULT_ATTACH names
 * the rank whose attach fails): every rank must get NULL back, promptly (the leaders stop their kernels);
 * then the process builds a second engine and runs mode_parents on it. */
static void mode_parents(int len);
int rlo_dropin_test_fault(int what, int rank); /* librootless_ops.so test hook (not in rootless_ops.h) */
static void mode_setupfail(int len) {
    const char* fa = getenv("RLO_FAULT_ATTACH");
    if (fa) rlo_dropin_test_fault(1, atoi(fa));
    RLO_engine_t* e = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    emit("{\"ev\":\"first\",\"rank\":%d,\"ok\":%d}", g_rank, e != NULL);
    if (e) RLO_progress_engine_cleanup(e);
    rlo_dropin_test_fault(1, -1);
    MPI_Barrier(MPI_COMM_WORLD);
    mode_parents(len);
}

/* twice ORIGIN DECLINER: with one own proposal per engine (no pool), ORIGIN submits "first" and, before
 * it is decided, "second", which DECLINER declines.  my_own_proposal is then the second one
 * (rootless_ops.c:878-883, votes count only for its pid, :756): the result ORIGIN reads must be the
 * second proposal's (0), never the first's (1). */
static int judge_second_cb(const void* arg, void* ctx) {
    MaskCtx* c = (MaskCtx*)ctx;
    return (arg && !strcmp((const char*)arg, "second") && ((c->mask >> c->rank) & 1u)) ? 0 : 1;
}
static void mode_twice(int origin, int decliner) {
    MaskCtx ctx = {1u << decliner, g_rank};
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &judge_second_cb, &ctx, NULL);
    MPI_Barrier(MPI_COMM_WORLD);
    if (g_rank == origin) {
        RLO_submit_proposal(eng, "first", 5, 501);
        RLO_submit_proposal(eng, "second", 6, 502);
        while (RLO_check_proposal_state(eng, 502) != RLO_COMPLETED) RLO_make_progress_all();
        emit("{\"ev\":\"result\",\"rank\":%d,\"vote\":%d}", g_rank, RLO_get_vote_my_proposal(eng));
    } else {
        int done = 0;
        while (!done) {
            RLO_make_progress_all();
            RLO_user_msg* u = NULL;
            while (RLO_user_pickup_next(eng, &u)) {
                if (u->type == RLO_IAR_DECISION) {
                    emit("{\"ev\":\"decision\",\"rank\":%d,\"pid\":%d,\"vote\":%d}", g_rank, u->pid, u->vote);
                    if (u->pid == 502) done = 1;
                }
                RLO_user_msg_recycle(eng, u);
            }
        }
    }
    RLO_progress_engine_cleanup(eng);
}
#endif

/* ---------------------------------------------------------------- multi */
static int judge_isp_log_cb(const void* arg, void* ctx) {
    int r = is_proposal_approved_cb(arg, ctx);
    char s[64];
    if (arg) json_str(s, sizeof s, (const char*)arg, 16); else s[0] = 0;
    emit("{\"ev\":\"judge\",\"rank\":%d,\"null\":%d,\"arg\":\"%s\",\"ret\":%d}", g_rank, arg == NULL, s, r);
    return r;
}

static void mode_multi(int active_1, int mod, int agree) {
    ISP isp;
    isp.my_proposal = NULL;
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &judge_isp_log_cb, &isp, &proposal_action_cb);
    int decision_needed = 1 + (g_size - 1) / mod + 1; /* testcases.c:414 */
    int proposer = 0;
    MPI_Barrier(MPI_COMM_WORLD);
    if (g_rank == active_1) { isp.my_proposal = "555"; proposer = 1; }
    else if (g_rank % mod == 0) { isp.my_proposal = agree ? "555" : "333"; proposer = 1; }
    else isp.my_proposal = agree ? "555" : "111";
    int result = -1, own_done = !proposer, got = 0;
    int need = proposer ? decision_needed - 1 : decision_needed;
    if (proposer) {
        int ret = RLO_submit_proposal(eng, isp.my_proposal, strlen(isp.my_proposal), g_rank);
        if (ret > -1) { result = RLO_get_vote_my_proposal(eng); own_done = 1; }
    }
    while (!own_done || got < need) {
        RLO_make_progress_all();
        if (!own_done && RLO_check_proposal_state(eng, 0) == RLO_COMPLETED) {
            result = RLO_get_vote_my_proposal(eng);
            own_done = 1;
        }
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            if (u->type == RLO_IAR_DECISION) {
                emit("{\"ev\":\"decision\",\"rank\":%d,\"pid\":%d,\"vote\":%d,\"origin\":%d}", g_rank, u->pid, u->vote, *(int*)u->buf);
                got++;
            }
            RLO_user_msg_recycle(eng, u);
        }
    }
    if (proposer) emit("{\"ev\":\"result\",\"rank\":%d,\"pid\":%d,\"vote\":%d}", g_rank, g_rank, result);
    RLO_progress_engine_cleanup(eng);
}

#ifdef RLO_HAVE_DEVICE_JUDGE
/* the multi-proposal roles of mode_multi with is_proposal_approved_cb registered on the device
 * (RLO_progress_engine_new_dj, RLO_DJUDGE_ISP): decisions and results must equal the reference's */
static void mode_multi_dj(int active_1, int mod, int agree) {
    const char* mine;
    int proposer = 0;
    if (g_rank == active_1) { mine = "555"; proposer = 1; }
    else if (g_rank % mod == 0) { mine = agree ? "555" : "333"; proposer = 1; }
    else mine = agree ? "555" : "111";
    RLO_device_judge j = {RLO_DJUDGE_ISP, mine, 0, 0};
    RLO_engine_t* eng = RLO_progress_engine_new_dj(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &j, NULL, &proposal_action_cb);
    int decision_needed = 1 + (g_size - 1) / mod + 1; /* testcases.c:414 */
    MPI_Barrier(MPI_COMM_WORLD);
    int result = -1, own_done = !proposer, got = 0;
    int need = proposer ? decision_needed - 1 : decision_needed;
    if (proposer) {
        int ret = RLO_submit_proposal(eng, (char*)mine, strlen(mine), g_rank);
        if (ret > -1) { result = RLO_get_vote_my_proposal(eng); own_done = 1; }
    }
    while (!own_done || got < need) {
        RLO_make_progress_all();
        if (!own_done && RLO_check_proposal_state(eng, 0) == RLO_COMPLETED) {
            result = RLO_get_vote_my_proposal(eng);
            own_done = 1;
        }
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            if (u->type == RLO_IAR_DECISION) {
                emit("{\"ev\":\"decision\",\"rank\":%d,\"pid\":%d,\"vote\":%d,\"origin\":%d}", g_rank, u->pid, u->vote, *(int*)u->buf);
                got++;
            }
            RLO_user_msg_recycle(eng, u);
        }
    }
    if (proposer) emit("{\"ev\":\"result\",\"rank\":%d,\"pid\":%d,\"vote\":%d}", g_rank, g_rank, result);
    RLO_progress_engine_cleanup(eng);
}
#endif

/* ---------------------------------------------------------------- tests */
static void mode_tests(void) {
    int r;
    r = test_wrapper_bcast(2);
    if (g_rank == 0) emit("{\"test\":\"test_wrapper_bcast(2)\",\"ret\":%d}", r);
    r = test_wrapper_hackysacking(3, 100);
    if (g_rank == 0) emit("{\"test\":\"test_wrapper_hackysacking(3,100)\",\"ret\":%d}", r);
    r = test_IAllReduce_single_proposal(MPI_COMM_WORLD, 1, 2, 0);
    if (g_rank == 0) emit("{\"test\":\"test_IAllReduce_single_proposal(1,2,0)\",\"ret\":%d}", r);
    r = test_IAllReduce_single_proposal(MPI_COMM_WORLD, 1, 2, 1);
    if (g_rank == 0) emit("{\"test\":\"test_IAllReduce_single_proposal(1,2,1)\",\"ret\":%d}", r);
    r = test_iar_multi_proposal(MPI_COMM_WORLD, 1, 3, 1);
    if (g_rank == 0) emit("{\"test\":\"test_iar_multi_proposal(1,3,1)\",\"ret\":%d}", r);
}

/* test_wrapper_hackysacking (testcases.c:726-740) stops a rank at its first failed round.  The
 * pass flag of a round is message timing (a send inside RLO_bcast_gen's progress call can surface
 * the next ball inside the same pickup loop, testcases.c:670-683 + rootless_ops.c:1602), and a
 * rank that fails while its peers pass leaves them waiting in the next round's collective engine
 * creation.  "tests_safe" runs every round on every rank (same hacky_sack_progress_engine, same
 * result aggregation) so a timing-dependent flag can be checked instead of hanging. */
int hacky_sack_progress_engine(MPI_Comm comm, int msg_cnt);                    /* testcases.c:638 */
int aggregate_test_result(MPI_Comm comm, int test_passed, char* test_name);  /* testcases.c:615 */

static int hackysacking_all_rounds(int cnt_round, int cnt_msg) {
    MPI_Comm comm;
    MPI_Comm_dup(MPI_COMM_WORLD, &comm);
    int failed = 0;
    for (int i = 0; i < cnt_round; i++)
        if (hacky_sack_progress_engine(comm, cnt_msg) != 1) failed++;
    return aggregate_test_result(comm, failed == 0, "Hackysack");
}

static void mode_tests_safe(void) {
    int r;
    r = test_wrapper_bcast(2);
    if (g_rank == 0) emit("{\"test\":\"test_wrapper_bcast(2)\",\"ret\":%d}", r);
    r = hackysacking_all_rounds(3, 100);
    if (g_rank == 0) emit("{\"test\":\"test_wrapper_hackysacking(3,100)\",\"ret\":%d}", r);
    r = test_IAllReduce_single_proposal(MPI_COMM_WORLD, 1, 2, 0);
    if (g_rank == 0) emit("{\"test\":\"test_IAllReduce_single_proposal(1,2,0)\",\"ret\":%d}", r);
    r = test_IAllReduce_single_proposal(MPI_COMM_WORLD, 1, 2, 1);
    if (g_rank == 0) emit("{\"test\":\"test_IAllReduce_single_proposal(1,2,1)\",\"ret\":%d}", r);
    r = test_iar_multi_proposal(MPI_COMM_WORLD, 1, 3, 1);
    if (g_rank == 0) emit("{\"test\":\"test_iar_multi_proposal(1,3,1)\",\"ret\":%d}", r);
}

/* the reference's two-engine tests (testcases.c:110-241, :488-595) */
int test_concurrent_iar_single_proposal(MPI_Comm comm, int starter, int no_rank, int agree);
int test_concurrent_iar_multi_proposal(MPI_Comm comm, int active_1, int active_2_mod, int agree);

static void mode_tests2(void) {
    int r;
    r = test_concurrent_iar_single_proposal(MPI_COMM_WORLD, 1, 2, 0);
    if (g_rank == 0) emit("{\"test\":\"test_concurrent_iar_single_proposal(1,2,0)\",\"ret\":%d}", r);
    r = test_concurrent_iar_single_proposal(MPI_COMM_WORLD, 1, 2, 1);
    if (g_rank == 0) emit("{\"test\":\"test_concurrent_iar_single_proposal(1,2,1)\",\"ret\":%d}", r);
    r = test_concurrent_iar_multi_proposal(MPI_COMM_WORLD, 1, 3, 1);
    if (g_rank == 0) emit("{\"test\":\"test_concurrent_iar_multi_proposal(1,3,1)\",\"ret\":%d}", r);
    r = test_concurrent_iar_multi_proposal(MPI_COMM_WORLD, 1, 3, 0);
    if (g_rank == 0) emit("{\"test\":\"test_concurrent_iar_multi_proposal(1,3,0)\",\"ret\":%d}", r);
}

/* ---------------------------------------------------------------- bench */
static double now_s(void) { struct timeval tv; gettimeofday(&tv, NULL); return tv.tv_sec + tv.tv_usec * 1e-6; }

static void mode_bench(int K, int len) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    uint8_t* buf = calloc(1, len + 8);
    int expect = K * (g_size - 1), got = 0, sent = 0;
    long bad = 0;
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = now_s();
    while (got < expect || sent < K) {
        if (sent < K) {
            rlo_tv_payload(g_rank, sent, buf, len);
            RLO_bcast_gen(eng, RLO_msg_new_bc(eng, buf, len), RLO_BCAST);
            sent++;
        }
        RLO_make_progress_all();
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            uint64_t w0;
            memcpy(&w0, u->data, 8);
            uint64_t w1 = rlo_tv_word((uint32_t)w0, (uint32_t)(w0 >> 32), 1);
            if (len >= 16 && memcmp(&w1, u->data + 8, 8) != 0) bad++;
            RLO_user_msg_recycle(eng, u);
            got++;
        }
    }
    double t1 = now_s(), dt = t1 - t0, dtmax;
    MPI_Reduce(&dt, &dtmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    long badsum;
    MPI_Reduce(&bad, &badsum, 1, MPI_LONG, MPI_SUM, 0, MPI_COMM_WORLD);
    if (g_rank == 0)
        emit("{\"mode\":\"bench\",\"ranks\":%d,\"K\":%d,\"len\":%d,\"seconds\":%.6f,\"bcast_per_s\":%.1f,\"deliveries_per_s\":%.1f,\"bad\":%ld}",
             g_size, K, len, dtmax, g_size * (double)K / dtmax, g_size * (double)K * (g_size - 1) / dtmax, badsum);
    RLO_progress_engine_cleanup(eng);
    free(buf);
}

static int cmp_d(const void* a, const void* b) { double x = *(const double*)a, y = *(const double*)b; return (x > y) - (x < y); }

static void mode_lat(int rounds, int len, uint64_t seed) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    uint8_t* buf = calloc(1, len + 16);
    double* lat = calloc(rounds, sizeof(double));
    for (int i = 0; i < rounds; i++) {
        int o = (int)rlo_tv_origin(seed, i, g_size);
        MPI_Barrier(MPI_COMM_WORLD);
        double t_send = 0, t_recv = 0;
        if (g_rank == o) {
            rlo_tv_payload(o, i, buf, len);
            t_send = now_s();
            RLO_bcast_gen(eng, RLO_msg_new_bc(eng, buf, len), RLO_BCAST);
        } else {
            int got = 0;
            while (!got) {
                RLO_make_progress_all();
                RLO_user_msg* u = NULL;
                while (RLO_user_pickup_next(eng, &u)) { t_recv = now_s(); RLO_user_msg_recycle(eng, u); got = 1; }
            }
        }
        double ts, tr;
        MPI_Allreduce(&t_send, &ts, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        MPI_Allreduce(&t_recv, &tr, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        lat[i] = (tr - ts) * 1e6;
        for (int k = 0; k < 20; k++) RLO_make_progress_all();
    }
    if (g_rank == 0) {
        qsort(lat, rounds, sizeof(double), cmp_d);
        emit("{\"mode\":\"lat\",\"ranks\":%d,\"rounds\":%d,\"len\":%d,\"p50_us\":%.2f,\"p99_us\":%.2f}", g_size, rounds, len,
             lat[rounds / 2], lat[(int)(rounds * 0.99)]);
    }
    MPI_Barrier(MPI_COMM_WORLD);
    RLO_progress_engine_cleanup(eng);
    free(buf); free(lat);
}

static int approve_all_cb(const void* a, void* c) { (void)a; (void)c; return 1; }
static int noop_action_cb(const void* a, void* c) { (void)a; (void)c; return 0; }

static void mode_iarbench(int P) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &approve_all_cb, NULL, &noop_action_cb);
    char prop[16] = "0123456789abcdef";
    int expect = P * (g_size - 1), got = 0, done = 0, inflight = 0;
    long approved = 0;
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = now_s();
    while (got < expect || done < P) {
        if (!inflight && done < P) {
            int ret = RLO_submit_proposal(eng, prop, 16, done * g_size + g_rank);
            inflight = 1;
            if (ret > -1) { approved += RLO_get_vote_my_proposal(eng); inflight = 0; done++; }
        }
        RLO_make_progress_all();
        if (inflight && RLO_check_proposal_state(eng, 0) == RLO_COMPLETED) {
            approved += RLO_get_vote_my_proposal(eng);
            inflight = 0;
            done++;
        }
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            if (u->type == RLO_IAR_DECISION) got++;
            RLO_user_msg_recycle(eng, u);
        }
    }
    double dt = now_s() - t0, dtmax;
    MPI_Reduce(&dt, &dtmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    long app;
    MPI_Reduce(&approved, &app, 1, MPI_LONG, MPI_SUM, 0, MPI_COMM_WORLD);
    if (g_rank == 0)
        emit("{\"mode\":\"iarbench\",\"ranks\":%d,\"P\":%d,\"seconds\":%.6f,\"decisions_per_s\":%.1f,\"approved\":%ld}", g_size, P,
             dtmax, g_size * (double)P / dtmax, app);
    RLO_progress_engine_cleanup(eng);
}

int main(int argc, char** argv) {
    setvbuf(stdout, NULL, _IOLBF, 0); /* progress lines survive a kill */
    MPI_Init(&argc, &argv);
    MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
    MPI_Comm_size(MPI_COMM_WORLD, &g_size);
    if (argc < 3) {
        if (g_rank == 0) fprintf(stderr, "usage: ref_harness OUT MODE args...\n");
        MPI_Finalize();
        return 2;
    }
    const char* out = argv[1];
    const char* mode = argv[2];
    /* reference prints engine new/cleanup lines on stdout; keep them off our files */
    if (!strcmp(mode, "topo")) mode_topo(atoi(argv[3]));
    else if (!strcmp(mode, "parents")) mode_parents(atoi(argv[3]));
    else if (!strcmp(mode, "stream")) mode_stream(strtoull(argv[3], 0, 0), atoi(argv[4]), atoi(argv[5]));
    else if (!strcmp(mode, "bulkstream")) mode_bulkstream(strtoull(argv[3], 0, 0), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]));
    else if (!strcmp(mode, "iar")) mode_iar(atoi(argv[3]), (unsigned)strtoul(argv[4], 0, 0));
    else if (!strcmp(mode, "multi")) mode_multi(atoi(argv[3]), atoi(argv[4]), atoi(argv[5]));
#ifdef RLO_HAVE_DEVICE_JUDGE
    else if (!strcmp(mode, "multi_dj")) mode_multi_dj(atoi(argv[3]), atoi(argv[4]), atoi(argv[5]));
#endif
#ifdef RLO_HAVE_PROPOSAL_POOL
    else if (!strcmp(mode, "pool")) mode_pool(atoi(argv[3]), (unsigned)strtoul(argv[4], 0, 0));
#endif
#ifdef RLO_DROPIN
    else if (!strcmp(mode, "setupfail")) mode_setupfail(atoi(argv[3]));
    else if (!strcmp(mode, "twice")) mode_twice(atoi(argv[3]), atoi(argv[4]));
#endif
    else if (!strcmp(mode, "tests")) mode_tests();
    else if (!strcmp(mode, "tests_safe")) mode_tests_safe();
    else if (!strcmp(mode, "tests2")) mode_tests2();
    else if (!strcmp(mode, "bench")) mode_bench(atoi(argv[3]), atoi(argv[4]));
    else if (!strcmp(mode, "lat")) mode_lat(atoi(argv[3]), atoi(argv[4]), strtoull(argv[5], 0, 0));
    else if (!strcmp(mode, "iarbench")) mode_iarbench(atoi(argv[3]));
    gather_write(out);
    MPI_Finalize();
    return 0;
}
