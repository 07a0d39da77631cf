/*
 * api_bench.c -- throughput / latency of the rootless_ops.h API under host MPI, one rank per
 * process.  The same source is linked twice:
 *   rootless-coll-mpi-ops_amd/lib/rlo_api_bench  against librootless_ops.so (MI355X drop-in)
 *   oracle/_ref/ref_api_bench                    against the compiled reference (CPU baseline)
 * so bench.py compares the two through identical calls (testcases.c:59-108 / :638-697 style).
 *
 *   mpiexec -n N api_bench storm K LEN      every rank originates K bcasts of LEN bytes,
 *                                           progress + pickup until all (N-1)K arrived
 *   mpiexec -n N api_bench lat ROUNDS LEN   one random originator per round, barrier between
 *   mpiexec -n N api_bench iar P            every rank keeps one proposal outstanding, P each
 *   RLO_PROPOSAL_POOL=d mpiexec -n N api_bench iarpool P   d in flight per rank (extension)
 * Rank 0 prints one JSON line.  Payload bytes are checked at every receiver.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <unistd.h>

#include "rootless_ops.h"

static int g_rank, g_size;
static FILE* g_out; /* results; stdout goes to /dev/null (the reference prints setup lines there) */

static double now_s(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return tv.tv_sec + tv.tv_usec * 1e-6;
}

/* payload of bcast (origin, seq): [origin i32][seq i32] then an LCG byte stream */
static void fill(uint8_t* b, int origin, int seq, int len) {
    uint32_t x = (uint32_t)origin * 2654435761u + (uint32_t)seq * 40503u + 1u;
    for (int i = 0; i < len; i++) {
        x = x * 1103515245u + 12345u;
        b[i] = (uint8_t)(x >> 16);
    }
    if (len >= 8) {
        memcpy(b, &origin, 4);
        memcpy(b + 4, &seq, 4);
    }
}

static long check(const RLO_user_msg* u, int len, uint8_t* tmp) {
    int origin = *(const int*)u->buf, seq = 0;
    if (len < 8) return 0;
    memcpy(&seq, u->data + 4, 4);
    fill(tmp, origin, seq, len);
    return memcmp(tmp, u->data, (size_t)len) != 0;
}

static void storm(int K, int len) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    uint8_t* buf = calloc(1, (size_t)len + 16);
    uint8_t* tmp = calloc(1, (size_t)len + 16);
    long expect = (long)K * (g_size - 1), got = 0, bad = 0;
    int sent = 0;
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = now_s(), t_last = t0;
    while (got < expect || sent < K) {
        for (int b = 0; b < 8 && sent < K; b++, sent++) {
            fill(buf, g_rank, sent, len);
            RLO_bcast_gen(eng, RLO_msg_new_bc(eng, buf, len), RLO_BCAST);
        }
        RLO_make_progress_all();
        RLO_user_msg* u = NULL;
        long before = got;
        while (RLO_user_pickup_next(eng, &u)) {
            bad += check(u, len, tmp);
            got++;
            RLO_user_msg_recycle(eng, u);
        }
        if (got != before) t_last = now_s();
        else if (now_s() - t_last > 5.0) { /* watchdog: say where a stalled run stands */
            fprintf(stderr, "api_bench rank %d: stalled, sent %d/%d, got %ld/%ld\n", g_rank, sent, K, got, expect);
            t_last = now_s();
        }
    }
    double dt = now_s() - t0, dtmax = 0;
    long badall = 0;
    MPI_Reduce(&dt, &dtmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    MPI_Reduce(&bad, &badall, 1, MPI_LONG, MPI_SUM, 0, MPI_COMM_WORLD);
    if (g_rank == 0)
        fprintf(g_out, "{\"mode\":\"storm\",\"ranks\":%d,\"K\":%d,\"len\":%d,\"seconds\":%.6f,\"bcast_per_s\":%.1f,"
               "\"deliveries_per_s\":%.1f,\"bad\":%ld}\n",
               g_size, K, len, dtmax, g_size * (double)K / dtmax, g_size * (double)K * (g_size - 1) / dtmax, badall);
    RLO_progress_engine_cleanup(eng);
    free(buf);
    free(tmp);
}

static int cmp_d(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

static void lat(int rounds, int len) {
    RLO_engine_t* eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, NULL, NULL, NULL);
    uint8_t* buf = calloc(1, (size_t)len + 16);
    double* l = calloc((size_t)rounds, sizeof(double));
    uint64_t x = 0x5EEDull;
    for (int i = 0; i < rounds; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        int o = (int)((x >> 33) % (uint64_t)g_size);
        MPI_Barrier(MPI_COMM_WORLD);
        double ts = 0, tr = 0;
        if (g_rank == o) {
            fill(buf, o, i, len);
            ts = now_s();
            RLO_bcast_gen(eng, RLO_msg_new_bc(eng, buf, len), RLO_BCAST);
        } else {
            int got = 0;
            while (!got) {
                RLO_make_progress_all();
                RLO_user_msg* u = NULL;
                while (RLO_user_pickup_next(eng, &u)) {
                    tr = now_s();
                    RLO_user_msg_recycle(eng, u);
                    got = 1;
                }
            }
        }
        double a, b;  /* one wall clock: every rank runs on the same host */
        MPI_Allreduce(&ts, &a, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        MPI_Allreduce(&tr, &b, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        l[i] = (b - a) * 1e6;
        for (int k = 0; k < 4; k++) RLO_make_progress_all();
    }
    if (g_rank == 0) {
        qsort(l, (size_t)rounds, sizeof(double), cmp_d);
        fprintf(g_out, "{\"mode\":\"lat\",\"ranks\":%d,\"rounds\":%d,\"len\":%d,\"p50_us\":%.2f,\"p99_us\":%.2f}\n", g_size, rounds,
               len, l[rounds / 2], l[(int)(rounds * 0.99)]);
    }
    MPI_Barrier(MPI_COMM_WORLD);
    RLO_progress_engine_cleanup(eng);
    free(buf);
    free(l);
}

/* API_DIAG=1: per-rank loop-gap / round-latency / context-switch counts on stderr (is a slow run
 * the host descheduling us, or the engine?) */
static long ctx_switches(const char* key) {
    FILE* f = fopen("/proc/self/status", "r");
    char line[256];
    long v = -1;
    size_t kl = strlen(key);
    if (!f) return -1;
    while (fgets(line, sizeof line, f))
        if (!strncmp(line, key, kl)) v = atol(line + kl + 1);
    fclose(f);
    return v;
}

static int approve_cb(const void* a, void* c) {
    (void)a;
    (void)c;
    return 1;
}
static int action_cb(const void* a, void* c) {
    (void)a;
    (void)c;
    return 0;
}

/* dj: the approve-all judge registered on the device (RLO_progress_engine_new_dj, an extension of
 * this library; the reference has no such call) */
static void iar(int P, int dj) {
    RLO_engine_t* eng = NULL;
#ifdef RLO_HAVE_DEVICE_JUDGE
    if (dj) {
        RLO_device_judge j = {RLO_DJUDGE_APPROVE, NULL, 0, 0};
        eng = RLO_progress_engine_new_dj(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &j, NULL, &action_cb);
    } else
#endif
        eng = RLO_progress_engine_new(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &approve_cb, NULL, &action_cb);
    if (!eng) {
        if (g_rank == 0) fprintf(g_out, "{\"mode\":\"%s\",\"error\":\"no engine\"}\n", dj ? "iardj" : "iar");
        return;
    }
    char prop[17] = "0123456789abcdef";
    long expect = (long)P * (g_size - 1), got = 0, approved = 0;
    int done = 0, inflight = 0;
    const int diag = getenv("API_DIAG") != NULL;
    double* rl = diag ? calloc((size_t)P + 1, sizeof(double)) : NULL;
    double gap_max = 0, t_prev = 0, t_sub = 0, t_mine = 0;
    long gaps_1ms = 0, nvcs0 = diag ? ctx_switches("nonvoluntary_ctxt_switches") : 0;
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = now_s();
    t_prev = t0;
    while (got < expect || done < P) {
        if (diag) {
            double tn = now_s();
            if (tn - t_prev > gap_max) gap_max = tn - t_prev;
            if (tn - t_prev > 1e-3) gaps_1ms++;
            t_prev = tn;
        }
        if (!inflight && done < P) {
            if (diag) t_sub = now_s();
            int ret = RLO_submit_proposal(eng, prop, 16, done * g_size + g_rank);
            inflight = 1;
            if (ret > -1) {
                approved += RLO_get_vote_my_proposal(eng);
                inflight = 0;
                if (diag) rl[done] = now_s() - t_sub;
                done++;
            }
        }
        RLO_make_progress_all();
        if (inflight && RLO_check_proposal_state(eng, 0) == RLO_COMPLETED) {
            approved += RLO_get_vote_my_proposal(eng);
            inflight = 0;
            if (diag) rl[done] = now_s() - t_sub;
            done++;
            if (diag && done == P) t_mine = now_s() - t0;
        }
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            if (u->type == RLO_IAR_DECISION) got++;
            RLO_user_msg_recycle(eng, u);
        }
    }
    double dt = now_s() - t0, dtmax = 0;
    long app = 0;
    if (diag) {
        qsort(rl, (size_t)P, sizeof(double), cmp_d);
        fprintf(stderr, "diag rank %d: own %.3f s all %.3f s; round us p50 %.1f p99 %.1f max %.1f; loop gap max %.1f us, >1ms %ld; "
                "nonvoluntary ctx %ld\n", g_rank, t_mine, dt, rl[P / 2] * 1e6, rl[(int)(P * 0.99)] * 1e6, rl[P - 1] * 1e6,
                gap_max * 1e6, gaps_1ms, ctx_switches("nonvoluntary_ctxt_switches") - nvcs0);
        free(rl);
    }
    MPI_Reduce(&dt, &dtmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    MPI_Reduce(&approved, &app, 1, MPI_LONG, MPI_SUM, 0, MPI_COMM_WORLD);
    if (g_rank == 0)
        fprintf(g_out, "{\"mode\":\"%s\",\"ranks\":%d,\"P\":%d,\"seconds\":%.6f,\"decisions_per_s\":%.1f,\"approved\":%ld}\n",
               dj ? "iardj" : "iar", g_size, P, dtmax, g_size * (double)P / dtmax, app);
    RLO_progress_engine_cleanup(eng);
}

#ifdef RLO_HAVE_PROPOSAL_POOL
/* the proposal pool (extension; RLO_PROPOSAL_POOL=d at engine creation): every rank keeps d of its
 * P proposals in flight, device judge approving all (the reference allows one, rootless_ops.c:241) */
static void iarpool(int P) {
    RLO_device_judge j = {RLO_DJUDGE_APPROVE, NULL, 0, 0};
    RLO_engine_t* eng = RLO_progress_engine_new_dj(MPI_COMM_WORLD, RLO_MSG_SIZE_MAX, &j, NULL, &action_cb);
    if (!eng) {
        if (g_rank == 0) fprintf(g_out, "{\"mode\":\"iarpool\",\"error\":\"no engine\"}\n");
        return;
    }
    const int D = RLO_proposal_pool_depth(eng);
    char prop[17] = "0123456789abcdef";
    long expect = (long)P * (g_size - 1), got = 0, approved = 0;
    int sub = 0, done = 0, fl[16], nfl = 0;
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = now_s();
    while (got < expect || done < P) {
        while (nfl < D && sub < P) {
            const int pid = sub * g_size + g_rank;
            RLO_submit_proposal(eng, prop, 16, pid);
            fl[nfl++] = pid;
            sub++;
        }
        RLO_make_progress_all();
        for (int i = 0; i < nfl;) {
            const int v = RLO_get_vote_proposal(eng, fl[i]);
            if (v < 0) { i++; continue; }
            approved += v;
            done++;
            fl[i] = fl[--nfl];
        }
        RLO_user_msg* u = NULL;
        while (RLO_user_pickup_next(eng, &u)) {
            if (u->type == RLO_IAR_DECISION) got++;
            RLO_user_msg_recycle(eng, u);
        }
    }
    double dt = now_s() - t0, dtmax = 0;
    long app = 0;
    MPI_Reduce(&dt, &dtmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    MPI_Reduce(&approved, &app, 1, MPI_LONG, MPI_SUM, 0, MPI_COMM_WORLD);
    if (g_rank == 0)
        fprintf(g_out, "{\"mode\":\"iarpool\",\"ranks\":%d,\"P\":%d,\"pool\":%d,\"seconds\":%.6f,\"decisions_per_s\":%.1f,\"approved\":%ld}\n",
               g_size, P, D, dtmax, g_size * (double)P / dtmax, app);
    RLO_progress_engine_cleanup(eng);
}
#endif

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
    MPI_Comm_size(MPI_COMM_WORLD, &g_size);
    g_out = fdopen(dup(1), "w");
    if (!g_out || !freopen("/dev/null", "w", stdout)) return 3;
    if (argc < 3) {
        if (g_rank == 0) fprintf(stderr, "usage: api_bench storm K LEN | lat ROUNDS LEN | iar P | iardj P | iarpool P\n");
        MPI_Finalize();
        return 2;
    }
    if (!strcmp(argv[1], "storm")) storm(atoi(argv[2]), argc > 3 ? atoi(argv[3]) : 64);
    else if (!strcmp(argv[1], "lat")) lat(atoi(argv[2]), argc > 3 ? atoi(argv[3]) : 64);
    else if (!strcmp(argv[1], "iar")) iar(atoi(argv[2]), 0);
#ifdef RLO_HAVE_DEVICE_JUDGE
    else if (!strcmp(argv[1], "iardj")) iar(atoi(argv[2]), 1);
#endif
#ifdef RLO_HAVE_PROPOSAL_POOL
    else if (!strcmp(argv[1], "iarpool")) iarpool(atoi(argv[2]));
#endif
    fflush(g_out);
#ifdef RLO_HAVE_DEVICE_JUDGE
    /* the drop-in's extension: every engine is gone -- the device memory the engines pooled goes back (world-wide) */
    if (RLO_device_memory_release(MPI_COMM_WORLD) != 0 && g_rank == 0) fprintf(stderr, "api_bench: device memory release refused\n");
#endif
    MPI_Finalize();
    return 0;
}
