/*
 * rlo_oracle.c -- TEST INFRASTRUCTURE ONLY.  Clean-room CPU restatement of the
 * reference's hot path (mierl/rootless-coll-mpi-ops, rootless_ops.c), used as
 * the parity checker for the HIP engine and as bench.py's "port" CPU baseline.
 * The product never links this file.  See rlo_oracle.h for the contract; each
 * function cites the reference lines it restates.
 *
 * MPI is replaced by an in-memory per-rank FIFO inbox (ANY_SOURCE, ANY_TAG
 * receive order = arrival order, rootless_ops.c:656), which keeps MPI's
 * per-sender non-overtaking guarantee that the IAR protocol relies on.
 */
#define _POSIX_C_SOURCE 200809L
#include "rlo_oracle.h"
#include "rlo_testvec.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ topology */

/* rootless_ops.c:1416-1425 */
static int is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

/* floor(log2(n)) in integers; the reference truncates a double log2 (:1430-1432) */
static int ilog2(int n) {
    int l = 0;
    while ((n >> (l + 1)) != 0) l++;
    return l;
}

/* rootless_ops.c:1427-1441 */
static int level_of(int n, int rank) {
    if (rank == 0) return is_pow2(n) ? ilog2(n) - 1 : ilog2(n);
    int l = 0;
    while (rank != 0 && (rank & 1) == 0) { rank >>= 1; l++; }
    return l;
}

typedef struct {
    int level, last_wall, scc, sll;
    int send_list[ORC_MAX_FANOUT];
} topo_t;

/* rootless_ops.c:1454-1522 (bcomm_init), with pow()/log2() restated as exact integer ops */
static void topo_init(int n, int rank, topo_t* t) {
    t->level = level_of(n, rank);
    if (rank == 0) t->last_wall = 1 << t->level;        /* :1478-1479 */
    else t->last_wall = rank & (rank - 1);               /* :1444-1452: clear lowest set bit */
    t->scc = t->level;
    t->sll = t->scc + 1;
    if (is_pow2(n)) {
        for (int i = 0; i < t->sll; i++) t->send_list[i] = (rank + (1 << i)) % n;
    } else {
        for (int i = 0; i < t->sll; i++) {
            int dest = rank + (1 << i);
            if (dest >= n) {
                if (rank == n - 1) { t->scc = 0; t->send_list[0] = 0; }
                else { t->scc = i; t->send_list[i] = 0; }
                t->sll = t->scc + 1;
                break;
            }
            t->send_list[i] = dest;
        }
    }
}

int orc_topology(int n, int rank, int* level, int* last_wall, int* scc, int* sll, int* send_list) {
    if (n < 2 || rank < 0 || rank >= n) return -1; /* :1464-1467 */
    topo_t t;
    topo_init(n, rank, &t);
    if (level) *level = t.level;
    if (last_wall) *last_wall = t.last_wall;
    if (scc) *scc = t.scc;
    if (sll) *sll = t.sll;
    if (send_list) memcpy(send_list, t.send_list, sizeof(int) * t.sll);
    return 0;
}

/* rootless_ops.c:1534-1556 */
static int passed_origin(int me, int origin, int to) {
    if (to == origin) return 1;
    if (me >= origin) {
        if (to > me) return 0;
        if (to >= 0 && to < origin) return 0;
        return 1;
    }
    if (to > me && to < origin) return 0;
    return 1;
}

int orc_check_passed_origin(int n, int rank, int origin, int to) {
    (void)n;
    return passed_origin(rank, origin, to);
}

/* children in the reference's send order (farthest first).
 * originate: rootless_ops.c:1587 ; forward: :1116-1223                                  */
static int children_t(const topo_t* t, int me, int origin, int from, int* out) {
    int c = 0;
    if (from < 0) {
        for (int i = t->sll - 1; i >= 0; i--) out[c++] = t->send_list[i];
        return c;
    }
    if (t->level <= 0) return 0;                                /* leaf, :1208 */
    if (from > t->last_wall) {                                  /* branch A, :1120 */
        for (int j = t->scc; j >= 0; j--) out[c++] = t->send_list[j];
        return c;
    }
    for (int j = t->scc - 1; j >= 0; j--)                       /* branch B, :1144-1159 */
        if (passed_origin(me, origin, t->send_list[j]) == 0) out[c++] = t->send_list[j];
    return c;
}

int orc_children(int n, int rank, int origin, int from, int* out) {
    topo_t t;
    topo_init(n, rank, &t);
    return children_t(&t, rank, origin, from, out);
}

/* rootless_ops.c:1559-1579 (equals what _bc_forward sends) */
int orc_fwd_send_cnt(int n, int rank, int origin, int from) {
    int tmp[ORC_MAX_FANOUT];
    topo_t t;
    topo_init(n, rank, &t);
    if (from < 0) return t.sll;
    return children_t(&t, rank, origin, from, tmp);
}

/* ------------------------------------------------------------------ workload */

void orc_payload(uint32_t origin, uint32_t bid, uint8_t* out, size_t len) { rlo_tv_payload(origin, bid, out, len); }
uint32_t orc_origin_of(uint64_t seed, uint64_t bid, uint32_t n) { return rlo_tv_origin(seed, bid, n); }
uint64_t orc_region_hash(const uint8_t* p, size_t len) { return rlo_tv_region_hash(p, len); }
uint64_t orc_fnv1a(const uint8_t* p, size_t len) { return rlo_tv_fnv1a(p, len, RLO_TV_FNV_INIT); }

static inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

uint32_t orc_chunk_mix(uint32_t q, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    return fmix32(w0 ^ fmix32(w1 ^ fmix32(w2 ^ fmix32(w3 ^ (q * 0x9E3779B9u + 0x7F4A7C15u)))));
}

/* checksum of one delivered message: header term + one term per 16-byte payload chunk
 * (payload zero padded to a multiple of 16).                                            */
uint64_t orc_msg_checksum(uint32_t origin, uint32_t bid, uint32_t tag, const uint8_t* p, uint32_t len) {
    uint64_t s = orc_chunk_mix(0xFFFFFFFFu, origin, bid, tag, len);
    for (uint32_t off = 0, q = 0; off < len; off += 16, q++) {
        uint32_t w[4] = {0, 0, 0, 0};
        uint32_t k = len - off < 16 ? len - off : 16;
        memcpy(w, p + off, k);
        s += orc_chunk_mix(q, w[0], w[1], w[2], w[3]);
    }
    return s;
}

/* ------------------------------------------------------------------ mailboxes */

typedef struct {
    int32_t tag, origin, from, id, vote;
    uint32_t len;
    uint8_t* data; /* owned copy: every hop copies the bytes, like an MPI send */
    uint64_t cs;   /* storm: checksum of a bulk message (beyond the reference's 32,764-B cap, its
                      bytes are a pure function of (origin, bid, len) and are not copied per hop) */
} omsg;

typedef struct {
    omsg* q;
    size_t head, tail, cap; /* ring; cap power of 2 */
} ofifo;

static int fifo_push(ofifo* f, const omsg* m) {
    if (f->tail - f->head == f->cap) {
        size_t ncap = f->cap ? f->cap * 2 : 64;
        omsg* nq = malloc(ncap * sizeof(omsg));
        if (!nq) return -1;
        for (size_t i = f->head; i < f->tail; i++) nq[i - f->head] = f->q[i & (f->cap - 1)];
        f->tail -= f->head;
        f->head = 0;
        free(f->q);
        f->q = nq;
        f->cap = ncap;
    }
    f->q[f->tail++ & (f->cap - 1)] = *m;
    return 0;
}

static int fifo_pop(ofifo* f, omsg* m) {
    if (f->head == f->tail) return 0;
    *m = f->q[f->head++ & (f->cap - 1)];
    return 1;
}

/* send a copy of (hdr, bytes) from `me` to `to` (MPI_Isend of the whole buffer) */
static int post(ofifo* inbox, int to, int me, const omsg* m) {
    omsg c = *m;
    c.from = me;
    c.data = NULL;
    if (m->len && m->data) {
        c.data = malloc(m->len);
        if (!c.data) return -1;
        memcpy(c.data, m->data, m->len);
    }
    return fifo_push(&inbox[to], &c);
}

/* ------------------------------------------------------------------ single tree */

int orc_tree(int n, int origin, int32_t* parent) {
    if (n < 2 || origin < 0 || origin >= n) return -1;
    ofifo* inbox = calloc(n, sizeof(ofifo));
    topo_t* t = malloc(n * sizeof(topo_t));
    for (int r = 0; r < n; r++) { topo_init(n, r, &t[r]); parent[r] = -1; }
    omsg m = {ORC_BCAST, origin, -1, 0, -1, 0, NULL, 0};
    int kids[ORC_MAX_FANOUT], cnt = 0, busy = 1;
    int k = children_t(&t[origin], origin, origin, -1, kids);
    for (int i = 0; i < k; i++) post(inbox, kids[i], origin, &m);
    while (busy) {
        busy = 0;
        for (int r = 0; r < n; r++) {
            omsg in;
            while (fifo_pop(&inbox[r], &in)) {
                busy = 1;
                if (parent[r] != -1 || r == origin) cnt = -1000000; /* duplicate / self delivery */
                parent[r] = in.from;
                cnt++;
                int kk = children_t(&t[r], r, in.origin, in.from, kids);
                for (int i = 0; i < kk; i++) post(inbox, kids[i], r, &in);
                free(in.data);
            }
        }
    }
    for (int r = 0; r < n; r++) free(inbox[r].q);
    free(inbox);
    free(t);
    return cnt;
}

/* ------------------------------------------------------------------ storm */

#define ORC_COPY_MAX 32764 /* the reference's deliverable data region (rootless_ops.c:1588) */

int64_t orc_storm2(int n, uint64_t seed, int64_t k, uint32_t len_lo, uint32_t len_hi, uint32_t order, int32_t* parent,
                   int64_t* count, uint64_t* sum) {
    if (n < 2 || k < 0) return -1;
    if (len_hi < len_lo) len_hi = len_lo;
    ofifo* inbox = calloc(n, sizeof(ofifo));
    topo_t* t = malloc(n * sizeof(topo_t));
    int64_t* next = calloc(n + 1, sizeof(int64_t)); /* next bid index scan position per rank */
    uint8_t* buf = malloc(len_hi ? len_hi : 1);
    int64_t deliveries = 0, originated = 0;
    for (int r = 0; r < n; r++) {
        topo_init(n, r, &t[r]);
        if (count) count[r] = 0;
        if (sum) sum[r] = 0;
    }
    if (parent)
        for (int64_t i = 0; i < k * (int64_t)n; i++) parent[i] = -1;
    /* per-rank origination lists (CSR) */
    int64_t* off = calloc(n + 1, sizeof(int64_t));
    int64_t* ids = malloc((k ? k : 1) * sizeof(int64_t));
    for (int64_t b = 0; b < k; b++) off[rlo_tv_origin2(seed, b, n, order) + 1]++;
    for (int r = 0; r < n; r++) off[r + 1] += off[r];
    for (int64_t b = 0; b < k; b++) {
        uint32_t o = rlo_tv_origin2(seed, b, n, order);
        ids[off[o] + next[o]++] = b;
    }
    memset(next, 0, (n + 1) * sizeof(int64_t));
    int kids[ORC_MAX_FANOUT];
    int busy = 1;
    while (busy) {
        busy = 0;
        for (int r = 0; r < n; r++) {
            /* originate one bcast (RLO_msg_new_bc + RLO_bcast_gen, rootless_ops.c:311, :1581) */
            if (off[r] + next[r] < off[r + 1]) {
                uint32_t bid = (uint32_t)ids[off[r] + next[r]++];
                uint32_t len = rlo_tv_len(seed, bid, len_lo, len_hi);
                rlo_tv_payload(r, bid, buf, len);
                omsg m = {ORC_BCAST, r, -1, (int32_t)bid, -1, len, buf, 0};
                if (len > ORC_COPY_MAX) { /* a bulk message: every receiver gets exactly these bytes */
                    m.cs = orc_msg_checksum(r, bid, ORC_BCAST, buf, len);
                    m.data = NULL;
                }
                int kk = children_t(&t[r], r, r, -1, kids);
                for (int i = 0; i < kk; i++) post(inbox, kids[i], r, &m);
                originated++;
                busy = 1;
            }
            /* progress: receive, deliver (pickup), forward (make_progress_gen :569-624) */
            omsg in;
            while (fifo_pop(&inbox[r], &in)) {
                busy = 1;
                deliveries++;
                if (count) count[r]++;
                if (sum) sum[r] += in.data || in.len == 0 ? orc_msg_checksum(in.origin, in.id, ORC_BCAST, in.data, in.len) : in.cs;
                if (parent) parent[(int64_t)in.id * n + r] = in.from;
                int kk = children_t(&t[r], r, in.origin, in.from, kids);
                for (int i = 0; i < kk; i++) post(inbox, kids[i], r, &in);
                free(in.data);
            }
        }
    }
    for (int r = 0; r < n; r++) free(inbox[r].q);
    free(inbox); free(t); free(next); free(buf); free(off); free(ids);
    return originated == k ? deliveries : -1;
}

int64_t orc_storm(int n, uint64_t seed, int64_t k, uint32_t len, int32_t* parent, int64_t* count, uint64_t* sum) {
    return orc_storm2(n, seed, k, len, len, 0, parent, count, sum);
}

int64_t orc_storm_expected2(int n, uint64_t seed, int64_t k, uint32_t len_lo, uint32_t len_hi, uint32_t order,
                            int64_t* count, uint64_t* sum) {
    if (n < 2 || k < 0) return -1;
    if (len_hi < len_lo) len_hi = len_lo;
    uint8_t* buf = malloc(len_hi ? len_hi : 1);
    uint64_t total = 0;
    int64_t* own_cnt = calloc(n, sizeof(int64_t));
    uint64_t* own_sum = calloc(n, sizeof(uint64_t));
    for (int64_t b = 0; b < k; b++) {
        uint32_t o = rlo_tv_origin2(seed, b, n, order);
        uint32_t len = rlo_tv_len(seed, b, len_lo, len_hi);
        rlo_tv_payload(o, (uint32_t)b, buf, len);
        uint64_t cs = orc_msg_checksum(o, (uint32_t)b, ORC_BCAST, buf, len);
        total += cs;
        own_cnt[o]++;
        own_sum[o] += cs;
    }
    for (int r = 0; r < n; r++) {
        if (count) count[r] = k - own_cnt[r];
        if (sum) sum[r] = total - own_sum[r];
    }
    free(buf); free(own_cnt); free(own_sum);
    return k * (int64_t)(n - 1);
}

int64_t orc_storm_expected(int n, uint64_t seed, int64_t k, uint32_t len, int64_t* count, uint64_t* sum) {
    return orc_storm_expected2(n, seed, k, len, len, 0, count, sum);
}

/* ------------------------------------------------------------------ storm on host threads */

/* orc_storm2 on T threads.  Rank r is progressed by thread r % T only (its origination list, its
 * deliveries, its count / sum).  A forward copies the bytes into the sending thread's outgoing
 * batch for the receiving thread (one batch per thread pair per sweep, handed over under that
 * thread's inbox lock): every tree edge still copies the payload, as an MPI send does. */
typedef struct {
    int32_t origin, from, to, id;
    uint32_t len;
    uint64_t off, cs; /* bytes at batch.bytes + off (ring-sized messages); cs for bulk ones */
} mt_msg;

typedef struct mt_batch {
    mt_msg* m;
    size_t n, cap;
    uint8_t* bytes;
    size_t nb, bcap;
    struct mt_batch* next;
} mt_batch;

typedef struct {
    pthread_mutex_t mu;
    mt_batch* head;
} mt_inbox;

typedef struct {
    int n, nthr, tid;
    uint64_t seed;
    uint32_t lo, hi;
    const topo_t* t;
    const int64_t *off, *ids;
    const int* owner; /* thread of each rank */
    mt_inbox* in;
    atomic_llong* delivered;
    int64_t want;
    int64_t* count;
    uint64_t* sum;
    int err;
} mt_arg;

static int mt_put(mt_batch* b, int to, int from, int origin, int id, uint32_t len, const uint8_t* data, uint64_t cs) {
    if (b->n == b->cap) {
        size_t nc = b->cap ? 2 * b->cap : 256;
        mt_msg* nm = realloc(b->m, nc * sizeof(mt_msg));
        if (!nm) return -1;
        b->m = nm;
        b->cap = nc;
    }
    mt_msg* m = &b->m[b->n++];
    *m = (mt_msg){origin, from, to, id, len, b->nb, cs};
    if (data && len) {
        if (b->nb + len > b->bcap) {
            size_t nc = b->bcap ? 2 * b->bcap : 65536;
            while (nc < b->nb + len) nc *= 2;
            uint8_t* nb = realloc(b->bytes, nc);
            if (!nb) return -1;
            b->bytes = nb;
            b->bcap = nc;
        }
        memcpy(b->bytes + b->nb, data, len);
        b->nb += len;
    }
    return 0;
}

static void mt_forward(mt_arg* a, mt_batch** out, int me, int origin, int from, int id, uint32_t len,
                       const uint8_t* data, uint64_t cs) {
    int kids[ORC_MAX_FANOUT];
    int kk = children_t(&a->t[me], me, origin, from, kids);
    for (int i = 0; i < kk; i++) {
        mt_batch* b = out[a->owner[kids[i]]];
        a->err |= mt_put(b, kids[i], me, origin, id, len, data, cs);
    }
}

static mt_batch* mt_take(mt_batch** pool) { /* recycled batches keep their buffers (no page faults) */
    mt_batch* b = *pool;
    if (!b) return calloc(1, sizeof(mt_batch));
    *pool = b->next;
    b->n = b->nb = 0;
    b->next = NULL;
    return b;
}

static void mt_free_list(mt_batch* b) {
    while (b) {
        mt_batch* nx = b->next;
        free(b->m); free(b->bytes); free(b);
        b = nx;
    }
}

static void* mt_worker(void* vp) {
    mt_arg* a = (mt_arg*)vp;
    const int T = a->nthr;
    mt_batch* pool = NULL;
    /* a contiguous block of ranks per thread: every block holds the same mix of tree levels (a
     * strided deal would give one thread every multiple of T, the skip ring's interior ranks) */
    const int r0 = (int)((int64_t)a->tid * a->n / T), r1 = (int)((int64_t)(a->tid + 1) * a->n / T);
    int64_t* count = calloc(a->n, sizeof(int64_t)); /* thread-private: no false sharing between */
    uint64_t* sum = calloc(a->n, sizeof(uint64_t)); /* neighbouring ranks of different threads */
    uint8_t* buf = malloc(a->hi ? a->hi : 1);
    int64_t* next = calloc(a->n, sizeof(int64_t));
    mt_batch** out = calloc(T, sizeof(mt_batch*));
    for (int j = 0; j < T; j++) out[j] = mt_take(&pool);
    mt_batch* local = NULL; /* batches from this thread to itself, processed next sweep */
    while (atomic_load_explicit(a->delivered, memory_order_relaxed) < a->want && !a->err) {
        for (int r = r0; r < r1; r++) /* originate one per rank (RLO_bcast_gen :1581) */
            if (a->off[r] + next[r] < a->off[r + 1]) {
                uint32_t bid = (uint32_t)a->ids[a->off[r] + next[r]++];
                uint32_t len = rlo_tv_len(a->seed, bid, a->lo, a->hi);
                rlo_tv_payload(r, bid, buf, len);
                if (len > ORC_COPY_MAX)
                    mt_forward(a, out, r, r, -1, (int)bid, len, NULL, orc_msg_checksum(r, bid, ORC_BCAST, buf, len));
                else
                    mt_forward(a, out, r, r, -1, (int)bid, len, buf, 0);
            }
        pthread_mutex_lock(&a->in[a->tid].mu); /* take everything sent to my ranks */
        mt_batch* got = a->in[a->tid].head;
        a->in[a->tid].head = NULL;
        pthread_mutex_unlock(&a->in[a->tid].mu);
        if (local) { local->next = got; got = local; local = NULL; }
        int64_t mine = 0;
        while (got) { /* receive, deliver (pickup), forward (make_progress_gen :569-624) */
            mt_batch* b = got;
            got = b->next;
            for (size_t i = 0; i < b->n; i++) {
                const mt_msg* m = &b->m[i];
                const uint8_t* d = m->len && m->len <= ORC_COPY_MAX ? b->bytes + m->off : NULL;
                mine++;
                count[m->to]++;
                sum[m->to] += d || m->len == 0 ? orc_msg_checksum(m->origin, m->id, ORC_BCAST, d, m->len) : m->cs;
                mt_forward(a, out, m->to, m->origin, m->from, m->id, m->len, d, m->cs);
            }
            b->next = pool;
            pool = b;
        }
        for (int j = 0; j < T; j++) { /* hand the outgoing batches over */
            mt_batch* b = out[j];
            if (!b->n) continue;
            out[j] = mt_take(&pool);
            if (j == a->tid) { local = b; continue; }
            pthread_mutex_lock(&a->in[j].mu);
            b->next = a->in[j].head;
            a->in[j].head = b;
            pthread_mutex_unlock(&a->in[j].mu);
        }
        if (mine) atomic_fetch_add_explicit(a->delivered, mine, memory_order_relaxed);
    }
    for (int j = 0; j < T; j++) {
        if (out[j]->n) a->err = 1; /* nothing may be left unsent */
        free(out[j]->m); free(out[j]->bytes); free(out[j]);
    }
    if (local) { a->err = 1; mt_free_list(local); }
    for (int r = r0; r < r1; r++) {
        a->count[r] = count[r];
        a->sum[r] = sum[r];
    }
    free(count); free(sum);
    mt_free_list(pool);
    free(out); free(buf); free(next);
    return NULL;
}

int64_t orc_storm_mt(int n, uint64_t seed, int64_t k, uint32_t len_lo, uint32_t len_hi, uint32_t order, int threads,
                     int64_t* count, uint64_t* sum) {
    if (n < 2 || k < 0 || threads < 1 || !count || !sum) return -1;
    if (threads > n) threads = n;
    if (len_hi < len_lo) len_hi = len_lo;
    topo_t* t = malloc(n * sizeof(topo_t));
    mt_inbox* in = calloc(threads, sizeof(mt_inbox));
    int64_t* off = calloc(n + 1, sizeof(int64_t));
    int64_t* fill = calloc(n, sizeof(int64_t));
    int64_t* ids = malloc((k ? k : 1) * sizeof(int64_t));
    for (int r = 0; r < n; r++) {
        topo_init(n, r, &t[r]);
        count[r] = 0;
        sum[r] = 0;
    }
    for (int i = 0; i < threads; i++) pthread_mutex_init(&in[i].mu, NULL);
    for (int64_t b = 0; b < k; b++) off[rlo_tv_origin2(seed, b, n, order) + 1]++;
    for (int r = 0; r < n; r++) off[r + 1] += off[r];
    for (int64_t b = 0; b < k; b++) {
        uint32_t o = rlo_tv_origin2(seed, b, n, order);
        ids[off[o] + fill[o]++] = b;
    }
    int* owner = malloc(n * sizeof(int));
    for (int i = 0; i < threads; i++)
        for (int r = (int)((int64_t)i * n / threads); r < (int)((int64_t)(i + 1) * n / threads); r++) owner[r] = i;
    atomic_llong delivered = 0;
    mt_arg* args = calloc(threads, sizeof(mt_arg));
    pthread_t* th = malloc(threads * sizeof(pthread_t));
    for (int i = 0; i < threads; i++) {
        args[i] = (mt_arg){n, threads, i, seed, len_lo, len_hi, t, off, ids, owner, in, &delivered, k * (int64_t)(n - 1),
                           count, sum, 0};
        pthread_create(&th[i], NULL, mt_worker, &args[i]);
    }
    int err = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        err |= args[i].err;
    }
    for (int i = 0; i < threads; i++) {
        if (in[i].head) err = 1; /* nothing may be left in flight */
        mt_free_list(in[i].head);
        pthread_mutex_destroy(&in[i].mu);
    }
    int64_t d = atomic_load(&delivered);
    free(t); free(in); free(off); free(fill); free(ids); free(args); free(th); free(owner);
    return err ? -1 : d;
}

uint32_t orc_len_of(uint64_t seed, uint64_t bid, uint32_t lo, uint32_t hi) { return rlo_tv_len(seed, bid, lo, hi); }
uint32_t orc_origin_of2(uint64_t seed, uint64_t bid, uint32_t n, uint32_t order) {
    return rlo_tv_origin2(seed, bid, n, order);
}

/* ------------------------------------------------------------------ IAR */

uint32_t orc_judge_hash(uint64_t seed, uint32_t rank, int32_t pid) {
    uint64_t x = rlo_tv_splitmix64(seed ^ ((uint64_t)rank << 32) ^ (uint32_t)pid);
    return (uint32_t)(x % 1000000u);
}

typedef struct {
    const orc_judge_cfg* cfg;
    const char** isp; /* per-rank strings (ISP) */
} judge_ctx;

/* arg == NULL: the originator's final call (rootless_ops.c:773, eng->my_proposal is never set) */
static int judge_eval(const judge_ctx* j, int rank, int32_t pid, const char* arg) {
    switch (j->cfg->kind) {
        case ORC_JUDGE_MASK:
            return (arg && j->cfg->decline[rank]) ? 0 : 1;
        case ORC_JUDGE_HASH:
            return (arg && orc_judge_hash(j->cfg->seed, rank, pid) < j->cfg->ppm) ? 0 : 1;
        case ORC_JUDGE_ISP: { /* testcases.c:18-37 */
            const char* mine = j->isp[rank];
            if (!mine || strlen(mine) == 0) return 1;
            if (!arg) return 1;
            if (strcmp(mine, arg) == 0) return 1;
            if (((const char*)arg)[0] < mine[0]) return 0;
            return 1;
        }
        default:
            return 1;
    }
}

typedef struct {
    int32_t pid, origin, parent, vote, needed, recvd;
    uint32_t len;
    uint8_t* pbuf; /* serialized PBuf of the proposal (action argument, :842) */
} pending_t;

typedef struct {
    int32_t pid, vote, needed, recvd, state; /* state: 0 none, 1 in progress */
    int32_t iter;
} own_t;

typedef struct {
    int n;
    topo_t* t;
    ofifo* inbox;
    own_t* own;  /* [n][pool]: the proposal pool (PROPOSAL_POOL_SIZE, rootless_ops.c:30); pool 1 =
                    my_own_proposal (:241) */
    int pool;
    pending_t** pend; /* per rank dynamic array */
    int* npend;
    int* cappend;
    judge_ctx j;
    int32_t* ev;
    int cap, nev, overflow;
    int64_t decisions, approved, judge_calls, actions;
    int record;
} iar_sim;

static void ev_put(iar_sim* s, int e, int rank, int pid, int a, int b, int c) {
    if (!s->record) return;
    if (s->nev >= s->cap) { s->overflow = 1; return; }
    int32_t* p = s->ev + 6 * s->nev++;
    p[0] = e; p[1] = rank; p[2] = pid; p[3] = a; p[4] = b; p[5] = c;
}

/* PBuf wire codec, rootless_ops.c:1369-1410: [pid i32][vote i32][data_len u64][data] */
static uint8_t* pbuf_make(int32_t pid, int32_t vote, uint64_t dl, const void* data, uint32_t total) {
    uint8_t* b = calloc(1, total);
    memcpy(b, &pid, 4);
    memcpy(b + 4, &vote, 4);
    memcpy(b + 8, &dl, 8);
    if (dl) memcpy(b + 16, data, dl);
    return b;
}

static void bcast_from(iar_sim* s, int r, omsg* m) {
    int kids[ORC_MAX_FANOUT];
    int kk = children_t(&s->t[r], r, r, -1, kids);
    for (int i = 0; i < kk; i++) post(s->inbox, kids[i], r, m);
}

/* a free pool slot of rank r (proposalPool_proposal_add :1253-1279 "first available"), or NULL */
static own_t* own_free(iar_sim* s, int r) {
    for (int k = 0; k < s->pool; k++)
        if (s->own[r * s->pool + k].state == 0) return &s->own[r * s->pool + k];
    return NULL;
}

/* RLO_submit_proposal, rootless_ops.c:876-906 (pool 1: it overwrites my_own_proposal, as the
 * reference does; larger pools take a free slot, the caller checks there is one) */
static void submit(iar_sim* s, int r, int32_t pid, const char* data, uint32_t dl) {
    own_t* o = own_free(s, r);
    if (!o) o = &s->own[r * s->pool];
    o->pid = pid;
    o->vote = 1;
    o->needed = s->t[r].sll;
    o->recvd = 0;
    o->state = 1;
    uint32_t total = 16 + dl;
    omsg m = {ORC_PROPOSAL, r, -1, pid, 1, total, pbuf_make(pid, 1, dl, data, total), 0};
    bcast_from(s, r, &m);
    free(m.data);
}

static void vote_to(iar_sim* s, int r, int parent, int32_t pid, int32_t vote) { /* _vote_back :728-741 */
    omsg v = {ORC_VOTE, r, -1, pid, vote, 0, NULL, 0};
    post(s->inbox, parent, r, &v);
}

/* _iar_decision_bcast :908-917: PBuf(pid, decision, 7, "IAR_DEC") in a 64-byte buffer */
static void decision_bcast(iar_sim* s, int r, own_t* o, int32_t pid, int32_t d) {
    omsg m = {ORC_DECISION, r, -1, pid, d, 64, pbuf_make(pid, d, 7, "IAR_DEC", 64), 0};
    bcast_from(s, r, &m);
    free(m.data);
    s->decisions++;
    if (d) s->approved++;
    ev_put(s, ORC_EV_RESULT, r, pid, d, 0, 0);
    o->state = 0;
    o->vote = d;
}

/* the pool slot holding own proposal pid (any state: the reference keeps my_own_proposal.pid after
 * the decision until RLO_proposal_reset), or NULL */
static own_t* own_find(iar_sim* s, int r, int32_t pid) {
    for (int k = 0; k < s->pool; k++)
        if (s->own[r * s->pool + k].pid == pid) return &s->own[r * s->pool + k];
    return NULL;
}

static pending_t* find_pending(iar_sim* s, int r, int32_t pid, int* idx) { /* _find_proposal_msg :1036-1053 */
    if (pid < 0) return NULL;
    for (int i = 0; i < s->npend[r]; i++)
        if (s->pend[r][i].pid == pid) { if (idx) *idx = i; return &s->pend[r][i]; }
    return NULL;
}

static void drop_pending(iar_sim* s, int r, int i) {
    free(s->pend[r][i].pbuf);
    memmove(&s->pend[r][i], &s->pend[r][i + 1], (s->npend[r] - i - 1) * sizeof(pending_t));
    s->npend[r]--;
}

static void handle(iar_sim* s, int r, omsg* in) {
    int kids[ORC_MAX_FANOUT];
    switch (in->tag) {
        case ORC_PROPOSAL: { /* _iar_proposal_handler :668-726 */
            int32_t pid = in->id;
            uint64_t dl;
            memcpy(&dl, in->data + 8, 8);
            if (own_find(s, r, pid)) { ev_put(s, ORC_EV_ERROR, r, pid, 1, in->origin, 0); break; } /* :690-692 */
            char* arg = calloc(1, dl + 1);
            memcpy(arg, in->data + 16, dl);
            int jr = judge_eval(&s->j, r, pid, arg);
            s->judge_calls++;
            ev_put(s, ORC_EV_JUDGE, r, pid, 0, jr, in->origin);
            free(arg);
            if (jr == 0) { vote_to(s, r, in->from, pid, 0); break; }
            int kk = children_t(&s->t[r], r, in->origin, in->from, kids);
            for (int i = 0; i < kk; i++) post(s->inbox, kids[i], r, in);
            if (s->npend[r] == s->cappend[r]) {
                s->cappend[r] = s->cappend[r] ? 2 * s->cappend[r] : 8;
                s->pend[r] = realloc(s->pend[r], s->cappend[r] * sizeof(pending_t));
            }
            pending_t* p = &s->pend[r][s->npend[r]++];
            p->pid = pid; p->origin = in->origin; p->parent = in->from; p->vote = 1; p->needed = kk; p->recvd = 0;
            p->len = in->len;
            p->pbuf = malloc(in->len);
            memcpy(p->pbuf, in->data, in->len);
            if (kk == 0) vote_to(s, r, in->from, pid, 1); /* :715-717 */
            break;
        }
        case ORC_VOTE: { /* _iar_vote_handler :743-812 */
            own_t* o = own_find(s, r, in->id);  /* proposalPool_vote_merge :1286-1305 */
            if (o) {
                o->recvd++;
                o->vote &= in->vote;
                if (o->recvd == o->needed) {
                    if (o->vote) {
                        int jr = judge_eval(&s->j, r, o->pid, NULL); /* :773 */
                        s->judge_calls++;
                        ev_put(s, ORC_EV_JUDGE, r, o->pid, 1, jr, r);
                        o->vote = jr;
                    }
                    decision_bcast(s, r, o, o->pid, o->vote);
                }
                break;
            }
            pending_t* p = find_pending(s, r, in->id, NULL); /* _vote_merge :1056-1070 */
            if (!p) { ev_put(s, ORC_EV_ERROR, r, in->id, 2, in->from, 0); break; }
            p->vote &= in->vote;
            p->recvd++;
            if (p->recvd == p->needed) vote_to(s, r, p->parent, p->pid, p->vote);
            break;
        }
        case ORC_DECISION: { /* case RLO_IAR_DECISION :603-615, _iar_decision_handler :814-859 */
            int32_t pid, d;
            memcpy(&pid, in->data, 4);
            memcpy(&d, in->data + 4, 4);
            int idx;
            pending_t* p = find_pending(s, r, pid, &idx);
            if (p) {
                if (d != 0) {
                    int32_t pv;
                    uint64_t pdl;
                    memcpy(&pv, p->pbuf + 4, 4);
                    memcpy(&pdl, p->pbuf + 8, 8);
                    s->actions++;
                    ev_put(s, ORC_EV_ACTION, r, p->pid, pv, (int)pdl, p->origin);
                }
                drop_pending(s, r, idx);
            }
            ev_put(s, ORC_EV_PICKUP, r, pid, d, in->origin, 7);
            int kk = children_t(&s->t[r], r, in->origin, in->from, kids);
            for (int i = 0; i < kk; i++) post(s->inbox, kids[i], r, in);
            break;
        }
        default:
            break;
    }
}

static void sim_init(iar_sim* s, int n, const orc_judge_cfg* judge, int pool) {
    memset(s, 0, sizeof *s);
    s->n = n;
    s->pool = pool < 1 ? 1 : pool;
    s->t = malloc(n * sizeof(topo_t));
    s->inbox = calloc(n, sizeof(ofifo));
    s->own = calloc((size_t)n * s->pool, sizeof(own_t));
    s->pend = calloc(n, sizeof(pending_t*));
    s->npend = calloc(n, sizeof(int));
    s->cappend = calloc(n, sizeof(int));
    s->j.cfg = judge;
    s->j.isp = calloc(n, sizeof(char*));
    if (judge->kind == ORC_JUDGE_ISP && judge->isp) {
        const char* p = judge->isp;
        for (int r = 0; r < n; r++) { s->j.isp[r] = p; p += strlen(p) + 1; }
    }
    for (int r = 0; r < n; r++) {
        topo_init(n, r, &s->t[r]);
        for (int k = 0; k < s->pool; k++) s->own[r * s->pool + k].pid = -1; /* proposal_state_init :1238 */
    }
}

static void sim_free(iar_sim* s) {
    for (int r = 0; r < s->n; r++) {
        free(s->inbox[r].q);
        for (int i = 0; i < s->npend[r]; i++) free(s->pend[r][i].pbuf);
        free(s->pend[r]);
    }
    free(s->t); free(s->inbox); free(s->own); free(s->pend); free(s->npend); free(s->cappend); free(s->j.isp);
}

static int sim_step_all(iar_sim* s) {
    int busy = 0;
    for (int r = 0; r < s->n; r++) {
        omsg in;
        while (fifo_pop(&s->inbox[r], &in)) {
            busy = 1;
            handle(s, r, &in);
            free(in.data);
        }
    }
    return busy;
}

int orc_iar(int n, int nprop, const int32_t* origin, const int32_t* pid, const char* data, const int32_t* data_off,
            const int32_t* data_len, const orc_judge_cfg* judge, int32_t* events, int cap) {
    if (n < 2) return -1;
    iar_sim s;
    sim_init(&s, n, judge, 1);
    s.ev = events;
    s.cap = cap;
    s.record = 1;
    for (int i = 0; i < nprop; i++) submit(&s, origin[i], pid[i], data + data_off[i], (uint32_t)data_len[i]);
    while (sim_step_all(&s)) {}
    int nev = s.overflow ? -1 : s.nev;
    sim_free(&s);
    return nev;
}

/* the proposal pool (PROPOSAL_POOL_SIZE, rootless_ops.c:30, :159-165, :1251-1366 -- declared but
 * never wired into the reference's handlers): every origin submits its proposals in list order,
 * keeping up to `pool` of them in flight; a slot is free again once its decision went out.  Votes
 * and collisions are matched by pid over the pool's slots; everything else is orc_iar's. */
int orc_iar_pool(int n, int nprop, const int32_t* origin, const int32_t* pid, const char* data, const int32_t* data_off,
                 const int32_t* data_len, const orc_judge_cfg* judge, int pool, int32_t* events, int cap) {
    if (n < 2 || pool < 1) return -1;
    iar_sim s;
    sim_init(&s, n, judge, pool);
    s.ev = events;
    s.cap = cap;
    s.record = 1;
    int* next = calloc(n, sizeof(int));  /* per origin: index into the list of its next proposal */
    int busy = 1;
    while (busy) {
        busy = 0;
        for (int r = 0; r < n; r++) {
            for (;;) {
                while (next[r] < nprop && origin[next[r]] != r) next[r]++;
                if (next[r] >= nprop || !own_free(&s, r)) break;
                const int i = next[r]++;
                submit(&s, r, pid[i], data + data_off[i], (uint32_t)data_len[i]);
                busy = 1;
            }
        }
        busy |= sim_step_all(&s);
        for (int r = 0; r < n && !busy; r++) {
            while (next[r] < nprop && origin[next[r]] != r) next[r]++;
            busy |= next[r] < nprop;
        }
    }
    int nev = s.overflow ? -1 : s.nev;
    free(next);
    sim_free(&s);
    return nev;
}

/* every rank keeps `pool` outstanding proposals (pid = iter * n + rank, 16-byte body) for p
 * iterations; the next is submitted once a slot's decision went out (pool 1: once
 * RLO_get_vote_my_proposal saw the previous one decided, testcases.c :401-486 drive loop, at
 * scale).  events != NULL records them (orc_iar's format). */
static int64_t iar_rounds(int n, int p, int pool, const orc_judge_cfg* judge, int64_t* approved, int64_t* judge_calls,
                          int64_t* actions, int32_t* events, int cap, int* nev) {
    if (n < 2) return -1;
    iar_sim s;
    sim_init(&s, n, judge, pool);
    if (events) {
        s.ev = events;
        s.cap = cap;
        s.record = 1;
    }
    static const char body[16] = "0123456789abcdef";
    int* iter = calloc(n, sizeof(int));
    int busy = 1;
    while (busy) {
        busy = 0;
        for (int r = 0; r < n; r++) {
            while (own_free(&s, r) && iter[r] < p) {
                submit(&s, r, iter[r] * n + r, body, 16);
                iter[r]++;
                busy = 1;
            }
        }
        busy |= sim_step_all(&s);
        for (int r = 0; r < n && !busy; r++) {
            busy |= iter[r] < p;
            for (int k = 0; k < s.pool; k++) busy |= s.own[r * s.pool + k].state != 0;
        }
    }
    if (approved) *approved = s.approved;
    if (judge_calls) *judge_calls = s.judge_calls;
    if (actions) *actions = s.actions;
    if (nev) *nev = s.overflow ? -1 : s.nev;
    int64_t d = s.decisions;
    free(iter);
    sim_free(&s);
    return d;
}

int64_t orc_iar_bench(int n, int p, const orc_judge_cfg* judge, int64_t* approved, int64_t* judge_calls, int64_t* actions) {
    return iar_rounds(n, p, 1, judge, approved, judge_calls, actions, NULL, 0, NULL);
}

int orc_iar_rounds(int n, int p, const orc_judge_cfg* judge, int32_t* events, int cap) {
    return orc_iar_rounds_pool(n, p, 1, judge, events, cap);
}

int orc_iar_rounds_pool(int n, int p, int pool, const orc_judge_cfg* judge, int32_t* events, int cap) {
    int nev = 0;
    if (pool < 1 || iar_rounds(n, p, pool, judge, NULL, NULL, NULL, events, cap, &nev) < 0) return -1;
    return nev;
}
