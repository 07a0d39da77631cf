// rlo_client.cpp -- a rank process's side of the shared host service (rlo_shm.hpp): it drives its
// rank of a host-service part that another process (the GPU's leader) owns.  Plain host code over
// a mapped POSIX shared-memory segment: no HIP call here, so a client process never creates GPU
// queues of its own.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

#include "rlo_hip.h"
#include "rlo_shm.hpp"

struct rlo_client {
    uint8_t* base = nullptr;
    uint64_t bytes = 0;
    const rlo::ShmHdr* h = nullptr;
    int rank = 0, lr = 0;
    uint64_t* hctl = nullptr;       // this rank's device-written counters
    const uint8_t* ev = nullptr;   // tagged pickup records of my rank (kPkRecBytes each)
    const uint8_t* evp = nullptr;
    rlo::ClientBox* box = nullptr;
    uint8_t* cmd = nullptr;
    uint8_t* llc = nullptr;  // command doorbells (rlo_shm.hpp ll_cmd_put)
    uint8_t* stage = nullptr;
    uint64_t tail = 0, pk_head = 0, req = 0;
};

namespace {

template <class T>
T ld_acq(const T* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

// one bulk request through the leader's proxy; waits for its completion (the proxy answers every
// request promptly -- only ACQUIRE can come back RLO_E_AGAIN)
int request(rlo_client* c, uint32_t op, uint32_t arg, uint64_t off, uint64_t len, uint64_t* q) {
    rlo::ClientBox* b = c->box;
    b->op = op;
    b->arg = arg;
    b->off = off;
    b->len = len;
    const uint64_t r = ++c->req;
    __atomic_store_n(&b->req, r, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0; ld_acq(&b->ack) != r; spin++) {
        if (ld_acq(&c->h->leader_failed)) return RLO_E_DEVICE;
        if ((spin & 1023u) == 1023u) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return RLO_E_TIMEOUT;
            std::this_thread::yield();
        }
    }
    if (q) *q = b->q;
    return (int)b->rc;
}

}  // namespace

extern "C" {

int rlo_client_attach(const char* name, int rank, rlo_client_t** out) {
    if (!name || !out) return RLO_E_INVAL;
    *out = nullptr;
    const int fd = shm_open(name, O_RDWR, 0);
    if (fd < 0) return RLO_E_INVAL;
    struct stat sb;
    if (fstat(fd, &sb) != 0 || (uint64_t)sb.st_size < 4096) { close(fd); return RLO_E_INVAL; }
    void* p = mmap(nullptr, (size_t)sb.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return RLO_E_INVAL;
    rlo_client* c = new rlo_client();
    c->base = (uint8_t*)p;
    c->bytes = (uint64_t)sb.st_size;
    c->h = (const rlo::ShmHdr*)p;
    const rlo::ShmHdr& h = *c->h;
    if (ld_acq(&h.magic) != rlo::kShmMagic || h.version != rlo::kShmVersion || h.total != c->bytes ||
        rank < (int)h.rb || rank >= (int)(h.rb + h.nl)) {
        munmap(p, (size_t)sb.st_size);
        delete c;
        return RLO_E_INVAL;
    }
    c->rank = rank;
    c->lr = rank - (int)h.rb;
    const uint64_t lr = (uint64_t)c->lr;
    c->hctl = (uint64_t*)(c->base + h.off_hctl) + lr * rlo::kHctlWords;
    c->ev = c->base + h.off_ev + (uint64_t)lr * h.pk_cap * rlo::kPkRecBytes;
    c->evp = c->base + h.off_evp + lr * h.pk_cap * h.max_payload;
    c->box = (rlo::ClientBox*)(c->base + h.off_cli) + lr;
    c->cmd = c->base + h.off_cmd + lr * h.cmd_cap * h.stride;
    c->stage = c->base + h.off_stage + lr * h.stage_bytes;
    c->llc = c->base + h.off_llc + lr * h.cmd_cap * rlo::kLLCmdSlot;
    // the counters this side owns restart where the segment says (a fresh part: 0)
    c->tail = ld_acq(&c->box->mtail);
    c->pk_head = ld_acq(&c->box->mpk);
    c->req = ld_acq(&c->box->req);
    *out = c;
    return RLO_OK;
}

int rlo_client_detach(rlo_client_t* c) {
    if (!c) return RLO_E_INVAL;
    munmap(c->base, (size_t)c->bytes);
    delete c;
    return RLO_OK;
}

int rlo_client_state(rlo_client_t* c) {
    if (!c) return RLO_E_INVAL;
    if (ld_acq(&c->h->leader_failed)) return RLO_E_DEVICE;
    return (int)ld_acq(&c->hctl[rlo::kHctlState]);
}

// rlo_host_post's command encoding, into the client's shared ring; the leader's proxy copies it on
int rlo_client_post(rlo_client_t* c, const rlo_cmd_t* cmd, const void* payload, uint32_t len) {
    if (!c || !cmd) return RLO_E_INVAL;
    const rlo::ShmHdr& h = *c->h;
    if (len + rlo::kHdr > h.stride || len > 0xffffffu || (len && !payload)) return RLO_E_INVAL;
    const uint64_t head = ld_acq(&c->hctl[rlo::kHctlInjHead]);  // consumed by the device
    if (c->tail - head >= h.cmd_cap) return RLO_E_AGAIN;
    uint8_t* slot = c->cmd + (c->tail & (h.cmd_cap - 1)) * (uint64_t)h.stride;
    uint32_t hdr[4];
    hdr[0] = (uint32_t)(cmd->origin & 0xffff) | ((cmd->kind & 0xffu) << 16) | ((uint32_t)(cmd->vote & 0xff) << 24);
    hdr[1] = (uint32_t)cmd->id;
    hdr[2] = (len & 0xffffffu) | ((cmd->pseq & 0xffu) << 24);
    hdr[3] = 0;
    std::memcpy(slot, hdr, sizeof hdr);
    if (len) std::memcpy(slot + rlo::kHdr, payload, len);
    rlo::ll_cmd_put(c->llc + (c->tail & (h.cmd_cap - 1)) * (uint64_t)rlo::kLLCmdSlot, c->tail, hdr, payload, len);
    c->tail++;
    __atomic_store_n(&c->box->mtail, c->tail, __ATOMIC_RELEASE);
    return RLO_OK;
}

int rlo_client_poll(rlo_client_t* c, rlo_log_rec_t* ev, void* payload, uint32_t cap) {
    if (!c || !ev) return RLO_E_INVAL;
    const rlo::ShmHdr& h = *c->h;
    // the next event as soon as its tagged units landed (rlo_shm.hpp pk_take), not after the published tail
    if (!rlo::pk_take(c->ev, c->evp, h.pk_cap, h.max_payload, __atomic_load_n(&h.pk_epoch, __ATOMIC_ACQUIRE), c->pk_head,
                      &c->hctl[rlo::kHctlPkTail], reinterpret_cast<rlo::LogRec*>(ev), payload, cap))
        return 0;
    c->pk_head++;
    __atomic_store_n(&c->box->mpk, c->pk_head, __ATOMIC_RELEASE);
    return 1;
}

int rlo_client_cmd_count(rlo_client_t* c, uint64_t* consumed, uint64_t* posted) {
    if (!c) return RLO_E_INVAL;
    if (consumed) *consumed = ld_acq(&c->hctl[rlo::kHctlInjHead]);
    if (posted) *posted = c->tail;
    return RLO_OK;
}

int rlo_client_debug(rlo_client_t* c, uint64_t* out) {
    if (!c || !out) return RLO_E_INVAL;
    out[0] = c->tail;                                   // commands posted
    out[1] = ld_acq(&c->box->fwd);                      // forwarded by the leader's proxy
    out[2] = ld_acq(&c->hctl[rlo::kHctlInjHead]);       // consumed by the kernel
    out[3] = ld_acq(&c->hctl[rlo::kHctlBeat + 0]);      // command tail the kernel last saw
    out[4] = c->pk_head;                                // pickup events consumed here
    out[5] = ld_acq(&c->hctl[rlo::kHctlPkTail]);        // pickup events written by the kernel
    out[6] = ld_acq(&c->hctl[rlo::kHctlBeat + 1]);      // pickup head the kernel last saw
    out[7] = ld_acq(&c->hctl[rlo::kHctlBeat + 2]);      // kernel iterations (every 4096)
    out[8] = ld_acq(&c->hctl[rlo::kHctlState]);
    return RLO_OK;
}

int rlo_client_fwd(rlo_client_t* c, uint64_t* fwd, int64_t* fwd_ns) {
    if (!c || !fwd || !fwd_ns) return RLO_E_INVAL;
    *fwd = ld_acq(&c->box->fwd);
    *fwd_ns = ld_acq(&c->box->fwd_ns);
    return RLO_OK;
}

int rlo_client_hdiag(rlo_client_t* c, uint64_t* out) {
    if (!c || !out) return RLO_E_INVAL;
    for (int i = 0; i < 8; i++) out[i] = ld_acq(&c->hctl[rlo::kHctlDiag + i]);
    return RLO_OK;
}

int rlo_client_bulk_put(rlo_client_t* c, const void* data, uint64_t len, uint32_t timeout_us, uint32_t* q_out) {
    if (!c || !q_out || len == 0 || !data || len > c->h->bulk_max) return RLO_E_INVAL;
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t q = 0;
    int rc;
    while ((rc = request(c, rlo::SHM_OP_ACQUIRE, 0, 0, len, &q)) == RLO_E_AGAIN) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(timeout_us)) return RLO_E_AGAIN;
    }
    if (rc != RLO_OK) return rc;
    const uint64_t win = c->h->stage_bytes;
    for (uint64_t off = 0; off < len; off += win) {  // through the staging window, window by window
        const uint64_t n = len - off < win ? len - off : win;
        std::memcpy(c->stage, (const uint8_t*)data + off, n);
        rc = request(c, rlo::SHM_OP_PUT, (uint32_t)q, off, n, nullptr);
        if (rc != RLO_OK) return rc;  // q stays free: the next attempt acquires it again
    }
    rc = request(c, rlo::SHM_OP_COMMIT, (uint32_t)q, 0, 0, nullptr);
    if (rc != RLO_OK) return rc;
    *q_out = (uint32_t)q;
    return RLO_OK;
}

int rlo_client_bulk_get(rlo_client_t* c, const rlo_log_rec_t* ev, void* dst) {
    if (!c || !ev || !dst || ev->kind != RLO_EV_DELIVER_BULK || ev->origin < 0 || ev->origin >= (int)c->h->n ||
        ev->aux >= c->h->bslots || ev->len > c->h->bulk_max)
        return RLO_E_INVAL;
    const uint64_t win = c->h->stage_bytes;
    const uint32_t arg = ((uint32_t)ev->origin << 8) | ev->aux;
    for (uint64_t off = 0; off < ev->len; off += win) {
        const uint64_t n = ev->len - off < win ? ev->len - off : win;
        const int rc = request(c, rlo::SHM_OP_GET, arg, off, n, nullptr);
        if (rc != RLO_OK) return rc;
        std::memcpy((uint8_t*)dst + off, c->stage, n);
    }
    return RLO_OK;
}

}  // extern "C"
