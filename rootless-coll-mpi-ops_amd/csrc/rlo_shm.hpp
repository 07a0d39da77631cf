// rlo_shm.hpp -- the shared host service: the host side of a host-service part (rlo_program_host)
// in a POSIX shared-memory segment, so that rank processes with NO HIP context of their own can
// drive their ranks of a part that another process (the GPU's leader) owns and runs.
//
// Why: a persistent kernel per rank process means one set of hardware queues per process.  Once
// more processes hold queues on a GPU than its hardware scheduler maps at once, it time-slices
// whole processes and every persistent kernel stalls for whole quanta (profiles/
// r2_probe_oversub.txt: 8 rank processes 0.42 s, 8 beside one idle torch process 1.33 s, 9 rank
// processes 38-48 s, 12 rank processes > 60 s for the same 8-rank-style iar run).  With the shared
// service exactly one process per GPU holds queues, whatever the rank count.
//
// Segment layout (page-aligned regions, sizes in the header so a client derives them):
//   header page | hctl [nl][kHctlWords] (device-written counters) | ev [nl][pk_cap] tagged records (kPkRecBytes) |
//   evp [nl][pk_cap][pickup payload stride] | cli [nl] ClientBox | cmd [nl][cmd_cap][stride] |
//   stage [nl][stage_bytes]
// The leader registers the whole segment with HIP (the kernel writes hctl / ev / evp; the proxy
// DMAs bulk bytes through stage).  A client writes its commands into `cmd` and its counters into
// its ClientBox; the leader's proxy (rlo_host_proxy) moves commands into the part's VRAM command
// ring and the pickup head into the VRAM counter the kernel polls, and runs bulk copies between
// `stage` and the heap on the client's behalf.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "rlo_device.hpp"

namespace rlo {

constexpr uint32_t kShmMagic = 0x534f4c52u;  // "RLOS"
constexpr uint32_t kShmVersion = 5;

// a bulk origination: ACQUIRE (the next bulk sequence q, once its heap slot is free; q is not taken
// yet), PUT the bytes window by window, COMMIT q (taken: the announcement carries it).  A failed PUT
// leaves q free for the next attempt, so no heap slot is ever lost to a half-staged message
enum ShmOp : uint32_t { SHM_OP_NONE = 0, SHM_OP_ACQUIRE = 1, SHM_OP_PUT = 2, SHM_OP_GET = 3, SHM_OP_COMMIT = 4 };

struct ShmHdr {
    uint32_t magic, version;
    uint32_t nl, rb;                 // local ranks of the part, first world rank
    uint32_t n, bslots;              // world size, bulk heap slots per (receiver, origin)
    uint32_t cmd_cap, pk_cap;        // ring capacities per rank
    uint32_t stride, max_payload;    // command slot stride, pickup payload stride (pk_payload_stride)
    uint64_t bulk_max, stage_bytes;  // bulk message cap; staging window per rank
    uint64_t off_hctl, off_ev, off_evp, off_cli, off_cmd, off_stage, total;
    uint64_t off_llc;                // command doorbells [nl][cmd_cap] x kLLCmdSlot (ll_cmd_put)
    uint32_t leader_failed;          // the leader gave up (its kernel could not start / ended early)
    uint32_t pk_epoch;               // the running launch's pickup-tag epoch (rlo_device.hpp pk_tag)
};

// one per local rank; the two sides' words on separate 128-byte lines.  The kernel polls mtail and
// mpk here directly (its hctl_dev words kHctlInjTail / kHctlPkHead: the box IS that array, one
// kHctlWords stride per rank), and reads the commands from `cmd` -- no CPU store into VRAM on the
// command path (see rlo_world.cpp, cmd_host)
struct ClientBox {
    alignas(128) uint64_t mtail;  // client: commands written into its `cmd` ring
    alignas(128) uint64_t req;    // client: bulk request sequence (request fields below valid)
    uint32_t op, arg;             // ShmOp; ACQUIRE -, PUT q, GET origin << 8 | heap slot, COMMIT q
    uint64_t off, len;            // byte range of the message this request moves via `stage`
    alignas(128) uint64_t ack;    // leader: last request completed
    int64_t rc;                   // RLO_OK / RLO_E_AGAIN (ACQUIRE: slot still busy) / error
    uint64_t q;                   // ACQUIRE: the bulk sequence taken
    uint64_t fwd;                 // leader (RLO_BAR_CMDS): commands forwarded into the VRAM ring
    int64_t fwd_ns;               // leader (RLO_BAR_CMDS): CLOCK_MONOTONIC ns of that forward
    alignas(128) uint64_t mpk;    // client: pickup events consumed
};
static_assert(sizeof(ClientBox) == kHctlWords * 8, "ClientBox stride = the kernel's host counter stride");
static_assert(offsetof(ClientBox, mtail) == kHctlInjTail * 8 && offsetof(ClientBox, mpk) == kHctlPkHead * 8,
              "ClientBox words where the kernel polls its command tail / pickup head");

struct ShmLayout {
    uint64_t hctl, ev, evp, cli, cmd, stage, llc, total;
};

// Command doorbells: a command of at most kBellChunks 16-B chunks (header + 112 B) is also written,
// data-tagged, into the doorbell slot of its sequence number -- the forward doorbells' format
// (rlo_device.hpp): chunk q as two LL granule pairs {d0, T, d1, T}, {d2, T, d3, T}, T = bell_tag(sequence),
// every 8-byte half one atomic CPU store.  The kernel polls the slot of the next command it expects and
// takes the command from there when every half of its chunks carries T: one PCIe read instead of a tail
// poll followed by a slot load.  The ring slot and the tail are still written (the full path and longer
// commands use them); the doorbell slot of sequence s is reused at s + cmd_cap, after the kernel consumed s
constexpr uint32_t kLLCmdSlot = kBellChunks * 32u;
inline void ll_cmd_put(uint8_t* slot, uint64_t seq, const uint32_t hdr[4], const void* payload, uint32_t len) {
    if (kHdr + len > kBellChunks * 16u) return;  // longer commands: the ring slot only
    const uint64_t T = (uint64_t)bell_tag(seq) << 32;
    uint32_t w[kBellChunks * 4] = {0};
    for (int i = 0; i < 4; i++) w[i] = hdr[i];
    if (len) __builtin_memcpy(reinterpret_cast<uint8_t*>(w) + kHdr, payload, len);
    const uint32_t nw = 4u * ((kHdr + len + 15u) / 16u);
    uint64_t* d = reinterpret_cast<uint64_t*>(slot);
    for (uint32_t i = 0; i < nw; i++) __atomic_store_n(d + i, (uint64_t)w[i] | T, __ATOMIC_RELAXED);
}

inline uint64_t shm_page(uint64_t x) { return (x + 4095u) & ~uint64_t(4095); }

// Take pickup event `seq` of one rank's ring (records `evs`, payloads `evp` at `stride`, `cap` slots) if it is whole:
// each of its record's four units carries pk_tag16(seq, epoch) (rlo_device.hpp kPkRecBytes), so does every unit of a
// tagged payload (pk_tag); a plain payload (the full path's) is read only once the published tail covers the event.
// Returns 1 (ev / payload filled, the record decoded to rlo_log_rec_t's form), 0 (not yet).
inline int pk_take(const uint8_t* evs, const uint8_t* evp, uint32_t cap, uint32_t stride, uint32_t epoch, uint64_t seq,
                   const uint64_t* pk_tail, LogRec* ev, void* payload, uint32_t pcap) {
    const uint32_t i = (uint32_t)(seq & (cap - 1));
    const uint32_t t16 = pk_tag16(seq, epoch);
    const uint64_t* r = reinterpret_cast<const uint64_t*>(evs + (uint64_t)i * kPkRecBytes);
    uint64_t u[4];
    for (int k = 0; k < 4; k++) u[k] = __atomic_load_n(r + k, __ATOMIC_ACQUIRE);
    const uint32_t w0 = (uint32_t)u[0], w2 = (uint32_t)u[1], w5 = (uint32_t)(u[2] >> 32), w7 = (uint32_t)(u[3] >> 32);
    if ((w0 >> 16) != t16 || (w2 >> 16) != t16 || (w5 >> 16) != t16 || (w7 >> 16) != t16) return 0;
    ev->kind = w0 & 0xffffu;
    ev->origin = (int32_t)(uint32_t)(u[0] >> 32);
    ev->from = (int32_t)(w2 & 0xffffu) - 1;
    ev->id = (uint32_t)(u[1] >> 32);
    ev->len = (uint32_t)u[2];
    ev->vote = (int32_t)(int16_t)(w5 & 0xffffu);
    ev->aux = (uint32_t)u[3];
    const uint32_t pidx = w7 & 0xffffu;
    ev->payload_idx = pidx == kPkNoPayload ? 0xffffffffu : (pidx & ~kPkTaggedPayload);
    if (pidx != kPkNoPayload) {
        const uint32_t n = payload && pcap ? std::min(std::min(ev->len, pcap), stride) : 0u;
        const uint8_t* src = evp + (uint64_t)i * stride;
        if (pidx & kPkTaggedPayload) {
            const uint32_t tg = pk_tag(seq, epoch);
            const uint64_t* pu = reinterpret_cast<const uint64_t*>(src);
            uint8_t* out = static_cast<uint8_t*>(payload);
            for (uint32_t k = 0; 4 * k < n; k++) {
                const uint64_t x = __atomic_load_n(pu + k, __ATOMIC_ACQUIRE);
                if ((uint32_t)(x >> 32) != tg) return 0;
                const uint32_t d = (uint32_t)x;
                std::memcpy(out + 4 * k, &d, std::min(4u, n - 4 * k));
            }
        } else {
            if (__atomic_load_n(pk_tail, __ATOMIC_ACQUIRE) <= seq) return 0;
            if (n) std::memcpy(payload, src, n);
        }
    }
    return 1;
}

inline ShmLayout shm_layout(uint32_t nl, uint32_t cmd_cap, uint32_t pk_cap, uint32_t stride, uint32_t max_payload,
                            uint64_t stage_bytes) {
    ShmLayout L;
    uint64_t o = 4096;  // header page
    L.hctl = o; o = shm_page(o + (uint64_t)nl * kHctlWords * 8);
    L.ev = o; o = shm_page(o + (uint64_t)nl * pk_cap * kPkRecBytes);  // tagged records (rlo_device.hpp pk_tag16)
    L.evp = o; o = shm_page(o + (uint64_t)nl * pk_cap * max_payload);
    L.cli = o; o = shm_page(o + (uint64_t)nl * sizeof(ClientBox));
    L.cmd = o; o = shm_page(o + (uint64_t)nl * cmd_cap * stride);
    L.stage = o; o = shm_page(o + (uint64_t)nl * stage_bytes);
    L.llc = o; o = shm_page(o + (uint64_t)nl * cmd_cap * kLLCmdSlot);
    L.total = o;
    return L;
}

}  // namespace rlo
