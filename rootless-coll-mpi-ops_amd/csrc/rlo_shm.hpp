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
//   header page | hctl [nl][kHctlWords] (device-written counters) | ev [nl][pk_cap] LogRec |
//   evp [nl][pk_cap][max_payload] | cli [nl] ClientBox | cmd [nl][cmd_cap][stride] |
//   stage [nl][stage_bytes]
// The leader registers the whole segment with HIP (the kernel writes hctl / ev / evp; the proxy
// DMAs bulk bytes through stage).  A client writes its commands into `cmd` and its counters into
// its ClientBox; the leader's proxy (rlo_host_proxy) moves commands into the part's VRAM command
// ring and the pickup head into the VRAM counter the kernel polls, and runs bulk copies between
// `stage` and the heap on the client's behalf.
#pragma once
#include <cstddef>
#include <cstdint>

#include "rlo_device.hpp"

namespace rlo {

constexpr uint32_t kShmMagic = 0x534f4c52u;  // "RLOS"
constexpr uint32_t kShmVersion = 4;

// a bulk origination: ACQUIRE (the next bulk sequence q, once its heap slot is free; q is not taken
// yet), PUT the bytes window by window, COMMIT q (taken: the announcement carries it).  A failed PUT
// leaves q free for the next attempt, so no heap slot is ever lost to a half-staged message
enum ShmOp : uint32_t { SHM_OP_NONE = 0, SHM_OP_ACQUIRE = 1, SHM_OP_PUT = 2, SHM_OP_GET = 3, SHM_OP_COMMIT = 4 };

struct ShmHdr {
    uint32_t magic, version;
    uint32_t nl, rb;                 // local ranks of the part, first world rank
    uint32_t n, bslots;              // world size, bulk heap slots per (receiver, origin)
    uint32_t cmd_cap, pk_cap;        // ring capacities per rank
    uint32_t stride, max_payload;    // command slot stride, pickup payload stride
    uint64_t bulk_max, stage_bytes;  // bulk message cap; staging window per rank
    uint64_t off_hctl, off_ev, off_evp, off_cli, off_cmd, off_stage, total;
    uint64_t off_llc;                // command doorbells [nl][cmd_cap] x kLLCmdSlot (ll_cmd_put)
    uint32_t leader_failed, pad;     // the leader gave up (its kernel could not start / ended early)
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

inline ShmLayout shm_layout(uint32_t nl, uint32_t cmd_cap, uint32_t pk_cap, uint32_t stride, uint32_t max_payload,
                            uint64_t stage_bytes) {
    ShmLayout L;
    uint64_t o = 4096;  // header page
    L.hctl = o; o = shm_page(o + (uint64_t)nl * kHctlWords * 8);
    L.ev = o; o = shm_page(o + (uint64_t)nl * pk_cap * sizeof(LogRec));
    L.evp = o; o = shm_page(o + (uint64_t)nl * pk_cap * max_payload);
    L.cli = o; o = shm_page(o + (uint64_t)nl * sizeof(ClientBox));
    L.cmd = o; o = shm_page(o + (uint64_t)nl * cmd_cap * stride);
    L.stage = o; o = shm_page(o + (uint64_t)nl * stage_bytes);
    L.llc = o; o = shm_page(o + (uint64_t)nl * cmd_cap * kLLCmdSlot);
    L.total = o;
    return L;
}

}  // namespace rlo
