/*
 * rlo_testvec.h -- TEST INFRASTRUCTURE ONLY (oracle side).
 *
 * Definition of the synthetic workloads shared by the reference harness
 * (oracle/ref_harness.c, linked against the compiled reference), the CPU
 * restatement (oracle/rlo_oracle.c) and the tests.  The product keeps its
 * own device implementation of the same generator
 * (rootless-coll-mpi-ops_amd/csrc/rlo_device.hpp) -- it never includes this.
 *
 *   storm payload  : word0 = (bid << 32) | origin ; word k>=1 =
 *                    splitmix64(word0 ^ (k * GOLDEN)) ; little endian,
 *                    truncated to len bytes.
 *   storm origins  : origin(b) = splitmix64(seed + b) % N
 *   data hash      : FNV-1a 64 over the 32,764-byte data region the reference
 *                    delivers (payload followed by zero bytes).
 */
#ifndef RLO_TESTVEC_H
#define RLO_TESTVEC_H
#include <stdint.h>
#include <string.h>

#define RLO_TV_GOLDEN 0x9E3779B97F4A7C15ull
#define RLO_TV_DATA_REGION 32764 /* RLO_MSG_SIZE_MAX - sizeof(int): rootless_ops.c:1588 */

static inline uint64_t rlo_tv_splitmix64(uint64_t x) {
    uint64_t z = x + RLO_TV_GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t rlo_tv_word(uint32_t origin, uint32_t bid, uint32_t k) {
    uint64_t w0 = ((uint64_t)bid << 32) | (uint64_t)origin;
    if (k == 0) return w0;
    return rlo_tv_splitmix64(w0 ^ ((uint64_t)k * RLO_TV_GOLDEN));
}

static inline void rlo_tv_payload(uint32_t origin, uint32_t bid, uint8_t* out, size_t len) {
    for (size_t off = 0; off < len; off += 8) {
        uint64_t w = rlo_tv_word(origin, bid, (uint32_t)(off / 8));
        size_t n = len - off < 8 ? len - off : 8;
        memcpy(out + off, &w, n); /* little endian host */
    }
}

static inline uint32_t rlo_tv_origin(uint64_t seed, uint64_t b, uint32_t n) {
    return (uint32_t)(rlo_tv_splitmix64(seed + b) % n);
}

/* storm origins, by order: 0 random (above), 1 "slots": bcast b originates at rank b % n, so in
 * every slot of n consecutive bcasts every rank originates (BASELINE configs[4]) */
static inline uint32_t rlo_tv_origin2(uint64_t seed, uint64_t b, uint32_t n, uint32_t order) {
    return order == 1 ? (uint32_t)(b % n) : rlo_tv_origin(seed, b, n);
}

/* mixed payload sizes (BASELINE configs[4]): length of bcast b in [lo, hi], piecewise log-uniform --
 * an octave [2^e, 2^(e+1)) uniform over the octaves of [lo, hi), then uniform inside it; integer
 * only (the device's storm_len_of in rlo_device.hpp states the same) */
static inline uint32_t rlo_tv_len(uint64_t seed, uint64_t b, uint32_t lo, uint32_t hi) {
    if (hi <= lo) return lo;
    if (lo == 0) lo = 1;
    const int elo = 31 - __builtin_clz(lo), ehi = 31 - __builtin_clz(hi);
    const uint64_t x = rlo_tv_splitmix64(seed ^ 0xC5C5C5C5C5C5C5C5ull ^ (b * RLO_TV_GOLDEN));
    const uint32_t noct = (uint32_t)(ehi - elo) + ((hi & (hi - 1u)) ? 1u : 0u);
    if (noct == 0) return lo;
    const uint32_t e = (uint32_t)elo + (uint32_t)(x % noct);
    const uint64_t base = 1ull << e;
    uint64_t v = base + ((x >> 32) % base);
    if (v < lo) v = lo;
    if (v > hi) v = hi;
    return (uint32_t)v;
}

static inline uint64_t rlo_tv_fnv1a(const uint8_t* p, size_t len, uint64_t h) {
    for (size_t i = 0; i < len; i++) { h ^= p[i]; h *= 0x100000001b3ull; }
    return h;
}
#define RLO_TV_FNV_INIT 0xcbf29ce484222325ull

/* FNV-1a of (payload[0..len) ++ zeros) over the whole data region. */
static inline uint64_t rlo_tv_region_hash(const uint8_t* payload, size_t len) {
    static const uint8_t zeros[4096] = {0};
    if (len > RLO_TV_DATA_REGION) len = RLO_TV_DATA_REGION;
    uint64_t h = rlo_tv_fnv1a(payload, len, RLO_TV_FNV_INIT);
    size_t rest = RLO_TV_DATA_REGION - len;
    while (rest) { size_t n = rest < sizeof zeros ? rest : sizeof zeros; h = rlo_tv_fnv1a(zeros, n, h); rest -= n; }
    return h;
}
#endif
