// rlo_bulk.hip -- large-message rootless bcast (BASELINE configs[2]).
//
// The reference caps a message at 32,764 B (rootless_ops.c:1475, :1588); megabyte messages
// need segmentation.  A bulk bcast from any originator o moves S bytes to every other rank as a
// pipelined scatter + all-gather over the ranks' receive buffers in HBM (peer HBM over xGMI when
// the ranks sit on different GPUs):
//   * the message is cut into chunks; chunk c is cut into N-1 stripes, stripe k owned by the
//     k-th non-originator (o + 1 + k) mod N;
//   * scatter: the originator's workgroups store stripe k of chunk c straight into its owner's
//     buffer, then every workgroup bumps the owner's scatter flag of chunk c;
//   * all-gather: an owner whose scatter flag of chunk c is complete stores its stripe into the
//     buffers of the N-2 other non-originators and bumps their gather flags of chunk c.
// Each GPU pair's link then carries S/(N-1) per direction per phase instead of the whole message
// on every tree edge, and consecutive chunks' phases overlap.  Parity for a bulk bcast is
// byte-exact delivery to all N-1 ranks (tests/test_gpu_bulk.py).
//
// Memory ordering (MI355X_MICROARCH.md "Valid forms", first bullet, at system scope): every
// handed-off byte is stored sc0 sc1 and every storing wave drains vmcnt(0) before its workgroup
// barrier; wave 0 then runs a system release (+ explicit vmcnt(0)) and one lane per destination
// adds to the flag with a system-scope atomic.  A receiver polls with one lane, runs a system
// acquire, joins a barrier, and every wave loads the bytes (sc0 sc1).  Buffers are allocated
// uncached.  Work is split in 1-KiB blocks so that a wave's destination is uniform.
#include <hip/hip_runtime.h>

#include "rlo_device.hpp"

namespace rlo {

typedef uint32_t b32x4 __attribute__((ext_vector_type(4)));
static constexpr int kSys = 1 | 16;  // sc0 | sc1
static constexpr int kUnroll = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t bk_rsrc(void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}

// wait until *p >= target (one lane); bounded by the launch deadline and the error word
__device__ bool bk_wait(uint32_t* p, uint32_t target, uint64_t deadline, uint32_t* err) {
    uint32_t spins = 0;
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
        __builtin_amdgcn_s_sleep(1);
        if ((++spins & 255u) == 0 &&
            (__builtin_amdgcn_s_memrealtime() > deadline ||
             __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
    }
    return true;
}

// System-scope release / acquire around the flags (MI355X_MICROARCH.md "Valid forms", first
// bullet; the sc1-loads-instead-of-acquire form is measured for hipMalloc memory and agent-scope
// flags only, while these buffers are uncached and the flags system scope).  The wait after the
// release is explicit: the compiler may drop it (same section, "Compiler hazard").
__device__ __forceinline__ void bk_release() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void bk_acquire() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(256) void rlo_bulk_kernel(BulkParams P) {
    __shared__ uint32_t ok;
    const int me = P.rank_begin + (int)blockIdx.y, tid = threadIdx.x, lane = tid & 63;
    const int n = P.n, o = P.origin;
    const uint32_t B = gridDim.x, b = blockIdx.x;
    const uint32_t gw = b * 4u + (uint32_t)(tid >> 6), nw = B * 4u;  // global wave id / count
    const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + P.deadline_ticks;
    const __amdgpu_buffer_rsrc_t rme = bk_rsrc(P.buf[me], P.buf_bytes);
    const uint32_t slen = P.stripe;
    const int kme = (me - o - 1 + n) % n;  // my stripe index (non-originators)
    if (tid == 0) ok = 1;
    __syncthreads();

    for (uint32_t c = 0; c < P.nchunks; c++) {
        const uint64_t c0 = (uint64_t)c * P.chunk;
        const uint32_t clen = (uint32_t)min<uint64_t>(P.chunk, P.bytes - c0);
        if (me == o) {  // ---- scatter: block kb of the chunk goes to the owner of its stripe
            const uint32_t nblk = (clen + kBulkBlock - 1) / kBulkBlock;
            for (uint32_t kb0 = gw; kb0 < nblk; kb0 += nw * kUnroll) {
                b32x4 v[kUnroll];
#pragma unroll
                for (int u = 0; u < kUnroll; u++) {
                    const uint32_t kb = kb0 + (uint32_t)u * nw, off = kb * kBulkBlock + 16u * lane;
                    if (kb < nblk && off < clen)
                        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rme, (uint32_t)(c0 + off), 0, 0);
                }
#pragma unroll
                for (int u = 0; u < kUnroll; u++) {
                    const uint32_t kb = kb0 + (uint32_t)u * nw, off = kb * kBulkBlock + 16u * lane;
                    if (kb >= nblk) break;  // uniform
                    const int owner = (o + 1 + (int)(kb * kBulkBlock / slen)) % n;
                    const __amdgpu_buffer_rsrc_t rd = bk_rsrc(P.buf[owner], P.buf_bytes);
                    if (off < clen) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)(c0 + off), 0, kSys);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid < 64) {  // wave 0 releases, then one lane per owner: this workgroup's share has landed
                bk_release();
                if (tid < n - 1) {
                    const int owner = (o + 1 + tid) % n;
                    __hip_atomic_fetch_add(&P.sflag[owner][c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        } else {  // ---- all-gather: my stripe of chunk c, once the originator delivered it
            if (tid == 0) {
                if (!bk_wait(&P.sflag[me][c], B, deadline, P.err)) ok = 0;
                bk_acquire();
            }
            __syncthreads();
            if (!ok) break;
            const uint32_t s0 = (uint32_t)kme * slen;
            const uint32_t s1 = min(s0 + slen, clen);
            const uint32_t nblk = s1 > s0 ? (s1 - s0 + kBulkBlock - 1) / kBulkBlock : 0u;
            for (uint32_t kb0 = gw; kb0 < nblk; kb0 += nw * kUnroll) {
                b32x4 v[kUnroll];
#pragma unroll
                for (int u = 0; u < kUnroll; u++) {
                    const uint32_t kb = kb0 + (uint32_t)u * nw, off = s0 + kb * kBulkBlock + 16u * lane;
                    if (kb < nblk && off < s1)
                        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rme, (uint32_t)(c0 + off), 0, kSys);
                }
                for (int d = 1; d < n; d++) {  // every other non-originator (uniform)
                    const int dst = (o + d) % n;
                    if (dst == me) continue;
                    const __amdgpu_buffer_rsrc_t rd = bk_rsrc(P.buf[dst], P.buf_bytes);
#pragma unroll
                    for (int u = 0; u < kUnroll; u++) {
                        const uint32_t kb = kb0 + (uint32_t)u * nw, off = s0 + kb * kBulkBlock + 16u * lane;
                        if (kb < nblk && off < s1)
                            __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)(c0 + off), 0, kSys);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid < 64) {
                bk_release();
                if (tid < n - 1) {
                    const int dst = (o + 1 + tid) % n;
                    if (dst != me)
                        __hip_atomic_fetch_add(&P.gflag[dst][c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
    // delivery complete at this rank: every other owner's stripe of every chunk (workgroup 0)
    if (me != o && b == 0 && tid == 0 && ok) {
        const uint32_t want = B * (uint32_t)(n - 2);
        for (uint32_t c = 0; c < P.nchunks; c++)
            if (!bk_wait(&P.gflag[me][c], want, deadline, P.err)) break;
    }
}

}  // namespace rlo

extern "C" hipError_t rlo_launch_bulk(const rlo::BulkParams* p, int blocks, int local_ranks, hipStream_t stream) {
    hipLaunchKernelGGL(rlo::rlo_bulk_kernel, dim3(blocks, local_ranks), dim3(256), 0, stream, *p);
    return hipGetLastError();
}
