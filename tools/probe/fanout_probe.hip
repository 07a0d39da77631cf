// Fan-out copy probe for the bulk movers (rlo_kernel.hip mover_run, GATHER): G workgroups of 256 threads
// each read 64-KiB tiles of a source (16 B per lane, sc1) and store every tile into F destinations
// (sc1), the movers' access pattern.  Reports GB/s of (1 + F) x bytes per launch and per workgroup, for
// uncached (hipDeviceMallocUncached, the heap's memory type) and default memory, and three loop shapes:
//   0  batch of D loads, then its stores to every destination, next batch (the movers' loop);
//   1  the next batch's loads issued before this batch's stores (software pipelined);
//   2  like 0 with every destination's stores of a tile issued from one unrolled batch of 2 D.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/fanout_probe tools/probe/fanout_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kT = 256;
constexpr uint32_t kTile = 64u << 10;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs_of(void* p) {
    // the pointer made wave-uniform: a VGPR resource would wrap every access in a waterfall loop
    const uint64_t v = (uint64_t)p;
    const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ u32x4 ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

template <int MODE, int D>
__global__ __launch_bounds__(kT) void fanout(uint8_t* src, uint8_t* const* dst, int F, uint32_t tiles_per_wg) {
    const __amdgpu_buffer_rsrc_t rs = rs_of(src);
    const int tid = threadIdx.x;
    constexpr uint32_t ngr = kTile / 16u;
    for (uint32_t t = 0; t < tiles_per_wg; t++) {
        const uint32_t off0 = (blockIdx.x * tiles_per_wg + t) * kTile;
        if constexpr (MODE == 1) {
            u32x4 a[D], b[D];
#pragma unroll
            for (int u = 0; u < D; u++) a[u] = ld(rs, off0 + 16u * (u * kT + tid));
            for (uint32_t g0 = 0; g0 < ngr; g0 += D * kT) {
                const bool more = g0 + D * kT < ngr;
                if (more) {
#pragma unroll
                    for (int u = 0; u < D; u++) b[u] = ld(rs, off0 + 16u * (g0 + D * kT + u * kT + tid));
                }
                for (int f = 0; f < F; f++) {
                    const __amdgpu_buffer_rsrc_t rd = rs_of(dst[f]);
#pragma unroll
                    for (int u = 0; u < D; u++) st(rd, off0 + 16u * (g0 + u * kT + tid), a[u]);
                }
#pragma unroll
                for (int u = 0; u < D; u++) a[u] = b[u];
            }
        } else {
            constexpr int DD = MODE == 2 ? 2 * D : D;
            for (uint32_t g0 = 0; g0 < ngr; g0 += DD * kT) {
                u32x4 v[DD];
#pragma unroll
                for (int u = 0; u < DD; u++) v[u] = ld(rs, off0 + 16u * (g0 + u * kT + tid));
                for (int f = 0; f < F; f++) {
                    const __amdgpu_buffer_rsrc_t rd = rs_of(dst[f]);
#pragma unroll
                    for (int u = 0; u < DD; u++) st(rd, off0 + 16u * (g0 + u * kT + tid), v[u]);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

template <int MODE>
static float run_mode(uint8_t* src, uint8_t* const* dd, int F, int G, uint32_t tpw) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < 3; it++) {
        (void)hipEventRecord(a);
        fanout<MODE, 8><<<G, kT>>>(src, dd, F, tpw);
        (void)hipEventRecord(b);
        if (hipEventSynchronize(b) != hipSuccess) { std::printf("launch failed\n"); std::exit(1); }
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const int F = 6;
    const size_t bytes = (size_t)248 * 4 * kTile;  // 62 MiB per buffer: 248 workgroups x 4 tiles
    for (int uc = 1; uc >= 0; uc--) {
        uint8_t* buf[1 + F];
        for (int i = 0; i <= F; i++) {
            hipError_t e = uc ? hipExtMallocWithFlags((void**)&buf[i], bytes, hipDeviceMallocUncached) : hipMalloc(&buf[i], bytes);
            if (e != hipSuccess) { std::printf("alloc failed\n"); return 1; }
            (void)hipMemset(buf[i], i, bytes);
        }
        uint8_t** dd = nullptr;
        (void)hipMalloc(&dd, sizeof(uint8_t*) * F);
        (void)hipMemcpy(dd, buf + 1, sizeof(uint8_t*) * F, hipMemcpyHostToDevice);
        (void)hipDeviceSynchronize();
        for (int G : {16, 64, 124, 248}) {
            const uint32_t tpw = (uint32_t)(bytes / kTile / G);
            const double moved = (double)G * tpw * kTile * (1 + F);
            const float m0 = run_mode<0>(buf[0], dd, F, G, tpw), m1 = run_mode<1>(buf[0], dd, F, G, tpw),
                        m2 = run_mode<2>(buf[0], dd, F, G, tpw);
            std::printf("%s G %3d: batch %7.1f GB/s (%5.1f per WG) | pipelined %7.1f (%5.1f) | batch x2 %7.1f (%5.1f)\n",
                        uc ? "uncached" : "default ", G, moved / (m0 * 1e6), moved / (m0 * 1e6) / G, moved / (m1 * 1e6),
                        moved / (m1 * 1e6) / G, moved / (m2 * 1e6), moved / (m2 * 1e6) / G);
        }
        for (int i = 0; i <= F; i++) (void)hipFree(buf[i]);
        (void)hipFree(dd);
    }
    return 0;
}
