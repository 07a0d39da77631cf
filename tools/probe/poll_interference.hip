// Probe (round 5): does one wave's polling of pinned host memory slow another wave's VRAM loads on the same CU?
// (The host service's wave 1 polls the command doorbell over PCIe while wave 0 polls its VRAM bells: the host hop
// profile showed wave 0's bell loads ~1 us slower with the poller on.)  Wave 0 times dependent 16-B loads of
// uncached VRAM while wave 1 (a) idles, (b) polls host memory with vector loads (16 lanes x 16 B, the doorbell's
// shape), (c) polls it with scalar loads (s_load_dwordx2 glc: the scalar data path), and reports how many distinct
// values of a word the CPU keeps incrementing it saw (so the scalar poll is known to see fresh data).
//   hipcc --offload-arch=gfx950 -O2 poll_interference.hip -o poll_interference
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                         \
        }                                                                                         \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t s_load_glc(const uint64_t* p) {
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n s_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

__global__ void probe(const v4u* vram, const v4u* host, const uint64_t* hword, int mode, int n, uint64_t* out) {
    __shared__ int done;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (w == 0) {
        uint32_t acc = 0;
        const uint64_t t0 = wall_clock64();
        for (int i = 0; i < n; i++) {
            v4u v = {0u, 0u, 0u, 0u};
            if (lane < 16) v = __builtin_nontemporal_load(vram + lane + (acc & 1u) * 16);
            acc += (uint32_t)__shfl((int)v.x, 0) + 1u;
        }
        const uint64_t t1 = wall_clock64();
        if (lane == 0) {
            out[0] = t1 - t0;
            out[3] = acc;
            __hip_atomic_store(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else {
        uint64_t polls = 0, distinct = 0, last = ~0ull, acc = 0;
        while (!__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            if (mode == 1) {
                v4u v = {0u, 0u, 0u, 0u};
                if (lane < 16) v = __builtin_nontemporal_load(host + lane);
                acc += (uint32_t)__shfl((int)v.x, 0);
                const uint64_t x = __hip_atomic_load(hword, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (x != last) { distinct++; last = x; }
            } else if (mode == 2) {
                const uint64_t x = s_load_glc(hword);
                if (x != last) { distinct++; last = x; }
            } else {
                __builtin_amdgcn_s_sleep(8);
            }
            polls++;
        }
        if (lane == 0) { out[1] = polls; out[2] = distinct; out[4] = acc; }
    }
}

int main() {
    const int n = 4000;
    v4u *vram = nullptr;
    CK(hipExtMallocWithFlags((void**)&vram, 4096, hipDeviceMallocUncached));
    CK(hipMemset(vram, 0, 4096));
    uint64_t* h = nullptr;
    CK(hipHostMalloc((void**)&h, 8192, hipHostMallocCoherent | hipHostMallocMapped));
    for (int i = 0; i < 1024; i++) h[i] = 0;
    uint64_t* dh = nullptr;
    CK(hipHostGetDevicePointer((void**)&dh, h, 0));
    uint64_t* out = nullptr;
    CK(hipHostMalloc((void**)&out, 64, hipHostMallocCoherent));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    std::atomic<bool> stop{false};
    std::atomic<uint64_t>* word = reinterpret_cast<std::atomic<uint64_t>*>(h + 512);
    std::thread bump([&] {
        uint64_t i = 0;
        while (!stop.load(std::memory_order_relaxed)) {
            word->store(++i, std::memory_order_release);
            const auto t = std::chrono::steady_clock::now() + std::chrono::microseconds(2);
            while (std::chrono::steady_clock::now() < t) {
            }
        }
    });
    const char* names[3] = {"wave 1 idle", "wave 1 polls host memory, vector loads", "wave 1 polls host memory, scalar loads (glc)"};
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 3; mode++) {
            for (int k = 0; k < 8; k++) out[k] = 0;
            hipLaunchKernelGGL(probe, dim3(1), dim3(128), 0, 0, vram, reinterpret_cast<const v4u*>(dh), dh + 512, mode, n, out);
            CK(hipDeviceSynchronize());
            std::printf("%-46s: wave 0 VRAM load round trip %.3f us; wave 1 polls %llu, distinct host values seen %llu\n",
                        names[mode], out[0] * 1e3 / khz / n, (unsigned long long)out[1], (unsigned long long)out[2]);
        }
    stop = true;
    bump.join();
    return 0;
}
