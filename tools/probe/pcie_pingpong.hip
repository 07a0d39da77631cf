// Probe (round 5): what a host <-> device hand-off costs on this box, the floor under the drop-in's command-in and
// pickup-out legs.  (1) ping-pong: a CPU thread writes a sequence word into pinned host memory, one GPU wave polls
// it (system-scope loads) and answers into a second word, the CPU times the round trip; (2) one wave timing its own
// load round trips to host memory: 8 B (one lane) and 256 B (16 lanes x 16 B, the command doorbell's shape), and
// to uncached VRAM for comparison.   hipcc --offload-arch=gfx950 -O2 pcie_pingpong.hip -o pcie_pingpong
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                         \
        }                                                                                         \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wave 0 answers every ping; gives up after a bounded number of polls (the CPU side never stops early)
__global__ void pong_kernel(uint64_t* ping, uint64_t* pong, int n, unsigned long long limit) {
    if (threadIdx.x != 0) return;
    unsigned long long polls = 0;
    for (int i = 1; i <= n; i++) {
        while (ld_sys(ping) != (uint64_t)i) {
            if (++polls > limit) return;
        }
        __hip_atomic_store(pong, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// load round trips measured by the wave itself: every load waited for (its value feeds the next address)
__global__ void rt_kernel(const uint64_t* host8, const v4u* host256, const v4u* dev256, int n, uint64_t* out) {
    const int lane = threadIdx.x;
    uint64_t t0, t1, acc = 0;
    t0 = wall_clock64();
    for (int i = 0; i < n; i++) {
        if (lane == 0) acc += ld_sys(host8 + (acc & 1));
        acc = __shfl(acc, 0);
    }
    t1 = wall_clock64();
    if (lane == 0) out[0] = t1 - t0;
    t0 = wall_clock64();
    for (int i = 0; i < n; i++) {
        v4u v = {0u, 0u, 0u, 0u};
        if (lane < 16) v = __builtin_nontemporal_load(host256 + lane + (acc & 1) * 16);
        acc += __shfl((int)v.x, 0);
    }
    t1 = wall_clock64();
    if (lane == 0) out[1] = t1 - t0;
    t0 = wall_clock64();
    for (int i = 0; i < n; i++) {
        v4u v = {0u, 0u, 0u, 0u};
        if (lane < 16) v = __builtin_nontemporal_load(dev256 + lane + (acc & 1) * 16);
        acc += __shfl((int)v.x, 0);
    }
    t1 = wall_clock64();
    if (lane == 0) { out[2] = t1 - t0; out[3] = acc; }
}

int main() {
    const int n = 20000;
    uint64_t* h = nullptr;
    CK(hipHostMalloc((void**)&h, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    std::fill(h, h + 512, 0ull);
    std::atomic<uint64_t>* ping = reinterpret_cast<std::atomic<uint64_t>*>(h);
    std::atomic<uint64_t>* pong = reinterpret_cast<std::atomic<uint64_t>*>(h + 64);
    uint64_t *dping = nullptr, *dpong = nullptr;
    CK(hipHostGetDevicePointer((void**)&dping, h, 0));
    dpong = dping + 64;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipLaunchKernelGGL(pong_kernel, dim3(1), dim3(64), 0, s, dping, dpong, n, 4000000000ull);
    std::vector<double> rt;
    rt.reserve(n);
    for (int i = 1; i <= n; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        ping->store((uint64_t)i, std::memory_order_release);
        const auto tl = t0 + std::chrono::seconds(2);
        while (pong->load(std::memory_order_acquire) != (uint64_t)i)
            if (std::chrono::steady_clock::now() > tl) { std::fprintf(stderr, "pong %d timed out\n", i); return 1; }
        rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CK(hipStreamSynchronize(s));
    std::sort(rt.begin(), rt.end());
    std::printf("CPU ping -> GPU wave -> CPU pong (pinned host memory): p50 %.2f us p10 %.2f p90 %.2f (one-way ~ p50/2)\n",
                rt[n / 2], rt[n / 10], rt[n * 9 / 10]);
    v4u* dv = nullptr;
    CK(hipExtMallocWithFlags((void**)&dv, 4096, hipDeviceMallocUncached));
    CK(hipMemset(dv, 0, 4096));
    uint64_t* out = nullptr;
    CK(hipHostMalloc((void**)&out, 64, hipHostMallocCoherent));
    const int m = 2000;
    hipLaunchKernelGGL(rt_kernel, dim3(1), dim3(64), 0, s, dping + 128, reinterpret_cast<const v4u*>(dping + 256), dv, m, out);
    CK(hipStreamSynchronize(s));
    int hz = 0;
    CK(hipDeviceGetAttribute(&hz, hipDeviceAttributeWallClockRate, 0));  // kHz
    const double us = 1e3 / hz;
    std::printf("wave load round trips (wall clock %d kHz): host 8 B %.2f us, host 256 B %.2f us, uncached VRAM 256 B %.2f us\n",
                hz, out[0] * us / m, out[1] * us / m, out[2] * us / m);
    return 0;
}
