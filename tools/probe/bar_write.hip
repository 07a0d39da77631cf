// Probe: can the CPU store into fine-grained device memory (host-visible VRAM through the BAR),
// and how fast does a kernel polling that word see it?  Used to decide where the host-service
// command counters live.  Prints one line per variant.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void spin(volatile unsigned long long* flag, unsigned long long want, unsigned long long* out) {
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), n = 0;
    while (__hip_atomic_load((unsigned long long*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
        if (++n > (1ull << 22)) break;
    }
    out[0] = __builtin_amdgcn_s_memrealtime() - t0;
    out[1] = n;
}

static void run(const char* name, unsigned long long* flag, bool host_ptr_ok) {
    unsigned long long* out;
    hipHostMalloc((void**)&out, 64, hipHostMallocCoherent);
    if (!host_ptr_ok) { printf("%s: no host pointer\n", name); return; }
    *flag = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, 0, flag, 77ull, out);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    auto t = std::chrono::steady_clock::now();
    __atomic_store_n(flag, 77ull, __ATOMIC_RELEASE);
    hipError_t e = hipDeviceSynchronize();
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
    // polls per us of kernel time: the round-trip cost of one poll of this memory
    printf("%s: sync %s, host->kernel-exit %.1f us, kernel %.1f us, polls %llu (%.3f us/poll)\n", name, hipGetErrorString(e),
           us, out[0] * 0.01, out[1], out[1] ? out[0] * 0.01 / out[1] : 0.0);
}

int main() {
    unsigned long long *h = nullptr, *d = nullptr;
    hipHostMalloc((void**)&h, 4096, hipHostMallocCoherent | hipHostMallocMapped);
    run("pinned host memory (coherent)", h, true);
    hipError_t e = hipExtMallocWithFlags((void**)&d, 4096, hipDeviceMallocFinegrained);
    printf("finegrained vram alloc: %s\n", hipGetErrorString(e));
    fflush(stdout);
    run("fine-grained VRAM, CPU store through BAR", d, e == hipSuccess);
    unsigned long long* u = nullptr;
    e = hipExtMallocWithFlags((void**)&u, 4096, hipDeviceMallocUncached);
    printf("uncached vram alloc: %s\n", hipGetErrorString(e));
    fflush(stdout);
    run("uncached VRAM, CPU store through BAR", u, e == hipSuccess);
    return 0;
}
