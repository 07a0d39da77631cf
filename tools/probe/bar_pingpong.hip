// Probe: round trip host -> kernel -> host, the drop-in's command path in isolation.  The host
// stores i into a command word, a one-wave kernel polling that word answers i into coherent host
// memory, the host waits for the answer.  Variants: the command word in uncached VRAM written
// through the BAR (what rlo_host_proxy does), the same plus an HDP flush after the store, and the
// word in pinned host memory (the kernel polls over PCIe).  The host thread is pinned to a given
// CPU (argv[1], -1 = unpinned) so socket placement can be compared.  Prints a latency histogram.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void echo(const unsigned long long* cmd, unsigned long long* ack, unsigned long long n, unsigned long long* out) {
    if (threadIdx.x != 0) return;
    unsigned long long polls = 0, timeouts = 0;
    for (unsigned long long i = 1; i <= n; i++) {
        unsigned long long spin = 0;
        while (__hip_atomic_load(cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < i) {
            polls++;
            if (++spin > (1ull << 24)) { timeouts++; break; }  // every wave reaches the exit
        }
        __hip_atomic_store(ack, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    out[0] = polls;
    out[1] = timeouts;
}

// ack: where the kernel answers (nullptr: coherent hipHostMalloc); flush: clflush the line before each read
static void run(const char* name, unsigned long long* cmd, volatile unsigned* hdp, int n, unsigned long long* ack_host = nullptr,
                unsigned long long* ack_dev = nullptr, bool flush = false) {
    unsigned long long *ack = ack_host, *out = nullptr;
    if (!ack) hipHostMalloc((void**)&ack, 4096, hipHostMallocCoherent | hipHostMallocMapped);
    unsigned long long* dack = ack_dev ? ack_dev : ack;
    hipHostMalloc((void**)&out, 4096, hipHostMallocCoherent | hipHostMallocMapped);
    *ack = 0;
    __atomic_store_n(cmd, 0ull, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    if (hdp) *hdp = 1u;
    hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, 0, cmd, dack, (unsigned long long)n, out);
    std::vector<double> us(n);
    bool lost = false;
    for (int i = 1; i <= n && !lost; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(cmd, (unsigned long long)i, __ATOMIC_RELEASE);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        if (hdp) *hdp = 1u;
        for (;;) {
            if (flush) { _mm_clflush(ack); _mm_mfence(); }
            if (__atomic_load_n(ack, __ATOMIC_ACQUIRE) >= (unsigned long long)i) break;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) { lost = true; break; }
        }
        us[i - 1] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    if (lost) __atomic_store_n(cmd, ~0ull >> 1, __ATOMIC_RELEASE);  // let the kernel finish
    hipDeviceSynchronize();
    std::vector<double> s = us;
    std::sort(s.begin(), s.end());
    const double edges[] = {5, 10, 20, 50, 100, 200, 500, 1000};
    int hist[9] = {};
    for (double x : us) {
        int b = 0;
        while (b < 8 && x >= edges[b]) b++;
        hist[b]++;
    }
    printf("%-34s cpu %2d: p50 %7.1f p90 %7.1f p99 %7.1f max %8.1f us | <5 %d <10 %d <20 %d <50 %d <100 %d <200 %d <500 %d <1000 %d >=1000 %d | "
           "kernel polls %llu timeouts %llu%s\n",
           name, sched_getcpu(), s[n / 2], s[(int)(n * 0.9)], s[(int)(n * 0.99)], s[n - 1], hist[0], hist[1], hist[2], hist[3],
           hist[4], hist[5], hist[6], hist[7], hist[8], out[0], out[1], lost ? " LOST" : "");
    fflush(stdout);
    if (!ack_host) hipHostFree(ack);
    hipHostFree(out);
}

int main(int argc, char** argv) {
    const int cpu = argc > 1 ? atoi(argv[1]) : -1;
    const int n = argc > 2 ? atoi(argv[2]) : 5000;
    if (cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpu, &set);
        if (sched_setaffinity(0, sizeof set, &set) != 0) printf("affinity to cpu %d failed\n", cpu);
    }
    unsigned* hdp = nullptr;
    hipError_t he = hipDeviceGetAttribute(reinterpret_cast<int*>(&hdp), hipDeviceAttributeHdpMemFlushCntl, 0);
    printf("hdp flush register: %s %p\n", hipGetErrorString(he), (void*)hdp);
    unsigned long long *u = nullptr, *h = nullptr;
    if (hipExtMallocWithFlags((void**)&u, 4096, hipDeviceMallocUncached) != hipSuccess) { printf("uncached alloc failed\n"); return 1; }
    hipHostMalloc((void**)&h, 4096, hipHostMallocCoherent | hipHostMallocMapped);
    run("uncached VRAM via BAR", u, nullptr, n);
    if (he == hipSuccess && hdp) run("uncached VRAM via BAR + HDP flush", u, hdp, n);
    run("pinned host memory", h, nullptr, n);
    // the drop-in's event region: a POSIX shm segment registered with HIP
    for (int reg = 0; reg < 2; reg++) {
        char name[64];
        snprintf(name, sizeof name, "/rlo_probe_%d_%d", (int)getpid(), reg);
        int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, 1 << 20) != 0) { printf("shm failed\n"); return 1; }
        void* p = mmap(nullptr, 1 << 20, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        shm_unlink(name);
        memset(p, 0, 1 << 20);
        unsigned flags = hipHostRegisterMapped | (reg == 0 ? hipExtHostRegisterUncached : 0u);
        hipError_t e = hipHostRegister(p, 1 << 20, flags);
        void* dp = nullptr;
        if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, p, 0);
        if (e != hipSuccess) { printf("register failed: %s\n", hipGetErrorString(e)); return 1; }
        unsigned long long* a = (unsigned long long*)((char*)p + 4096);
        unsigned long long* da = (unsigned long long*)((char*)dp + 4096);
        run(reg == 0 ? "shm registered uncached" : "shm registered default", u, nullptr, n, a, da, false);
        run(reg == 0 ? "shm registered uncached + clflush" : "shm registered default + clflush", u, nullptr, n, a, da, true);
        hipHostUnregister(p);
        munmap(p, 1 << 20);
    }
    run("uncached VRAM via BAR (again)", u, nullptr, n);
    return 0;
}
