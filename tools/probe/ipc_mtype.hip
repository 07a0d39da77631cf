// Probe (VERDICT r4 "next" 1): what memory type does a hipIpc-IMPORTED mapping of an uncached allocation
// have in the importing process, on the same GPU?  The engine's cross-process parts store ring slots / bulk
// tiles through such mappings with sc1 stores + vmcnt(0) + barrier + an agent-scope counter store, and the
// owner reads its own (uncached) mapping.  That hand-off is only sound if the importer's stores cannot sit
// in its XCD's L2.
//
// exporter: allocates X (uncached, or hipMalloc with "cached"), prints its IPC handle, then a watcher
//           workgroup runs K rounds: wait for flag X[0] >= k, read the data region with sc1 loads, count
//           words != k, store the ack X[16] = k.
// importer: opens the handle and a writer workgroup runs K rounds: store k into every data word with the
//           chosen flavour, s_waitcnt vmcnt(0), barrier, one agent-scope flag store X[0] = k, then poll the
//           ack X[16] through ITS mapping (a mapping whose reads are L2-cached never sees the ack: timeout).
// local:    the same writer on the exporter's own pointer, same process, another stream (control).
//
// Flavours: 0 plain global stores, 1 sc1 (agent), 2 sc0 sc1 (system), 3 sc1 stores + agent release fence
// before the flag.  With an uncached mapping every flavour must read 0 stale words; plain stores left dirty
// in a cached (RW/NC) mapping's L2 show up as stale words at the watcher.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                              \
        }                                                                              \
    } while (0)

constexpr uint32_t kDataOff = 1024;  // words: the data region starts 4 KiB into X
constexpr uint32_t kWords = 65536;   // 256 KiB of data per round
constexpr uint64_t kTmo = 20000000;     // 0.2 s of the 100-MHz clock per wait
constexpr uint64_t kTmo0 = 1000000000;  // 10 s for the first one: the peer process may still be starting

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// out: [0] rounds completed, [1] timeouts, [2] stale words (all rounds), [3] rounds with stale words,
//      [4] max stale in one round, [5] sum of flag-wait ticks
__global__ void watch(uint32_t* X, uint32_t K, unsigned long long* out) {
    __shared__ uint32_t bad, stop;
    const int tid = threadIdx.x;
    unsigned long long stale = 0, rounds_bad = 0, maxb = 0, waits = 0, tmo = 0, done = 0;
    for (uint32_t k = 1; k <= K; k++) {
        if (tid == 0) {
            bad = 0;
            stop = 0;
            const uint64_t t0 = now();
            while (__hip_atomic_load(&X[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k) {
                if (now() - t0 > (k == 1 ? kTmo0 : kTmo)) { stop = 1; break; }
            }
            if (k > 1) waits += now() - t0;  // (the first wait is the peer's start-up)
        }
        __syncthreads();
        if (stop) { tmo++; break; }
        uint32_t c = 0;
        for (uint32_t i = tid; i < kWords; i += blockDim.x)
            c += __hip_atomic_load(&X[kDataOff + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != k;
        atomicAdd(&bad, c);
        __syncthreads();
        if (tid == 0) {
            stale += bad;
            rounds_bad += bad != 0;
            maxb = bad > maxb ? bad : maxb;
            done++;
            __hip_atomic_store(&X[16], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
    if (tid == 0) {
        out[0] = done; out[1] = tmo; out[2] = stale; out[3] = rounds_bad; out[4] = maxb; out[5] = waits;
    }
}

// out: [0] rounds completed, [1] ack timeouts, [2] sum of ack-wait ticks
template <int F>
__global__ void writer(uint32_t* X, uint32_t K, unsigned long long* out) {
    __shared__ uint32_t stop;
    const int tid = threadIdx.x;
    unsigned long long done = 0, tmo = 0, waits = 0;
    for (uint32_t k = 1; k <= K; k++) {
        for (uint32_t i = tid; i < kWords; i += blockDim.x) {
            uint32_t* p = &X[kDataOff + i];
            if (F == 0) *p = k;  // (not volatile: gfx950 lowers volatile accesses with sc0 sc1)
            else if (F == 2) __hip_atomic_store(p, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            else __hip_atomic_store(p, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            stop = 0;
            if (F == 3) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_store(&X[0], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t t0 = now();
            while (__hip_atomic_load(&X[16], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k) {
                if (now() - t0 > kTmo) { stop = 1; break; }
            }
            waits += now() - t0;
        }
        __syncthreads();
        if (stop) { tmo++; break; }
        done++;
    }
    if (tid == 0) { out[0] = done; out[1] = tmo; out[2] = waits; }
}

static void launch_writer(int f, uint32_t* X, uint32_t K, unsigned long long* out, hipStream_t s) {
    switch (f) {
        case 0: hipLaunchKernelGGL(writer<0>, dim3(1), dim3(256), 0, s, X, K, out); break;
        case 1: hipLaunchKernelGGL(writer<1>, dim3(1), dim3(256), 0, s, X, K, out); break;
        case 2: hipLaunchKernelGGL(writer<2>, dim3(1), dim3(256), 0, s, X, K, out); break;
        default: hipLaunchKernelGGL(writer<3>, dim3(1), dim3(256), 0, s, X, K, out); break;
    }
}

static const char* kFl[4] = {"plain", "sc1", "sc0sc1", "sc1+release"};

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ipc_mtype export <cached|uncached> K | import <hex> flavour K | local <cached|uncached> flavour K\n"); return 2; }
    const std::string mode = argv[1];
    const size_t bytes = (kDataOff + kWords) * 4 + 4096;
    unsigned long long* out = nullptr;
    CK(hipHostMalloc((void**)&out, 64 * 8, hipHostMallocCoherent));
    std::memset(out, 0, 64 * 8);
    if (mode == "export" || mode == "local") {
        const bool cached = std::string(argv[2]) == "cached";
        const int f = mode == "local" ? std::atoi(argv[3]) : 0;
        const uint32_t K = (uint32_t)std::atoi(argv[mode == "local" ? 4 : 3]);
        uint32_t* X = nullptr;
        if (cached) CK(hipMalloc((void**)&X, bytes));
        else CK(hipExtMallocWithFlags((void**)&X, bytes, hipDeviceMallocUncached));
        CK(hipMemset(X, 0, bytes));
        CK(hipDeviceSynchronize());
        hipStream_t sw, sr;
        CK(hipStreamCreateWithFlags(&sw, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&sr, hipStreamNonBlocking));
        hipLaunchKernelGGL(watch, dim3(1), dim3(256), 0, sw, X, K, out);
        if (mode == "export") {
            hipIpcMemHandle_t h;
            CK(hipIpcGetMemHandle(&h, X));
            std::printf("HANDLE ");
            for (size_t i = 0; i < sizeof h; i++) std::printf("%02x", ((unsigned char*)&h)[i]);
            std::printf("\n");
            std::fflush(stdout);
            CK(hipStreamSynchronize(sw));
            char line[16];
            if (!std::fgets(line, sizeof line, stdin)) {}  // the importer has exited: X may go
        } else {
            launch_writer(f, X, K, out + 8, sr);
            CK(hipStreamSynchronize(sw));
            CK(hipStreamSynchronize(sr));
        }
        std::printf("WATCH %s %s: rounds %llu timeouts %llu stale_words %llu stale_rounds %llu max_stale %llu flag_wait_us %.2f\n",
                    mode.c_str(), cached ? "cached" : "uncached", out[0], out[1], out[2], out[3], out[4],
                    out[0] > 1 ? out[5] * 0.01 / (double)(out[0] - 1) : 0.0);
        if (mode == "local")
            std::printf("WRITE local %s: rounds %llu ack_timeouts %llu ack_wait_us %.2f\n", kFl[f], out[8], out[9],
                        out[8] ? out[10] * 0.01 / (double)out[8] : 0.0);
        CK(hipFree(X));
        return 0;
    }
    if (mode == "import") {
        hipIpcMemHandle_t h;
        const char* hex = argv[2];
        for (size_t i = 0; i < sizeof h; i++) {
            unsigned v = 0;
            std::sscanf(hex + 2 * i, "%2x", &v);
            ((unsigned char*)&h)[i] = (unsigned char)v;
        }
        const int f = std::atoi(argv[3]);
        const uint32_t K = (uint32_t)std::atoi(argv[4]);
        uint32_t* X = nullptr;
        CK(hipIpcOpenMemHandle((void**)&X, h, hipIpcMemLazyEnablePeerAccess));
        launch_writer(f, X, K, out, 0);
        CK(hipDeviceSynchronize());
        std::printf("WRITE import %s: rounds %llu ack_timeouts %llu ack_wait_us %.2f\n", kFl[f], out[0], out[1],
                    out[0] ? out[2] * 0.01 / (double)out[0] : 0.0);
        CK(hipIpcCloseMemHandle(X));
        return 0;
    }
    return 2;
}
