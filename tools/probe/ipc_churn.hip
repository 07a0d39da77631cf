// Probe (VERDICT r4 "next" 1, second suspect): the create -> export -> import -> run -> close -> free churn of
// the cross-process rehearsals, without the engine.  Does a store through a FRESH hipIpc import (whose virtual
// range may be the one a just-closed import used) always land in the exporter's CURRENT allocation?
//
// exporter, R rounds: allocate X_r (uncached, S bytes), zero it, print its IPC handle, wait for the importer's
//   "written" line, then a checker kernel reads every 16-B granule with sc1 loads and counts the granules that
//   differ from pattern(r, g); X_r is freed and the next round allocates again (same VA / pages come back).
// importer, R rounds: read a handle, open it, a writer kernel (many workgroups) stores pattern(r, g) into every
//   granule with the chosen flavour, hipDeviceSynchronize, close the import, print "written".
// A stale translation or mapping in the importer shows up as granules of X_r that never got their pattern.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            std::exit(2);                                                                            \
        }                                                                                            \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 pattern(uint32_t r, uint64_t g) {
    const uint32_t a = (uint32_t)g * 2654435761u ^ (r * 40503u + 1u);
    return u32x4{a, (uint32_t)(g >> 32) ^ r, a ^ 0x5A5A5A5Au, r + 1u};
}

template <int F>
__global__ void writer(u32x4* X, uint64_t ngr, uint32_t r) {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < ngr; g += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = pattern(r, g);
        if (F == 0) X[g] = v;
        else __builtin_nontemporal_store(v, &X[g]);
    }
}

__global__ void checker(const u32x4* X, uint64_t ngr, uint32_t r, unsigned long long* bad, unsigned long long* first) {
    unsigned long long c = 0;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < ngr; g += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(&X[g]);
        const u32x4 w = pattern(r, g);
        if (v.x != w.x || v.y != w.y || v.z != w.z || v.w != w.w) {
            c++;
            atomicMin(first, (unsigned long long)g);
        }
    }
    if (c) atomicAdd(bad, c);
}

int main(int argc, char** argv) {
    if (argc < 4) { std::fprintf(stderr, "usage: ipc_churn export R MiB | import R flavour\n"); return 2; }
    const std::string mode = argv[1];
    const int R = std::atoi(argv[2]);
    char line[512];
    if (mode == "export") {
        const uint64_t bytes = (uint64_t)std::atoi(argv[3]) << 20, ngr = bytes / 16;
        unsigned long long* out = nullptr;
        CK(hipHostMalloc((void**)&out, 64, hipHostMallocCoherent));
        unsigned long long total_bad = 0;
        int bad_rounds = 0;
        for (int r = 0; r < R; r++) {
            void* X = nullptr;
            CK(hipExtMallocWithFlags(&X, bytes, hipDeviceMallocUncached));
            CK(hipMemset(X, 0, bytes));
            CK(hipDeviceSynchronize());
            hipIpcMemHandle_t h;
            CK(hipIpcGetMemHandle(&h, X));
            std::printf("HANDLE %llu ", (unsigned long long)ngr);
            for (size_t i = 0; i < sizeof h; i++) std::printf("%02x", ((unsigned char*)&h)[i]);
            std::printf("\n");
            std::fflush(stdout);
            if (!std::fgets(line, sizeof line, stdin)) return 3;
            out[0] = 0;
            out[1] = ~0ull;
            hipLaunchKernelGGL(checker, dim3(1024), dim3(256), 0, 0, (const u32x4*)X, ngr, (uint32_t)r, out, out + 1);
            CK(hipDeviceSynchronize());
            if (out[0]) {
                bad_rounds++;
                std::fprintf(stderr, "round %d: %llu of %llu granules stale, first %llu (X %p)\n", r, out[0],
                             (unsigned long long)ngr, out[1], X);
            }
            total_bad += out[0];
            CK(hipFree(X));
        }
        std::printf("CHURN rounds %d bad_rounds %d stale_granules %llu\n", R, bad_rounds, total_bad);
        return 0;
    }
    const int f = std::atoi(argv[3]);
    for (int r = 0; r < R; r++) {
        if (!std::fgets(line, sizeof line, stdin)) return 3;
        unsigned long long ngr = 0;
        char hex[300] = {0};
        if (std::sscanf(line, "HANDLE %llu %299s", &ngr, hex) != 2) return 4;
        hipIpcMemHandle_t h;
        for (size_t i = 0; i < sizeof h; i++) {
            unsigned v = 0;
            std::sscanf(hex + 2 * i, "%2x", &v);
            ((unsigned char*)&h)[i] = (unsigned char)v;
        }
        void* X = nullptr;
        CK(hipIpcOpenMemHandle(&X, h, hipIpcMemLazyEnablePeerAccess));
        if (f == 0) hipLaunchKernelGGL(writer<0>, dim3(2048), dim3(256), 0, 0, (u32x4*)X, (uint64_t)ngr, (uint32_t)r);
        else hipLaunchKernelGGL(writer<1>, dim3(2048), dim3(256), 0, 0, (u32x4*)X, (uint64_t)ngr, (uint32_t)r);
        CK(hipDeviceSynchronize());
        CK(hipIpcCloseMemHandle(X));
        std::printf("written %d %p\n", r, X);
        std::fflush(stdout);
    }
    return 0;
}
