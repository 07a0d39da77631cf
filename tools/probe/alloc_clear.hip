// Probe (round 5, the 8-part rehearsal's stale heap nonce): does a word written into a FRESH uncached allocation
// right after hipExtMallocWithFlags stay written?  A clear or wipe of the allocation's pages that the driver
// still runs behind the allocation would overwrite it later.  R rounds: free the previous buffers, allocate a
// "churn" buffer of C MiB (released at once: wipe-on-release work for the driver), then the big buffer of B
// MiB; write a nonce at its first and last 8 bytes (hipMemcpy H2D, synchronous), read both back at once,
// after 2 ms and after 50 ms.  Prints every round whose read-back differs.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
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

int main(int argc, char** argv) {
    const int R = argc > 1 ? std::atoi(argv[1]) : 20;
    const uint64_t big = (uint64_t)(argc > 2 ? std::atoi(argv[2]) : 4096) << 20;
    const uint64_t churn = (uint64_t)(argc > 3 ? std::atoi(argv[3]) : 1024) << 20;
    int bad = 0;
    void* prev = nullptr;
    for (int r = 0; r < R; r++) {
        if (prev) CK(hipFree(prev));
        void* c = nullptr;
        CK(hipExtMallocWithFlags(&c, churn, hipDeviceMallocUncached));
        CK(hipMemset(c, 0x5A, churn));
        CK(hipDeviceSynchronize());
        CK(hipFree(c));
        void* b = nullptr;
        CK(hipExtMallocWithFlags(&b, big, hipDeviceMallocUncached));
        const uint64_t nonce = 0x1234567800000000ull | (uint64_t)(r + 1);
        uint8_t* p0 = (uint8_t*)b;
        uint8_t* p1 = (uint8_t*)b + big - 8;
        CK(hipMemcpy(p0, &nonce, 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(p1, &nonce, 8, hipMemcpyHostToDevice));
        uint64_t g[6] = {0, 0, 0, 0, 0, 0};
        CK(hipMemcpy(&g[0], p0, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&g[1], p1, 8, hipMemcpyDeviceToHost));
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        CK(hipMemcpy(&g[2], p0, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&g[3], p1, 8, hipMemcpyDeviceToHost));
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        CK(hipMemcpy(&g[4], p0, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&g[5], p1, 8, hipMemcpyDeviceToHost));
        bool ok = true;
        for (int i = 0; i < 6; i++) ok &= g[i] == nonce;
        if (!ok) {
            bad++;
            std::printf("round %d (%p): first word now/2ms/50ms %016llx %016llx %016llx, last %016llx %016llx %016llx\n", r, b,
                        (unsigned long long)g[0], (unsigned long long)g[2], (unsigned long long)g[4], (unsigned long long)g[1],
                        (unsigned long long)g[3], (unsigned long long)g[5]);
        }
        prev = b;
    }
    std::printf("ALLOC_CLEAR rounds %d big %llu MiB churn %llu MiB: %d rounds lost a word\n", R, (unsigned long long)(big >> 20),
                (unsigned long long)(churn >> 20), bad);
    return 0;
}
