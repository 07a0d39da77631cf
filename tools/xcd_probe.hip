// One hop's memory cost by placement and allocation, for the hop kernel's next step.
// Two one-wave workgroups pass a message back and forth the way the hop kernel hands one over: the
// producer stores a 16-B payload, drains, stores the counter; the consumer polls the counter with an sc1
// load, then loads the payload (sc1) and checks it.  Per configuration: the pair on one XCD (blocks 0 and
// 8; blocks are dealt round-robin over the 8 XCDs, and the XCC ids each block read are printed to show it)
// or on two; the rings' allocation (uncached, as the product's) or the default cached one; stores with
// sc1 (the product's) or plain (a plain store keeps the line in the XCD's L2, an sc1 store drops it).
// Every poll is bounded (a stale L2 line never seen to change ends the run with an error, not a hang).
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/xcd_probe tools/xcd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ u32x4 ld4_sc1(const u32x4* p) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <bool SC1>
__device__ __forceinline__ void send(uint32_t* flag, u32x4* data, uint32_t v) {
    const u32x4 m = {v, v ^ 0x5A5A5A5Au, v + 1u, ~v};
    if (SC1) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" ::"v"(data), "v"(m) : "memory");
        asm volatile("global_store_dword %0, %1, off sc1" ::"v"(flag), "v"(v) : "memory");
    } else {
        asm volatile("global_store_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" ::"v"(data), "v"(m) : "memory");
        asm volatile("global_store_dword %0, %1, off" ::"v"(flag), "v"(v) : "memory");
    }
}

// out: [0..1] XCC id of A / B, [2..3] wall ticks of A / B, [4..5] errors of A / B (1 poll bound, 2 payload)
template <bool SC1>
__global__ __launch_bounds__(64) void pingpong(uint32_t* flag, u32x4* data, int a_blk, int b_blk, int iters, uint64_t* out) {
    const int b = (int)blockIdx.x;
    if (b != a_blk && b != b_blk) return;
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x != 0) return;
    const int me = b == a_blk ? 0 : 1;
    out[me] = xcc & 0xFu;
    uint64_t err = 0;
    const uint64_t t0 = wall_clock64();
    for (int i = 0; i < iters && !err; i++) {
        const uint32_t mine = 2u * (uint32_t)i + 1u + (uint32_t)me, theirs = me ? mine - 1u : mine + 1u;
        if (me == 0) send<SC1>(flag, data, mine);
        uint32_t spins = 0;
        while (ld_sc1(flag) != theirs)
            if (++spins > (1u << 20)) { err = 1; break; }
        if (err) break;
        const u32x4 m = ld4_sc1(data);
        if (m.x != theirs || m.y != (theirs ^ 0x5A5A5A5Au) || m.z != theirs + 1u || m.w != ~theirs) err = 2;
        if (me == 1 && !err) send<SC1>(flag, data, mine);
    }
    out[2 + me] = wall_clock64() - t0;
    out[4 + me] = err;
}

static int run(const char* mem, unsigned flags, bool sc1, int a, int b, int iters, double tick_ns) {
    void* region = nullptr;
    hipError_t e = flags ? hipExtMallocWithFlags(&region, 8192, flags) : hipMalloc(&region, 8192);
    if (e != hipSuccess) { std::printf("%s: alloc failed %d\n", mem, (int)e); return 1; }
    uint64_t* out = nullptr;
    if (hipMalloc(&out, 8 * sizeof(uint64_t)) != hipSuccess) return 1;
    uint32_t* flag = (uint32_t*)region;
    u32x4* data = (u32x4*)((char*)region + 4096);  // the payload on its own lines, as a ring slot
    for (int rep = 0; rep < 3; rep++) {
        if (hipMemset(region, 0, 8192) != hipSuccess || hipMemset(out, 0, 8 * sizeof(uint64_t)) != hipSuccess) return 1;
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        if (sc1) pingpong<true><<<16, 64>>>(flag, data, a, b, iters, out);
        else pingpong<false><<<16, 64>>>(flag, data, a, b, iters, out);
        if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); return 1; }
        uint64_t h[8];
        if (hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        const double rt_ns = (double)h[2] * tick_ns / iters;
        std::printf("%-9s stores %-5s blocks %d,%d  xcc %llu,%llu (%s)  rep %d: round trip %7.1f ns, one hop %6.1f ns%s\n",
                    mem, sc1 ? "sc1" : "plain", a, b, (unsigned long long)h[0], (unsigned long long)h[1],
                    h[0] == h[1] ? "same XCD" : "two XCDs", rep, rt_ns, rt_ns / 2,
                    h[4] | h[5] ? (h[4] == 2 || h[5] == 2 ? "  ERROR: stale payload" : "  ERROR: counter never seen (stale line)") : "");
    }
    (void)hipFree(out);
    (void)hipFree(region);
    return 0;
}

int main() {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || khz <= 0) return 1;
    const double tick_ns = 1e6 / khz;
    const int iters = 20000;
    std::printf("wall clock %d kHz; %d round trips per run\n", khz, iters);
    int rc = 0;
    rc |= run("uncached", hipDeviceMallocUncached, true, 0, 1, iters, tick_ns);   // the product today
    rc |= run("uncached", hipDeviceMallocUncached, true, 0, 8, iters, tick_ns);
    rc |= run("cached", 0, true, 0, 8, iters, tick_ns);
    rc |= run("cached", 0, false, 0, 8, iters, tick_ns);
    rc |= run("cached", 0, false, 0, 1, iters, tick_ns);  // cross-XCD with L2-kept lines: expected stale
    return rc;
}
