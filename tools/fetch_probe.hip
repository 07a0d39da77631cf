// FETCH_SIZE calibration for the bench's `traffic`: the gfx950 x2 correction of
// MI355X_MICROARCH.md was measured on cached streaming reads; the rings are uncached (MTYPE UC) and
// read with sc1 loads.  This reads a known number of bytes exactly once per launch, from an uncached
// and from a default (cached) allocation, with the rings' load instruction (16 B per lane, sc1), and
// writes nothing; `rocprofv3 --pmc FETCH_SIZE -- ./fetch_probe` then gives FETCH_SIZE per launch to
// set against the bytes read.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_probe tools/fetch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_once(const u32x4* __restrict__ src, size_t n16, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000);
    uint32_t acc = 0;
    // grid-stride over 16-B chunks; each chunk read once (offsets stay below 2 GiB: n16 * 16 < 2^31)
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(i * 16u), 0, 16 /* sc1, as the rings (kAuxSc1) */);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads; practically never stores
}

static int run(const char* what, unsigned flags, size_t bytes) {
    void* p = nullptr;
    hipError_t e = flags ? hipExtMallocWithFlags(&p, bytes, flags) : hipMalloc(&p, bytes);
    if (e != hipSuccess) { std::printf("%s: alloc failed %d\n", what, (int)e); return 1; }
    uint32_t* out = nullptr;
    if (hipMalloc(&out, 4) != hipSuccess) return 1;
    if (hipMemset(p, 0x5A, bytes) != hipSuccess) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int it = 0; it < 3; it++) {
        (void)hipEventRecord(a);
        read_once<<<2048, 256>>>((const u32x4*)p, bytes / 16, out);
        (void)hipEventRecord(b);
        if (hipEventSynchronize(b) != hipSuccess) return 1;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        std::printf("%s: launch %d read %zu bytes once, %.3f ms, %.1f GB/s\n", what, it, bytes, ms, bytes / (ms * 1e-3) / 1e9);
    }
    (void)hipFree(out);
    (void)hipFree(p);
    return 0;
}

int main() {
    const size_t bytes = (size_t)1 << 30;  // 1 GiB
    if (run("uncached (hipDeviceMallocUncached)", hipDeviceMallocUncached, bytes)) return 1;
    if (run("default (hipMalloc)", 0, bytes)) return 1;
    return 0;
}
