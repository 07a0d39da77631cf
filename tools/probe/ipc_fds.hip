// Probe (round 5): what a hipIpc handle holds on to in the exporting process.  Allocates 5 uncached regions,
// exports them one after another and lists the process's dmabuf file descriptors (/proc/self/fd) and the first
// 32 bytes of each handle after every step; then frees one region and exports a new one.
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                         \
        }                                                                                         \
    } while (0)

static void fds(const char* when) {
    std::string out;
    DIR* d = opendir("/proc/self/fd");
    if (!d) return;
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        char path[64], tgt[256] = {0};
        std::snprintf(path, sizeof path, "/proc/self/fd/%s", e->d_name);
        const ssize_t n = readlink(path, tgt, sizeof tgt - 1);
        if (n > 0 && (std::strstr(tgt, "dmabuf") || std::strstr(tgt, "dma_buf") || std::strstr(tgt, "anon_inode")))
            out += std::string(" ") + e->d_name + "=" + tgt;
    }
    closedir(d);
    std::printf("%-28s fds:%s\n", when, out.c_str());
}

static void show(const char* what, const hipIpcMemHandle_t& h) {
    std::printf("%-28s handle:", what);
    const unsigned* w = reinterpret_cast<const unsigned*>(&h);
    for (int i = 0; i < 16; i++) std::printf(" %08x", w[i]);
    std::printf("\n");
}

int main() {
    const size_t sz[5] = {1 << 20, 64 << 10, 16 << 10, 256 << 20, 64 << 10};
    void* p[5];
    hipIpcMemHandle_t h[5];
    fds("start");
    for (int i = 0; i < 5; i++) CK(hipExtMallocWithFlags(&p[i], sz[i], hipDeviceMallocUncached));
    fds("allocated");
    for (int i = 0; i < 5; i++) {
        CK(hipIpcGetMemHandle(&h[i], p[i]));
        char w[32];
        std::snprintf(w, sizeof w, "export %d", i);
        show(w, h[i]);
        fds(w);
    }
    hipIpcMemHandle_t again;
    CK(hipIpcGetMemHandle(&again, p[0]));
    show("export 0 again", again);
    fds("export 0 again");
    CK(hipFree(p[3]));
    fds("freed 3");
    void* q = nullptr;
    CK(hipExtMallocWithFlags(&q, sz[3], hipDeviceMallocUncached));
    std::printf("new allocation %p (old region 3 was %p)\n", q, p[3]);
    hipIpcMemHandle_t hq;
    CK(hipIpcGetMemHandle(&hq, q));
    show("export new", hq);
    fds("export new");
    return 0;
}
