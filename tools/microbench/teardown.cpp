// teardown.cpp -- process-exit cost after a large pageable host->device copy (measurement
// tool, not product).  The pipe path reads the stream's head into anonymous (THP) memory while
// the HIP runtime starts and copies it to the device from there; the process then takes
// 0.1-0.2 s to end.  Which part is it?
//   mode 0: touch N bytes of anonymous THP memory, _exit
//   mode 1: + hipMalloc N bytes, _exit
//   mode 2: + pageable hipMemcpyAsync of the N bytes to the device (the ingest), _exit
//   mode 3: mode 2, then munmap the host region before _exit
//   mode 4: mode 2 with the copy made through a 16 x 1 MiB pinned ring (memcpy + DMA), _exit
// Run under `time`; the program prints its own phases (ms since start).
//   hipcc -O2 -std=c++17 -o teardown teardown.cpp
//   ./teardown BYTES MODE
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));      \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

static const auto t0 = std::chrono::steady_clock::now();
static double ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: teardown BYTES MODE\n");
        return 2;
    }
    const size_t n = strtoull(argv[1], nullptr, 10);
    const int mode = atoi(argv[2]);
    char *h = (char *)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (h == MAP_FAILED) return 1;
    madvise(h, n, MADV_HUGEPAGE);
    for (size_t k = 0; k < n; k += 4096) h[k] = (char)k;
    printf("touched %.1f\n", ms());
    if (mode >= 1) {
        CK(hipSetDevice(0));
        void *d = nullptr;
        CK(hipMalloc(&d, n));
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        printf("device ready %.1f\n", ms());
        if (mode == 2 || mode == 3) {
            CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            printf("copied %.1f\n", ms());
        } else if (mode == 4) {
            const size_t slot = 1 << 20;
            const int ns = 16;
            std::vector<char *> ring(ns);
            std::vector<hipEvent_t> ev(ns);
            for (int i = 0; i < ns; i++) {
                CK(hipHostMalloc((void **)&ring[i], slot, 0));
                CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
            }
            std::vector<bool> used(ns, false);
            size_t at = 0;
            for (int k = 0; at < n; k = (k + 1) % ns) {
                if (used[k]) CK(hipEventSynchronize(ev[k]));
                const size_t b = n - at < slot ? n - at : slot;
                memcpy(ring[k], h + at, b);
                CK(hipMemcpyAsync((char *)d + at, ring[k], b, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(ev[k], s));
                used[k] = true;
                at += b;
            }
            CK(hipStreamSynchronize(s));
            printf("copied (ring) %.1f\n", ms());
        }
        if (mode == 3) {
            munmap(h, n);
            printf("unmapped %.1f\n", ms());
        }
    }
    printf("exit %.1f\n", ms());
    fflush(stdout);
    _exit(0);
}
