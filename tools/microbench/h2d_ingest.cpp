// h2d_ingest.cpp -- host->HBM ingest rates for a page-cache-warm file (measurement tool, not
// product).  Compares: one pageable hipMemcpy from the mmap (r01's vcfxg_load_host), a
// pinned staging ring fed by T threads memcpy'ing from the mmap, the same ring fed by T
// threads pread()ing the file, and the pinned->device DMA alone (the PCIe ceiling).
//   hipcc -O2 -std=c++17 -o h2d_ingest h2d_ingest.cpp -lpthread
//   ./h2d_ingest FILE [chunk_MiB] [slots]
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    size_t chunk = (argc > 2 ? atol(argv[2]) : 32) << 20;
    int slots = argc > 3 ? atoi(argv[3]) : 4;
    int fd = open(argv[1], O_RDONLY);
    struct stat st;
    fstat(fd, &st);
    size_t n = st.st_size;
    const char *m = (const char *)mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    madvise((void *)m, n, MADV_SEQUENTIAL | MADV_WILLNEED);
    // warm the page cache
    {
        std::vector<char> b(1 << 24);
        for (size_t o = 0; o < n; o += b.size()) pread(fd, b.data(), b.size(), o);
    }
    double t0 = now();
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    printf("hip init %.3f s\n", now() - t0);
    char *d;
    t0 = now();
    CK(hipMalloc(&d, n + 256));
    printf("hipMalloc %.1f GB %.3f s\n", n / 1e9, now() - t0);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // 1: pageable copy from the mmap
    for (int rep = 0; rep < 2; rep++) {
        t0 = now();
        CK(hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double dt = now() - t0;
        printf("pageable hipMemcpy from mmap: %.3f s  %.1f GB/s\n", dt, n / dt / 1e9);
    }
    std::vector<char *> pin(slots);
    std::vector<hipEvent_t> ev(slots);
    t0 = now();
    for (int i = 0; i < slots; i++) {
        CK(hipHostMalloc(&pin[i], chunk, hipHostMallocDefault));
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
        memset(pin[i], 0, chunk);
    }
    printf("pinned %d x %zu MiB: %.3f s\n", slots, chunk >> 20, now() - t0);
    // 4: DMA only (pinned -> device), the PCIe ceiling
    {
        t0 = now();
        for (size_t o = 0, k = 0; o < n; o += chunk, k++) {
            size_t len = std::min(chunk, n - o);
            CK(hipMemcpyAsync(d + o, pin[k % slots], len, hipMemcpyHostToDevice, s));
        }
        CK(hipStreamSynchronize(s));
        double dt = now() - t0;
        printf("pinned DMA only: %.3f s  %.1f GB/s\n", dt, n / dt / 1e9);
    }
    for (int mode = 0; mode < 2; mode++) {
        for (int T : {1, 4, 8, 16}) {
            // persistent workers: per chunk, each copies its 1/T slice into the slot
            t0 = now();
            std::vector<std::thread> th;
            std::atomic<long> go{-1}, done{0};
            const char *src_m = m;
            std::vector<size_t> off(1), lenv(1);
            std::atomic<int> slot_now{0};
            size_t cur_off = 0, cur_len = 0;
            volatile bool stop = false;
            for (int w = 0; w < T; w++)
                th.emplace_back([&, w] {
                    long seen = -1;
                    for (;;) {
                        long g;
                        while ((g = go.load(std::memory_order_acquire)) == seen && !stop) std::this_thread::yield();
                        if (stop) return;
                        seen = g;
                        size_t per = (cur_len / T + 4095) & ~(size_t)4095;
                        size_t a = std::min(cur_len, per * w), b = std::min(cur_len, per * (w + 1));
                        char *dst = pin[slot_now.load()] + a;
                        if (b > a) {
                            if (mode == 0) memcpy(dst, src_m + cur_off + a, b - a);
                            else {
                                size_t got = 0;
                                while (got < b - a) {
                                    ssize_t k = pread(fd, dst + got, b - a - got, cur_off + a + got);
                                    if (k <= 0) break;
                                    got += k;
                                }
                            }
                        }
                        done.fetch_add(1, std::memory_order_acq_rel);
                    }
                });
            long gen = 0;
            for (size_t o = 0, k = 0; o < n; o += chunk, k++) {
                int sl = (int)(k % slots);
                CK(hipEventSynchronize(ev[sl]));
                cur_off = o;
                cur_len = std::min(chunk, n - o);
                slot_now = sl;
                done = 0;
                go.store(gen++, std::memory_order_release);
                while (done.load(std::memory_order_acquire) < T) std::this_thread::yield();
                CK(hipMemcpyAsync(d + o, pin[sl], cur_len, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(ev[sl], s));
            }
            CK(hipStreamSynchronize(s));
            double dt = now() - t0;
            stop = true;
            for (auto &x : th) x.join();
            printf("%s T=%2d ring %d x %zu MiB: %.3f s  %.1f GB/s\n", mode == 0 ? "memcpy(mmap)" : "pread(fd)   ", T,
                   slots, chunk >> 20, dt, n / dt / 1e9);
        }
    }
    // host-side read rates alone (no GPU): memcpy from mmap single thread
    {
        std::vector<char> b(chunk);
        t0 = now();
        for (size_t o = 0; o < n; o += chunk) memcpy(b.data(), m + o, std::min(chunk, n - o));
        double dt = now() - t0;
        printf("memcpy(mmap) 1 thread, no GPU: %.1f GB/s\n", n / dt / 1e9);
    }
    return 0;
}
