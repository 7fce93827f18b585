// hip_open.cpp -- where the first-use cost of a HIP context goes (measurement tool): times each
// runtime call vcfxg_open makes, then a first kernel launch from libvcfx_gpu.so.
//   hipcc -O2 --offload-arch=gfx950 -o hip_open hip_open.cpp -Iinclude -Lbuild -lvcfx_gpu
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include "vcfx_gpu.h"
static double t0;
static double now() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define T(x) do { double a = now(); (void)(x); printf("%-40s %8.2f ms (at %8.2f)\n", #x, now() - a, now() - t0); } while (0)
int main() {
    t0 = now();
    int n = 0;
    T(hipGetDeviceCount(&n));
    hipDeviceProp_t p;
    T(hipGetDeviceProperties(&p, 0));
    T(hipSetDevice(0));
    hipStream_t s;
    T(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void *d;
    T(hipMalloc(&d, 4096));
    T(hipMalloc(&d, (size_t)5 << 30));
    vcfxg_ctx *c;
    T(vcfxg_open(0, &c));
    static char buf[1 << 20];
    for (int i = 0; i < (1 << 20); i++) buf[i] = (i % 100 == 99) ? '\n' : 'A';
    T(vcfxg_load_host(c, buf, sizeof buf));
    uint64_t nl;
    T(vcfxg_index(c, 0, &nl));
    T(vcfxg_index(c, 0, &nl));
    vcfxg_summary sm;
    T(vcfxg_allele_freq_region(c, 0, 0, &sm));
    T(vcfxg_allele_freq_region(c, 0, 0, &sm));
    T(vcfxg_close(c));
    return 0;
}
