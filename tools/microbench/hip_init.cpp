// hip_init.cpp -- the HIP runtime's own start-up with and without libvcfx_gpu.so loaded
// (measurement tool): -DWITH_VCFX links the engine library and references it, so its fat
// binary (every kernel's code object) is registered with the runtime.
//   hipcc -O2 --offload-arch=gfx950 -o hip_init_plain hip_init.cpp
//   hipcc -O2 --offload-arch=gfx950 -DWITH_VCFX -o hip_init_vcfx hip_init.cpp -Iinclude -Lbuild -lvcfx_gpu
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#ifdef WITH_VCFX
#include "vcfx_gpu.h"
#endif
static double now() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
__global__ void k_nop(int *p) {
    if (p) p[threadIdx.x] = 0;
}
#define T(x) do { double a = now(); (void)(x); printf("%-52s %8.2f ms\n", #x, now() - a); } while (0)
int main() {
#ifdef WITH_VCFX
    printf("with libvcfx_gpu.so (%s)\n", vcfxg_version());
#endif
    int n = 0;
    T(hipGetDeviceCount(&n));
    T(hipSetDevice(0));
    hipStream_t s;
    T(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *d;
    T(hipMalloc(&d, 4096));
    for (int i = 0; i < 2; i++) {
        const double a = now();
        hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, d);
        (void)hipStreamSynchronize(s);
        printf("%-52s %8.2f ms\n", i ? "second kernel launch + sync" : "first kernel launch + sync", now() - a);
    }
    return 0;
}
