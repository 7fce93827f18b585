// stream_fronts.hip -- diagnostic microbenchmark (not part of the product): does HBM read
// bandwidth depend on how many independent streams are open at once?  Reads a 4.3 GB buffer
// three ways, 16 B per lane, `kU` 1 KiB wave-steps in flight per batch (the walk's sweep):
//   A "walkers": one wave per C-byte chunk, streaming it front to back (the walk's pattern)
//   B "block":   a block of W waves per W*C bytes, the waves taking interleaved batches, so
//                each block advances as one contiguous front
//   C "sweep":   one wave per 16 KiB chunk, all its loads in flight at once (the index sweep)
// usage: stream_fronts [chunk_bytes]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
constexpr int kU = 6, kStep = 1024, kBatch = kU * kStep;

__global__ __launch_bounds__(256) void walkers(const uint4 *buf, int64_t n, int64_t chunk, uint32_t *sink) {
    const int64_t w = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    const int64_t cs = w * chunk, ce = cs + chunk < n ? cs + chunk : n;
    uint32_t acc = 0;
    for (int64_t b = cs; b < ce; b += kBatch) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            int64_t o = b + u * kStep + lane * 16;
            v[u] = buf[(o < ce ? o : cs) / 16];
        }
#pragma unroll
        for (int u = 0; u < kU; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void block_front(const uint4 *buf, int64_t n, int64_t chunk, uint32_t *sink) {
    const int wv = threadIdx.x / 64, lane = threadIdx.x & 63;
    const int64_t cs = (int64_t)blockIdx.x * 4 * chunk, ce = cs + 4 * chunk < n ? cs + 4 * chunk : n;
    uint32_t acc = 0;
    for (int64_t b = cs + wv * kBatch; b < ce; b += 4 * kBatch) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            int64_t o = b + u * kStep + lane * 16;
            v[u] = buf[(o < ce ? o : cs) / 16];
        }
#pragma unroll
        for (int u = 0; u < kU; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void sweep16k(const uint4 *buf, int64_t n, uint32_t *sink) {
    const int64_t w = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    const int64_t cs = w * 16384;
    uint32_t acc = 0;
    uint4 v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) {
        int64_t o = cs + u * kStep + lane * 16;
        v[u] = buf[(o < n ? o : 0) / 16];
    }
#pragma unroll
    for (int u = 0; u < 16; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
    const int64_t n = 4300000000ll & ~(int64_t)65535;
    const int64_t chunk = argc > 1 ? atoll(argv[1]) : 131072;
    uint4 *buf;
    uint32_t *sink;
    CHK(hipMalloc(&buf, n));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(buf, 0x31, n));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int k = 0; k < 3; k++) {
        const char *name = k == 0 ? "walkers" : k == 1 ? "block_front" : "sweep16k";
        float best = 1e9f;
        for (int it = 0; it < 6; it++) {
            CHK(hipEventRecord(a, 0));
            if (k == 0) {
                int64_t nw = (n + chunk - 1) / chunk;
                hipLaunchKernelGGL(walkers, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, buf, n, chunk, sink);
            } else if (k == 1) {
                int64_t nb = (n + 4 * chunk - 1) / (4 * chunk);
                hipLaunchKernelGGL(block_front, dim3((unsigned)nb), dim3(256), 0, 0, buf, n, chunk, sink);
            } else {
                int64_t nw = (n + 16383) / 16384;
                hipLaunchKernelGGL(sweep16k, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, buf, n, sink);
            }
            CHK(hipGetLastError());
            CHK(hipEventRecord(b, 0));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (it && ms < best) best = ms;
        }
        printf("%-12s chunk %7lld: %.3f ms  %.2f TB/s\n", name, (long long)chunk, best, n / (best * 1e-3) / 1e12);
    }
    return 0;
}
