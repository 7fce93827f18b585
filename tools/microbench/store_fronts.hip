// store_fronts.hip -- diagnostic microbenchmark (not part of the product): how does HBM store
// bandwidth depend on the order in which waves write a k_ac_fmt-shaped output?  42.6 GB written
// as 427,409 "records" of R bytes, each cut into T "tiles" of about 2.5 KB (the AC rows of one
// 64-row tile), 16 B per lane, one 1 KiB store instruction per wave-step:
//   rec     one wave per record at a time, its tiles front to back (k_ac_fmt's order)
//   tile    consecutive waves take consecutive tiles (unit u = wave + k * waves; G tiles per unit)
//   *+ld    the same with a dependent load per unit (the record's metadata: the wave waits for
//           its earlier stores, loads and stores sharing vmcnt)
//   fill    one contiguous chunk per block (a memset)
//   rows    a lane per ~39-byte text row, three unaligned 16 B stores (k_ac_rows' shape)
//   rows+ld the same with 16 tiles' GT dwords loaded together every 16 tiles
// Grid 2,048 blocks x 512 threads with 54 KiB of dynamic LDS (k_ac_fmt's occupancy: 3 blocks per
// CU).  usage: store_fronts
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void put_tile(char *out, int64_t a, int64_t e, v4u v) {
    for (int64_t b = a + 16 * (threadIdx.x & 63); b < e; b += 1024) *reinterpret_cast<v4u *>(out + b) = v;
}

// mode 0: record-major; 1: tile-major (G tiles per unit); bit 2: a dependent metadata load per unit
template <int kMode>
__global__ __launch_bounds__(512) void k_store(char *out, int64_t nrec, int64_t R, int64_t T, int64_t TB, int G,
                                               const int64_t *meta) {
    extern __shared__ char lds[];
    const int64_t w = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 8 + threadIdx.x / 64));
    const int64_t nw = (int64_t)gridDim.x * 8;
    const v4u v = {0x61616161u, 0x62626262u, 0x63636363u, (unsigned)threadIdx.x};
    if (threadIdx.x == 0) lds[0] = 0;
    if ((kMode & 3) == 0) {
        for (int64_t r = w; r < nrec; r += nw) {
            int64_t base = r * R;
            if (kMode & 4) base += meta[r];
            for (int64_t t = 0; t < T; t++) put_tile(out, base + t * TB, base + (t + 1 < T ? (t + 1) * TB : R), v);
        }
    } else {
        const int64_t units = (nrec * T + G - 1) / G;
        for (int64_t u = w; u < units; u += nw) {
            for (int g = 0; g < G; g++) {
                const int64_t q = u * G + g;
                if (q >= nrec * T) break;
                const int64_t r = q / T, t = q % T;
                int64_t base = r * R;
                if ((kMode & 4) && g == 0) base += meta[r];
                put_tile(out, base + t * TB, base + (t + 1 < T ? (t + 1) * TB : R), v);
            }
        }
    }
}

// rows: a lane per text row of rl bytes (P-byte prefix), written straight to global memory as
// three unaligned 16 B stores (prefix [0, 16), prefix [P - 16, P), the row's last 16 bytes)
__global__ __launch_bounds__(512) void k_rows(char *out, int64_t nrec, int64_t R, int rl, int P, int rows) {
    extern __shared__ char lds[];
    const int64_t w = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 8 + threadIdx.x / 64));
    const int64_t nw = (int64_t)gridDim.x * 8;
    const int lane = threadIdx.x & 63;
    const v4u a = {0x61616161u, 0x62626262u, 0x63636363u, 0x64646464u};
    const v4u b = {0x65656565u, 0x66666666u, 0x67676767u, 0x68686868u};
    if (threadIdx.x == 0) lds[0] = 0;
    for (int64_t r = w; r < nrec; r += nw) {
        char *base = out + r * R;
        for (int i0 = 0; i0 < rows; i0 += 64) {
            const int i = i0 + lane;
            if (i >= rows) break;
            char *q = base + (int64_t)i * rl;
            v4u c = b;
            c.w ^= (unsigned)i;
            __builtin_memcpy(q, &a, 16);
            __builtin_memcpy(q + P - 16, &b, 16);
            __builtin_memcpy(q + rl - 16, &c, 16);
        }
    }
}

// rows+ld: k_rows with the GT dwords of 16 tiles loaded together every 16 tiles (k_ac_rows'
// counts: each such wait also drains the wave's stores before it)
__global__ __launch_bounds__(512) void k_rows_ld(char *out, int64_t nrec, int64_t R, int rl, int P, int rows,
                                                 const uint32_t *gt) {
    extern __shared__ char lds[];
    const int64_t w = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 8 + threadIdx.x / 64));
    const int64_t nw = (int64_t)gridDim.x * 8;
    const int lane = threadIdx.x & 63;
    const v4u a = {0x61616161u, 0x62626262u, 0x63636363u, 0x64646464u};
    const v4u b = {0x65656565u, 0x66666666u, 0x67676767u, 0x68686868u};
    if (threadIdx.x == 0) lds[0] = 0;
    for (int64_t r = w; r < nrec; r += nw) {
        char *base = out + r * R;
        const uint32_t *g0 = gt + (r & 4095) * rows;
        uint32_t g[16];
        for (int i0 = 0; i0 < rows; i0 += 64) {
            const int t = i0 / 64;
            if ((t & 15) == 0) {
#pragma unroll
                for (int k = 0; k < 16; k++)
                    g[k] = __hip_atomic_load(g0 + min(i0 + 64 * k + lane, rows - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
            uint32_t gg = g[0];
#pragma unroll
            for (int k = 1; k < 16; k++) gg = (t & 15) == k ? g[k] : gg;
            const int i = min(i0 + lane, rows - 1);
            char *q = base + (int64_t)i * rl;
            v4u c = b;
            c.w ^= gg;
            __builtin_memcpy(q, &a, 16);
            __builtin_memcpy(q + P - 16, &b, 16);
            __builtin_memcpy(q + rl - 16, &c, 16);
        }
    }
}

__global__ __launch_bounds__(512) void k_fill(char *out, int64_t n, int64_t chunk) {
    extern __shared__ char lds[];
    if (threadIdx.x == 0) lds[0] = 0;
    const v4u v = {1u, 2u, 3u, 4u};
    const int64_t cs = (int64_t)blockIdx.x * chunk, ce = cs + chunk < n ? cs + chunk : n;
    for (int64_t b = cs + 16 * threadIdx.x; b < ce; b += 16 * 512) *reinterpret_cast<v4u *>(out + b) = v;
}

int main() {
    const int64_t nrec = 427409, T = 40, TB = 2496, R = T * TB;  // 99,840 B per record
    const int64_t n = nrec * R;
    char *out;
    int64_t *meta;
    CHK(hipMalloc(&out, n + 4096));
    CHK(hipMalloc(&meta, nrec * 8));
    CHK(hipMemset(meta, 0, nrec * 8));
    uint32_t *gtb;  // 4,096 records' GT dwords (40 MB: mostly L2 / MALL hits)
    CHK(hipMalloc(&gtb, 4096ull * 2560 * 4));
    CHK(hipMemset(gtb, 0x30, 4096ull * 2560 * 4));
    const size_t lds = 54 * 1024;
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    struct Case { const char *name; int mode, G; };
    const Case cases[] = {{"rec", 0, 1}, {"rec+ld", 4, 1}, {"tile G1", 1, 1}, {"tile G1+ld", 5, 1}, {"tile G4", 1, 4},
                          {"tile G4+ld", 5, 4}, {"tile G10+ld", 5, 10}, {"fill", -1, 0}, {"rows", 8, 0}, {"rows+ld", 9, 0}};
    for (const Case &c : cases) {
        float best = 1e9f, sum = 0;
        for (int it = 0; it < 6; it++) {
            CHK(hipEventRecord(a, 0));
            switch (c.mode) {
            case 0: hipLaunchKernelGGL(k_store<0>, dim3(2048), dim3(512), lds, 0, out, nrec, R, T, TB, c.G, meta); break;
            case 4: hipLaunchKernelGGL(k_store<4>, dim3(2048), dim3(512), lds, 0, out, nrec, R, T, TB, c.G, meta); break;
            case 1: hipLaunchKernelGGL(k_store<1>, dim3(2048), dim3(512), lds, 0, out, nrec, R, T, TB, c.G, meta); break;
            case 5: hipLaunchKernelGGL(k_store<5>, dim3(2048), dim3(512), lds, 0, out, nrec, R, T, TB, c.G, meta); break;
            case 8: hipLaunchKernelGGL(k_rows, dim3(2048), dim3(512), lds, 0, out, nrec, R, 39, 27, 2560); break;
            case 9: hipLaunchKernelGGL(k_rows_ld, dim3(2048), dim3(512), lds, 0, out, nrec, R, 39, 27, 2560, gtb); break;
            default: {
                const int64_t chunk = 4 << 20;
                hipLaunchKernelGGL(k_fill, dim3((unsigned)((n + chunk - 1) / chunk)), dim3(512), lds, 0, out, n, chunk);
            }
            }
            CHK(hipGetLastError());
            CHK(hipEventRecord(b, 0));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (it) {
                sum += ms;
                if (ms < best) best = ms;
            }
        }
        printf("%-12s %.3f ms best, %.3f mean  %.2f TB/s\n", c.name, best, sum / 5, n / (best * 1e-3) / 1e12);
    }
    return 0;
}
