// vcfxg_ld_mask.hip -- LD r^2 for 128x128 variant tiles with missing genotypes, on the FP4 MFMA.
//
// VCFX_ld_calculator's computeRsqSIMD (VCFX_ld_calculator.cpp:352-393) sums over the samples
// valid in BOTH variants.  With a missing call coded as 0 in the dosage plane X, a valid-mask
// plane V (1 valid, 0 missing) and Q = X^2, every term is a GEMM of 0/1/2/4-valued operands:
//     n   = V_i . V_j          Sxy = X_i . X_j
//     Sx  = X_i . V_j          Sy  = V_i . X_j
//     Sxx = Q_i . V_j          Syy = V_i . Q_j
// 0, 1, 2 and 4 are exact e2m1 values and every partial sum is an integer below 2^24, so the
// fp32-accumulating block-scaled MFMA (scales 2^0) gives all six sums exactly: six products
// per 32x32 sub-tile, executed at the FP4 rate (the dense kernel, vcfxg_ld_fast.hip, needs only
// Sxy).  The planes are zero-padded past the samples, so padding adds nothing.
//
//   * tile: 128 rows (variants i) x 128 columns (variants j), 8 waves as 4 (rows) x 2
//     (columns); a wave owns 32 rows x 64 columns = 2 sub-tiles x 6 accumulators (192 regs);
//   * staging: per 64-byte k-slice (128 samples) the six operand slabs (X, V, Q of the row
//     tile and of the column tile, 128 rows x 64 B each = 48 KiB) by global_load_lds into a
//     3-buffer ring (144 KiB), 16-byte slots XOR-swizzled through the source address so the
//     ds_read_b128 fragment reads are conflict free; 9 fragment reads feed 12 MFMAs per k-step;
//   * epilogue per pair: window (j - window <= i < j), an fp32 prefilter on the exact integer
//     sums that keeps every pair whose exact r^2 can reach the threshold (the error bound is
//     explicit below), then the reference's fp64 sequence (rsq_epilogue: the computeRsqFast
//     gate, n < 2, correctly rounded ops) on the candidates only;
//   * count pass (P = 1): per (column j, 64-row quarter) pass counts into the count table
//     shared with the other LD kernels; emit pass (P = 2, tiles holding pairs only): the same
//     sums again, each passing pair written at its ordered offset (rank of its row among the
//     column's passing rows of the quarter, from LDS masks).
#include "vcfxg_device.h"
#include "vcfxg_ld.h"

#include <algorithm>

namespace vcfxg {

namespace {
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int kFmtFp4 = 4;             // cbsz / blgp operand format: e2m1
constexpr int kScaleOne = 0x7F7F7F7F;  // E8M0 block scales 2^0

constexpr int kT = kLdMaskTile;        // tile side: 128 variants
constexpr int kBK = 64;                // k-slice bytes (128 samples)
constexpr int kPlanes = 3;             // X, V, Q
constexpr int kSlab = kT * kBK;        // one plane of one side per stage: 8 KiB
constexpr int kStage = 2 * kPlanes * kSlab;  // 48 KiB
constexpr int kNBuf = 3;
constexpr int kWaves = 8;
constexpr int kGlds = kStage / 1024 / kWaves;  // 1 KiB LDS-DMA instructions per wave per stage: 6
static_assert(kGlds == 6, "the k-loop's vmcnt counts assume 6 glds per wave per stage");

__device__ __forceinline__ void glds16(const void *src, int8_t *lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

// bijective XCD-aware remap: consecutive list entries land on one XCD (shared operand tiles)
__device__ __forceinline__ uint32_t xcd_remap_m(uint32_t b, uint32_t n) {
    const uint32_t q = n / 8, r = n % 8, x = b % 8, k = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

__device__ __forceinline__ v16f mfma4(const v4i &a, const v4i &b, const v16f &c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v8i{a.x, a.y, a.z, a.w, 0, 0, 0, 0},
                                                           v8i{b.x, b.y, b.z, b.w, 0, 0, 0, 0}, c, kFmtFp4, kFmtFp4, 0,
                                                           kScaleOne, 0, kScaleOne);
}
}  // namespace

// mask_candidate / mask_r2: vcfxg_ld.h (shared with the sparse-missing kernel)

template <int P>
__global__ __launch_bounds__(kWaves * kWave) void k_ld_mask(const uint8_t *__restrict__ Gx,
                                                            const uint8_t *__restrict__ Gv,
                                                            const uint8_t *__restrict__ Gq,
                                                            const LdVar *__restrict__ vars,
                                                            const uint32_t *__restrict__ chrom_id, LdWindowArgs a,
                                                            const uint32_t *__restrict__ tiles, uint32_t ntiles,
                                                            uint16_t *__restrict__ cnt, LdOffsets off,
                                                            LdPair *__restrict__ pairs, float pe) {
    // ONE LDS array: the staging ring, then (after the k-loop) the per-column counts / masks
    __shared__ __attribute__((aligned(16))) int8_t lds[kNBuf * kStage];
    const uint32_t b = xcd_remap_m(blockIdx.x, ntiles);
    const uint32_t I2 = tiles[2 * b], J2 = tiles[2 * b + 1];
    const int t = threadIdx.x, w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int wi = w >> 1, wj = w & 1;  // rows wi*32.., columns wj*64..
    const int64_t M = (int64_t)a.m;
    const int64_t ibase = (int64_t)I2 * kT, jbase = (int64_t)J2 * kT;
    // count-table slot of 64-block pair (bI, bJ); false outside the window triangle
    auto sub = [&](uint64_t bI, uint64_t bJ, uint64_t &slot) {
        const uint64_t jrow0 = bJ * kLdBlock;
        const uint64_t ifirst = jrow0 > a.window ? (jrow0 - a.window) / kLdBlock : 0;
        slot = bI - ifirst;
        return bI >= ifirst && bI <= bJ;
    };
    if (P == 2) {  // emit pass: only tiles holding a counted pair (4 quarters x 64 columns)
        uint32_t any = 0;
        if (t < 2 * kT) {
            const int qi = t >> 7, col = t & 127;
            const uint64_t bI = 2ull * I2 + qi, bJ = 2ull * J2 + (col >> 6);
            uint64_t slot;
            const int64_t jj = jbase + col;
            if (sub(bI, bJ, slot) && jj < M && jj >= (int64_t)a.j_lo && jj < (int64_t)a.j_hi)
                any = cnt[(uint64_t)(jj - (int64_t)a.j_lo) * a.nb + slot];
        }
        if (!__syncthreads_or(any != 0)) return;
    }
    const int kpad = a.kp4;
    // staging sources: instruction q of wave w is slab piece idx = 6w + q: side s = idx / 24,
    // plane p = (idx / 8) % 3, rows 16 (idx % 8) ..; lane l -> row (l >> 2), physical 16 B slot
    // l & 3 holding logical slot (l & 3) ^ ((row >> 2) & 3)
    const uint8_t *src[kGlds];
#pragma unroll
    for (int q = 0; q < kGlds; q++) {
        const int idx = kGlds * w + q;
        const int s = idx / 24, p = (idx >> 3) % 3;
        const int lrow = (idx & 7) * 16 + (l >> 2);
        int64_t g = (s ? jbase : ibase) + lrow;
        if (g >= M) g = M - 1;
        const int logical = (l & 3) ^ ((lrow >> 2) & 3);
        const uint8_t *plane = p == 0 ? Gx : p == 1 ? Gv : Gq;
        src[q] = plane + g * (int64_t)kpad + logical * 16;
    }
    auto stage = [&](int ks, int buf) {
#pragma unroll
        for (int q = 0; q < kGlds; q++) glds16(src[q] + ks * kBK, lds + buf * kStage + (kGlds * w + q) * 1024);
    };
    // accumulators per column sub-tile y: xx, xv, vx, vv, qv, vq
    v16f xx[2], xv[2], vx[2], vv[2], qv[2], vq[2];
#pragma unroll
    for (int y = 0; y < 2; y++) xx[y] = xv[y] = vx[y] = vv[y] = qv[y] = vq[y] = v16f{};
    const int nk = kpad / kBK;
    // fragment of plane p, side s, tile row `row`, k-half kh of the k-slice in buffer base
    auto frag = [&](const int8_t *base, int s, int p, int row, int kh) {
        const int lg = 2 * kh + h;
        return *reinterpret_cast<const v4i *>(base + ((s * kPlanes + p) * kT + row) * kBK +
                                              ((lg ^ ((row >> 2) & 3)) << 4));
    };
    asm volatile("" ::"s"(cnt), "s"(vars), "s"(pairs));
    stage(0, 0);
    stage(nk > 1 ? 1 : 0, 1);
    for (int ks = 0; ks < nk; ks++) {
        // stage ks landed (stage ks + 1 may still load): this wave's, then every wave's
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // buffer (ks + 2) % 3 was last read in step ks - 1, before this barrier; past the end
        // a re-read of the last slice keeps the counts constant
        stage(ks + 2 < nk ? ks + 2 : nk - 1, (ks + 2) % kNBuf);
        const int8_t *base = lds + (ks % kNBuf) * kStage;
#pragma unroll
        for (int kh = 0; kh < 2; kh++) {
            const int ra = wi * 32 + r;
            const v4i ax = frag(base, 0, 0, ra, kh), av = frag(base, 0, 1, ra, kh), aq = frag(base, 0, 2, ra, kh);
#pragma unroll
            for (int y = 0; y < 2; y++) {
                const int rb = wj * 64 + y * 32 + r;
                const v4i bx = frag(base, 1, 0, rb, kh), bv = frag(base, 1, 1, rb, kh), bq = frag(base, 1, 2, rb, kh);
                xx[y] = mfma4(ax, bx, xx[y]);
                xv[y] = mfma4(ax, bv, xv[y]);
                vx[y] = mfma4(av, bx, vx[y]);
                vv[y] = mfma4(av, bv, vv[y]);
                qv[y] = mfma4(aq, bv, qv[y]);
                vq[y] = mfma4(av, bq, vq[y]);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is done with the ring: its bytes are reused below
    // epilogue: lane (h, r) holds, for sub-tile y, column j = jbase + wj*64 + 32y + r and rows
    // i = ibase + wi*32 + (k & 3) + 8 (k >> 2) + 4h in accumulator element k
    const float tmf = a.all_pass ? 0.f : (float)(a.tm * (1.0 - 1e-5));
    const int64_t i0 = ibase + wi * 32;
    const int qi = wi >> 1;                     // the 64-row quarter of these rows
    uint32_t *cl = reinterpret_cast<uint32_t *>(lds);  // [2 quarters][128 columns] counts / [..][2] masks
    if (t < 2 * kT * 2) cl[t] = 0;
    __syncthreads();
    uint32_t bits[2] = {0u, 0u};  // per sub-tile: bit k = pair (row(k), j) passes
#pragma unroll
    for (int y = 0; y < 2; y++) {
        const int64_t j = jbase + wj * 64 + 32 * y + r;
        const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
        if (!jok) continue;
        // rows i of this lane's 16 with j - window <= i < j
        const int64_t lo_i = j - (int64_t)a.window;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int64_t i = i0 + (k & 3) + 8 * (k >> 2) + 4 * h;
            if (i >= j || i < lo_i) continue;
            if (!a.all_pass &&
                !mask_candidate(vv[y][k], xv[y][k], vx[y][k], xx[y][k], qv[y][k], vq[y][k], pe, tmf))
                continue;
            const LdVar &vi = vars[i], &vj = vars[j];
            if (a.max_dist > 0 && chrom_id[i] == chrom_id[j]) {
                int d = vj.pos - vi.pos;
                if (d < 0) d = -d;
                if (d > a.max_dist) continue;
            }
            const double rr = mask_r2(vi.varx, vj.varx, (int)vv[y][k], (int)xv[y][k], (int)vx[y][k], (int)xx[y][k],
                                      (int)qv[y][k], (int)vq[y][k]);
            if (rr >= a.threshold) bits[y] |= 1u << k;
        }
    }
    if (P == 1) {
#pragma unroll
        for (int y = 0; y < 2; y++) {
            const uint32_t c = __popc(bits[y]) + __popc((uint32_t)__shfl_xor((int)bits[y], 32));
            if (h == 0 && c) atomicAdd(&cl[qi * kT + wj * 64 + 32 * y + r], c);
        }
        __syncthreads();
        if (t < 2 * kT) {
            const int q = t >> 7, col = t & 127;
            const uint64_t bI = 2ull * I2 + q, bJ = 2ull * J2 + (col >> 6);
            uint64_t slot;
            const int64_t jj = jbase + col;
            if (sub(bI, bJ, slot) && jj < M && jj >= (int64_t)a.j_lo && jj < (int64_t)a.j_hi)
                cnt[(uint64_t)(jj - (int64_t)a.j_lo) * a.nb + slot] = (uint16_t)cl[q * kT + col];
        }
        return;
    }
    // emit: the 32-row pass mask of each column from this wave (lanes h = 0, 1 hold rows 4h +
    // ...), into LDS [quarter][column][half]; then each passing pair's rank in its column
    uint32_t m32[2];
#pragma unroll
    for (int y = 0; y < 2; y++) {
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (bits[y] & (1u << k)) m |= 1u << ((k & 3) + 8 * (k >> 2) + 4 * h);
        m |= (uint32_t)__shfl_xor((int)m, 32);
        m32[y] = m;
        if (h == 0) cl[(qi * kT + wj * 64 + 32 * y + r) * 2 + (wi & 1)] = m;
    }
    __syncthreads();
#pragma unroll
    for (int y = 0; y < 2; y++) {
        if (!bits[y]) continue;
        const int col = wj * 64 + 32 * y + r;
        const int64_t j = jbase + col;
        const uint64_t bI = 2ull * I2 + qi, bJ = 2ull * J2 + (col >> 6);
        uint64_t slot;
        if (!sub(bI, bJ, slot)) continue;  // (no pair passes outside the window: defensive)
        const uint64_t dst = off.at((uint64_t)(j - (int64_t)a.j_lo), a.nb, slot);
        const uint32_t above = (wi & 1) ? __popc(cl[(qi * kT + col) * 2]) : 0u;
        const LdVar &vj = vars[j];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            if (!(bits[y] & (1u << k))) continue;
            const int row = (k & 3) + 8 * (k >> 2) + 4 * h;
            const int64_t i = i0 + row;
            LdPair pr;
            pr.i = (uint32_t)i;
            pr.j = (uint32_t)j;
            pr.r2 = mask_r2(vars[i].varx, vj.varx, (int)vv[y][k], (int)xv[y][k], (int)vx[y][k], (int)xx[y][k],
                            (int)qv[y][k], (int)vq[y][k]);
            pairs[dst + above + __popc(m32[y] & ((1u << row) - 1u))] = pr;
        }
    }
}

hipError_t launch_ld_mask(int pass, const uint8_t *Gx, const uint8_t *Gv, const uint8_t *Gq, const LdVar *vars,
                          const uint32_t *chrom_id, const LdWindowArgs &a, const uint32_t *tiles, uint32_t ntiles,
                          uint16_t *cnt, LdOffsets off, LdPair *pairs, hipStream_t s) {
    if (!ntiles) return hipSuccess;
    if (a.kp4 % kBK || a.kp4 <= 0 || a.ns > (1 << 21)) return hipErrorInvalidValue;
    // the prefilter's error bound: twice ulp(4 ns^2) plus one
    const double big = 4.0 * (double)a.ns * (double)a.ns;
    const float pe = (float)(big * std::ldexp(1.0, -23) + 1.0);
    if (pass == 1)
        hipLaunchKernelGGL(k_ld_mask<1>, dim3(ntiles), dim3(kWaves * kWave), 0, s, Gx, Gv, Gq, vars, chrom_id, a, tiles,
                           ntiles, cnt, off, pairs, pe);
    else
        hipLaunchKernelGGL(k_ld_mask<2>, dim3(ntiles), dim3(kWaves * kWave), 0, s, Gx, Gv, Gq, vars, chrom_id, a, tiles,
                           ntiles, cnt, off, pairs, pe);
    return hipGetLastError();
}

// the valid-mask and squared-dosage FP4 planes next to the dosage plane (k_ld_pack4): code
// 0/1/2 -> V 1.0 (0x2), Q 0 / 1.0 / 4.0 (0x0 / 0x2 / 0x6); missing (-1) and padding -> 0
__global__ void k_ld_pack_vq(const int8_t *__restrict__ Gc, uint64_t m, int kpad, int ns, uint8_t *__restrict__ Gv,
                             uint8_t *__restrict__ Gq, int kp4) {
    const int per = kp4 / 16;  // 16 output bytes per thread and plane
    const uint64_t total = m * (uint64_t)per;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = t / per;
        const int c = (int)(t - v * per);
        const int8_t *row = Gc + v * (uint64_t)kpad;
        uint32_t in[8] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};  // 32 codes, 4 per dword
        if (c * 32 + 32 <= kpad) {
            const uint4 u0 = reinterpret_cast<const uint4 *>(row)[2 * c];
            const uint4 u1 = reinterpret_cast<const uint4 *>(row)[2 * c + 1];
            in[0] = u0.x, in[1] = u0.y, in[2] = u0.z, in[3] = u0.w;
            in[4] = u1.x, in[5] = u1.y, in[6] = u1.z, in[7] = u1.w;
        }
        uint32_t wv[4] = {0, 0, 0, 0}, wq[4] = {0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 32; e++) {
            const int g = (int8_t)(in[e >> 2] >> (8 * (e & 3)));
            const bool ok = c * 32 + e < ns && g >= 0;
            const uint32_t cv = ok ? 0x2u : 0x0u;
            const uint32_t cq = !ok ? 0x0u : g == 1 ? 0x2u : g == 2 ? 0x6u : 0x0u;
            wv[e >> 3] |= cv << (4 * (e & 7));
            wq[e >> 3] |= cq << (4 * (e & 7));
        }
        reinterpret_cast<uint4 *>(Gv + v * (uint64_t)kp4)[c] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        reinterpret_cast<uint4 *>(Gq + v * (uint64_t)kp4)[c] = make_uint4(wq[0], wq[1], wq[2], wq[3]);
    }
}

hipError_t launch_ld_pack_vq(const int8_t *Gc, uint64_t m, int kpad, int ns, uint8_t *Gv, uint8_t *Gq, int kp4,
                             hipStream_t s) {
    if (!m) return hipSuccess;
    if (kp4 % 64 || 2 * (int64_t)kp4 < ns) return hipErrorInvalidValue;
    const uint64_t total = m * (uint64_t)(kp4 / 16);
    const unsigned grid = (unsigned)std::min<uint64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_ld_pack_vq, dim3(grid), dim3(256), 0, s, Gc, m, kpad, ns, Gv, Gq, kp4);
    return hipGetLastError();
}

}  // namespace vcfxg
