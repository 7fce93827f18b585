// vcfxg_ld_fast.hip -- LD r^2 for 128x128 variant blocks whose genotypes are complete.
//
// The common case of VCFX_ld_calculator's pair loop (computeLDStreamingMmap :511-648 /
// computeLDStreaming :864-987 calling computeRsqFast :397-401): with no missing genotype
// among the ns samples, the pair sums need only S_xy = X.X^T (n = ns and Sx, Sx2 are
// per-variant), so a block is one int8 GEMM tile:
//   * operands: 128 rows of I and 128 rows of J, K = kpad bytes, staged in 64-byte k-slices
//     by global_load_lds (16 B/lane, lane-linear LDS image, XOR-swizzled 16 B slots via the
//     SOURCE address so the ds_read_b128 fragment reads are bank-conflict free), double
//     buffered, one barrier per k-slice;
//   * 4 waves as 2x2, each a 64x64 output = 2x2 v_mfma_i32_32x32x32_i8 accumulators;
//   * epilogue per pair: an exact integer prefilter (C = n*Sxy - Sx*Sy; r^2 = C^2/(Vx*Vy))
//     rejects pairs whose exact r^2 is below threshold - delta without any fp64 division;
//     candidates run the reference's fp64 operation sequence (correctly rounded __d*_rn
//     ops, per-variant mean / variance / sqrt precomputed with the same ops), so the kept
//     r^2 and the threshold decision are bit-identical to the reference;
//   * each wave's 64x64 output is one 64-block of the count table (cnt[row j][column block])
//     shared with the general kernel (vcfxg_ld.hip k_ld_block), so pass 1 counts and pass 2
//     writes pairs in the reference's (j, i) order; pass 2 skips blocks with no pair.
#include "vcfxg_device.h"
#include "vcfxg_ld.h"

namespace vcfxg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kFB = 128;        // block side (variants)
constexpr int kBK = 64;         // k-slice bytes per stage
constexpr int kStage = 2 * kFB * kBK;  // A rows then B rows: 16 KiB
constexpr int kNBuf = 4;               // staging ring depth (kNBuf - 1 stages in flight)
constexpr int kTileBytes = 4 * 64 * 64 * 4;
static_assert(kNBuf * kStage <= kTileBytes, "staging ring must fit under the epilogue tiles");

__device__ __forceinline__ void glds16(const int8_t *src, int8_t *lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

// bijective XCD-aware remap: consecutive list entries (sharing J rows) land on one XCD
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
    const uint32_t q = n / 8, r = n % 8, x = b % 8, k = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

template <int P>
__global__ __launch_bounds__(256) void k_ld_fast(const int8_t *__restrict__ Gc, const LdFast *__restrict__ fv,
                                                 const uint32_t *__restrict__ chrom_id, LdWindowArgs a,
                                                 const uint32_t *__restrict__ blocks, uint32_t nblocks,
                                                 uint16_t *__restrict__ cnt, const uint64_t *__restrict__ off,
                                                 LdPair *__restrict__ pairs) {
    // ONE LDS array (a second __shared__ object makes hipcc drain vmcnt before the k-loop's
    // ds_reads): 3 staging buffers (3 x 16 KiB) during the k-loop, then the 4 waves' 64x64
    // int32 tiles (64 KiB) over them; the per-row prefilter terms after that
    __shared__ __attribute__((aligned(16))) int8_t lds[kTileBytes + kFB * (8 + 4 + 4)];
    double *rvx = reinterpret_cast<double *>(lds + kTileBytes);
    int *rsx = reinterpret_cast<int *>(lds + kTileBytes + kFB * 8);
    float *rvxf = reinterpret_cast<float *>(lds + kTileBytes + kFB * 12);
    const uint32_t b = xcd_remap(blockIdx.x, nblocks);
    const uint32_t I2 = blocks[2 * b], J2 = blocks[2 * b + 1];
    const int t = threadIdx.x, w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int wi = w >> 1, wj = w & 1;
    const int64_t M = (int64_t)a.m;
    const int64_t ibase = (int64_t)I2 * kFB, jbase = (int64_t)J2 * kFB;
    // this wave's 64-block of the count table
    const uint64_t bI = 2ull * I2 + wi, bJ = 2ull * J2 + wj;
    const uint64_t jrow0 = bJ * kLdBlock;
    const uint64_t ifirst = jrow0 > a.window ? (jrow0 - a.window) / kLdBlock : 0;
    const bool slot_ok = bI >= ifirst && bI <= bJ;
    const uint64_t slot = bI - ifirst;
    if (P == 2) {  // emit pass: skip blocks without a counted pair
        const int64_t jj = (int64_t)jrow0 + l;
        uint32_t c = 0;
        if (slot_ok && jj < M && jj >= (int64_t)a.j_lo && jj < (int64_t)a.j_hi)
            c = cnt[(uint64_t)(jj - (int64_t)a.j_lo) * a.nb + slot];
        if (!__syncthreads_or(c != 0)) return;
    }
    if (t < kFB) {
        const int64_t i = ibase + t < M ? ibase + t : M - 1;
        const LdFast f = fv[i];
        rvx[t] = f.vxp;
        rvxf[t] = (float)f.vxp;
        rsx[t] = f.sx;
    }
    const int kpad = a.kpad;
    // staging: 16 wave-instructions of 1 KiB per stage, 4 per wave; instruction q of wave w
    // fills LDS [(4w+q) KiB, +1 KiB) = 16 rows x 64 B; lane l -> row (l>>2), physical slot
    // l&3 holding logical 16 B slot (l&3) ^ ((row>>2)&3)
    const int8_t *src[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int idx = 4 * w + q;
        const int lrow = (idx & 7) * 16 + (l >> 2);  // row within the A or B tile
        int64_t g = (idx < 8 ? ibase : jbase) + lrow;
        if (g >= M) g = M - 1;
        const int logical = (l & 3) ^ ((lrow >> 2) & 3);
        src[q] = Gc + g * (int64_t)kpad + logical * 16;
    }
    auto stage = [&](int ks, int buf) {
#pragma unroll
        for (int q = 0; q < 4; q++) glds16(src[q] + ks * kBK, lds + buf * kStage + (4 * w + q) * 1024);
    };
    v16i acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = v16i{};
    const int nk = kpad / kBK;
    // kNBuf-buffer ring, kNBuf-1 stages in flight: at step ks a wave waits only for its own
    // loads of stage ks (counted vmcnt: the later stages' glds may stay outstanding), then a
    // raw barrier (no __syncthreads: its fence would drain every glds) makes all waves'
    // stage-ks bytes visible and frees buffer (ks-1)%kNBuf, last read at step ks-1
    for (int q = 0; q < kNBuf - 1 && q < nk; q++) stage(q, q);
    for (int ks = 0; ks < nk; ks++) {
        // stages ks+1 .. ks+kNBuf-2 (4 glds each) may stay outstanding
        const int ahead = nk - 1 - ks < kNBuf - 2 ? nk - 1 - ks : kNBuf - 2;
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ks + kNBuf - 1 < nk) stage(ks + kNBuf - 1, (ks + kNBuf - 1) % kNBuf);
        const int8_t *base = lds + (ks % kNBuf) * kStage;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            v4i af[2], bf[2];
#pragma unroll
            for (int x = 0; x < 2; x++) {
                const int ra = wi * 64 + x * 32 + r, rb = wj * 64 + x * 32 + r;
                const int lg = 2 * s + h;
                af[x] = *reinterpret_cast<const v4i *>(base + ra * kBK + ((lg ^ ((ra >> 2) & 3)) << 4));
                bf[x] = *reinterpret_cast<const v4i *>(base + kFB * kBK + rb * kBK + ((lg ^ ((rb >> 2) & 3)) << 4));
            }
#pragma unroll
            for (int x = 0; x < 2; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[x], bf[y], acc[x][y], 0, 0, 0);
        }
    }
    // ---- epilogue.  The 4 waves' 64x64 int32 tiles go to LDS (over the staging buffers), so
    // each lane then owns one column j of its wave's 64-block and walks its 64 rows with
    // runtime indices (low register pressure, a 64-bit pass mask per column, no shuffles).
    __syncthreads();  // every wave is done reading the staging buffers
    int *tile = reinterpret_cast<int *>(lds) + w * 64 * 64;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++)
#pragma unroll
            for (int k = 0; k < 16; k++)
                tile[(32 * x + (k & 3) + 8 * (k >> 2) + 4 * h) * 64 + 32 * y + r] = acc[x][y][k];
    if (!slot_ok) return;  // wave-uniform: a sub-block outside the window triangle
    const int pad = kpad - a.ns;
    const double dn = (double)a.ns;
    const int64_t n = a.ns;
    const int64_t j = (int64_t)jrow0 + l;
    const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
    uint64_t mask = 0;
    LdFast fj{};
    if (jok) {
        fj = fv[j];
        const uint32_t cj = a.max_dist > 0 ? chrom_id[j] : 0u;
        const double rhs_j = a.all_pass ? 0.0 : a.tm * fj.vxp;
        // fp32 form of the prefilter while n*Sxy and Sx*Sy fit int32 (n <= 23170): C exact in
        // int32, C^2 and tm*Vx*Vy within ~1e-6 relative in fp32, so a further 1e-5 relative
        // slack keeps every pair that can reach the threshold
        const bool f32 = a.ns <= 23170;
        const float rhs_jf = (float)(a.tm * (1.0 - 1e-5)) * (float)fj.vxp;
        const int64_t i0 = (int64_t)bI * kLdBlock;
        // rows i in [max(i0, j - window), min(i0 + 64, j))
        const int lo = (int)(j - (int64_t)a.window > i0 ? j - (int64_t)a.window - i0 : 0);
        const int hi = (int)(j - i0 < 64 ? j - i0 : 64);
        for (int row = lo; row < hi; row++) {
            const int lr = wi * 64 + row;
            const int sxy = tile[row * 64 + l] - pad;
            if (!a.all_pass) {
                if (f32) {
                    const float c = (float)(a.ns * sxy - rsx[lr] * fj.sx);
                    if (!(c * c >= rvxf[lr] * rhs_jf)) continue;
                } else {
                    const int64_t C = n * sxy - (int64_t)rsx[lr] * fj.sx;
                    const double c = (double)C;
                    if (!(c * c >= rvx[lr] * rhs_j)) continue;
                }
            }
            const int64_t i = i0 + row;
            const LdFast fi = fv[i];
            if (a.max_dist > 0 && chrom_id[i] == cj) {
                int d = fj.pos - fi.pos;
                if (d < 0) d = -d;
                if (d > a.max_dist) continue;
            }
            if (ld_fast_r2(fi, fj, sxy, dn) >= a.threshold) mask |= 1ull << row;
        }
    }
    if (P == 1) {
        if (jok) cnt[(uint64_t)(j - (int64_t)a.j_lo) * a.nb + slot] = (uint16_t)__popcll(mask);
        return;
    }
    if (!mask) return;
    const uint64_t base = off[(uint64_t)(j - (int64_t)a.j_lo) * a.nb + slot];
    const int64_t i0 = (int64_t)bI * kLdBlock;
    uint32_t rank = 0;
    while (mask) {
        const int row = __builtin_ctzll(mask);
        mask &= mask - 1;
        LdPair pr;
        pr.i = (uint32_t)(i0 + row);
        pr.j = (uint32_t)j;
        pr.r2 = ld_fast_r2(fv[i0 + row], fj, tile[row * 64 + l] - pad, dn);
        pairs[base + rank++] = pr;
    }
}

hipError_t launch_ld_fast(int pass, const int8_t *Gc, const LdFast *fv, const uint32_t *chrom_id,
                          const LdWindowArgs &a, const uint32_t *blocks, uint32_t nblocks, uint16_t *cnt,
                          const uint64_t *off, LdPair *pairs, hipStream_t s) {
    if (!nblocks) return hipSuccess;
    if (a.kpad % kBK) return hipErrorInvalidValue;
    if (pass == 1)
        hipLaunchKernelGGL(k_ld_fast<1>, dim3(nblocks), dim3(256), 0, s, Gc, fv, chrom_id, a, blocks, nblocks, cnt,
                           off, pairs);
    else
        hipLaunchKernelGGL(k_ld_fast<2>, dim3(nblocks), dim3(256), 0, s, Gc, fv, chrom_id, a, blocks, nblocks, cnt,
                           off, pairs);
    return hipGetLastError();
}

// per 128-variant group: 1 if every variant of the group is complete
__global__ void k_ld_groups(const LdVar *__restrict__ vars, uint64_t m, uint8_t *__restrict__ gflag) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x / 64 + threadIdx.x / 64;
    const uint64_t ng = (m + kFB - 1) / kFB;
    if (g >= ng) return;
    const int l = threadIdx.x & 63;
    bool ok = true;
    for (int k = l; k < kFB; k += 64) {
        const uint64_t v = g * kFB + k;
        if (v < m) ok = ok && vars[v].complete;
    }
    ok = __all(ok);
    if (l == 0) gflag[g] = ok ? 1 : 0;
}

hipError_t launch_ld_groups(const LdVar *vars, uint64_t m, uint8_t *gflag, hipStream_t s) {
    const uint64_t ng = (m + kFB - 1) / kFB;
    if (!ng) return hipSuccess;
    hipLaunchKernelGGL(k_ld_groups, dim3((unsigned)((ng + 3) / 4)), dim3(256), 0, s, vars, m, gflag);
    return hipGetLastError();
}

}  // namespace vcfxg
