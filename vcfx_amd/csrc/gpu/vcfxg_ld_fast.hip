// vcfxg_ld_fast.hip -- LD r^2 for 256x256 variant blocks whose genotypes are complete.
//
// The common case of VCFX_ld_calculator's pair loop (computeLDStreamingMmap :511-648 /
// computeLDStreaming :864-987 calling computeRsqFast :397-401): with no missing genotype
// among the ns samples, the pair sums need only S_xy = X.X^T (n = ns and Sx, Sx2 are
// per-variant), so a block is one GEMM tile over the dosages 0/1/2:
//   * operands: FP4 (e2m1) rows -- 0, 1, 2 are exact e2m1 values and every product and
//     partial sum is an integer below 2^24, so the fp32-accumulating block-scaled MFMA
//     (scales 2^0) computes S_xy exactly at twice the int8 rate and half the operand bytes;
//     zero padding needs no correction.  256 rows of I and 256 rows of J, K = kp4 bytes
//     (2 dosages per byte), staged in 64-byte k-slices
//     by global_load_lds (16 B/lane, lane-linear LDS image, XOR-swizzled 16 B slots via the
//     SOURCE address so the ds_read_b128 fragment reads are bank-conflict free) into a
//     4-buffer ring, fragments read one k-half ahead of the MFMAs (counted vmcnt + raw
//     s_barrier between two MFMA groups);
//   * 8 waves as 4 (I) x 2 (J), each a 64x128 output = 2x4 v_mfma_scale_f32_32x32x64_f8f6f4
//     accumulators: per k-step a wave reads 6 fragments for 8 MFMAs, and the block loads
//     32 KiB per 128 MFMAs (half the operand traffic per MFMA of a 128x128 block);
//   * epilogue per 64x64 quarter of a wave's output (two per wave): the int32 tile goes to
//     the wave's own LDS region and each lane walks one column: an exact integer prefilter
//     (C = n*Sxy - Sx*Sy; r^2 = C^2/(Vx*Vy)) rejects pairs whose exact r^2 is below
//     threshold - delta; candidates run the reference's fp64 operation sequence (correctly
//     rounded __d*_rn ops, per-variant mean / variance / sqrt precomputed with the same
//     ops), so the kept r^2 and the threshold decision are bit-identical to the reference;
//   * every 64x64 quarter is one 64-block of the count table (cnt[row j][column block])
//     shared with the general kernel (vcfxg_ld.hip k_ld_block), so pass 1 counts and pass 2
//     writes pairs in the reference's (j, i) order; pass 2 skips blocks with no pair.
#include "vcfxg_device.h"
#include "vcfxg_ld.h"

#include <algorithm>
#include <type_traits>

// VCFXG_LD_EXPT (diagnostic builds only, results invalid): bit 0 skips the epilogue, bit 3
// stages k-slice 0 every step, bit 4 reads rows 0..255 for every block; sparse epilogue: bit 5
// skips the missing-entry gathers, bit 6 the per-pair prefilter, bit 7 the tables and exact
// pairs after the prefilter, bit 8 counts halves / halves with tables / candidates (VCFXG_LD_DEBUG),
// bit 9 skips the exact pass on the candidates, bit 10 the tables (zeroing and gathers), bit 11 both
// behind a run-time test (the code stays in the kernel)
#ifndef VCFXG_LD_EXPT
#define VCFXG_LD_EXPT 0
#endif

namespace vcfxg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int kFmtFp4 = 4;              // cbsz / blgp operand format: e2m1
constexpr int kScaleOne = 0x7F7F7F7F;   // E8M0 block scales 2^0

constexpr int kFB = kLdFastBlock;      // block side (variants): 256
constexpr int kBK = 64;                // k-slice bytes per stage
constexpr int kStage = 2 * kFB * kBK;  // A rows then B rows: 32 KiB
constexpr int kNBuf = 4;               // staging ring depth (kNBuf - 1 stages in flight)
constexpr int kWaves = 8;
constexpr int kRing = kNBuf * kStage;  // 128 KiB
constexpr int kQuarter = 64 * 64 * 4;  // one wave's 64x64 int32 epilogue tile
static_assert(kWaves * kQuarter <= kRing, "epilogue tiles must fit in the staging ring");
constexpr int kGlds = kStage / 1024 / kWaves;  // 1 KiB glds instructions per wave per stage
constexpr int kFvBytes = kFB * 40;             // one side's LdFast records (40 B each)
constexpr int kFvGlds = kFvBytes / 1024;       // 1 KiB pieces of them
static_assert(kFvBytes % 1024 == 0, "the records are DMA'd in whole 1 KiB pieces");
static_assert(sizeof(LdFast) == 40, "LdFast layout");
static_assert(kGlds == 4, "the k-loop's vmcnt counts assume 4 glds per wave per stage");

__device__ __forceinline__ void glds16(const void *src, int8_t *lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

// bijective XCD-aware remap: consecutive list entries (one super-tile) land on one XCD
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
    const uint32_t q = n / 8, r = n % 8, x = b % 8, k = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// exact decision for one candidate pair (kept out of line: the rare path)
__device__ __forceinline__ int ld_exact_pass(const LdFast *__restrict__ fv, const uint32_t *__restrict__ chrom_id,
                                          int max_dist, double threshold, int64_t i, int64_t j, int sxy,
                                          double dn) {
    const LdFast fi = fv[i], fj = fv[j];
    if (max_dist > 0 && chrom_id[i] == chrom_id[j]) {
        int d = fj.pos - fi.pos;
        if (d < 0) d = -d;
        if (d > max_dist) return 0;
    }
    return ld_fast_r2(fi, fj, sxy, dn) >= threshold ? 1 : 0;
}

// Count-pass epilogue straight from the accumulators (no LDS tile): lane (h, r) of a wave
// holds, for each of its 4 column tiles y, column wj*128 + 32y + r and the 32 rows
// 32x + 8g + 4h + e of the wave's 64-row block.  Candidate test per pair in C/n units, two
// pairs per packed fp32 instruction and no conversion (the accumulator is already fp32):
//   c' = Sxy + Sx_i * w_j               w_j = -Sy_j / n            (C' = C / n exactly)
//   candidate iff |c'| >= u_i * v_j - E,  u_i = sqrt(tm' Vx_i) / n, v_j = sqrt(Vy_j)
// Sxy and Sx_i are exact integers in fp32, w_j carries one rounding and the fma one more,
// so |c' - C/n| <= 12 n 2^-24 < E = 32 n 2^-23 for the exact C = n*Sxy - Sx*Sy; tm' =
// tm (1 - 1e-5) absorbs the roundings of u, v (< 1e-6 relative): every pair whose exact r^2
// can reach the threshold (C^2 >= tm Vx Vy) is a candidate.  Candidates (rare at useful
// thresholds) run the exact fp64 r^2 of ld_fast_r2 -- the same decision the LDS-tile
// epilogue and the general kernel make.  tm <= 0 (all_pass): u = v = 0, E = +inf, every
// pair in the window is a candidate.  The two lanes of a column (h = 0, 1) add their counts.
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void ld_count_regs(const v16f (&acc)[2][4], const LdWindowArgs &a,
                                              const LdFast *__restrict__ fv, const uint32_t *__restrict__ chrom_id,
                                              uint16_t *__restrict__ cnt, const float *ru, const float *rsf,
                                              const float *cw, const float *cv, uint32_t I4, uint32_t J4, int wi,
                                              int wj, int h, int r, int (&qtot)[2]) {
    const int64_t M = (int64_t)a.m;
    const double dn = (double)a.ns;
    const uint64_t bI = 4ull * I4 + wi;
    const int64_t i0 = (int64_t)bI * kLdBlock;
    const float negE = a.all_pass ? -INFINITY : -(float)(32.0 * a.ns / 8388608.0);
    int64_t jv[4];
    int lo[4], span[4], nc[4];
    float wv[4], vj[4];
    bool full = true;
#pragma unroll
    for (int y = 0; y < 4; y++) {
        const uint64_t bJ = 4ull * J4 + 2 * wj + (y >> 1);
        const int64_t j = (int64_t)(bJ * kLdBlock) + 32 * (y & 1) + r;
        jv[y] = j;
        const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
        const int cj = (2 * wj + (y >> 1)) * kLdBlock + 32 * (y & 1) + r;  // column within the tile
        wv[y] = cw[cj];
        vj[y] = cv[cj];
        // valid rows [lo, lo + span) of the 64-block: i in [j - window, j)
        const int64_t l0 = j - (int64_t)a.window - i0;
        const int64_t h0 = j - i0;
        const int l = (int)(l0 > 0 ? (l0 < 64 ? l0 : 64) : 0);
        const int hh = (int)(h0 > 0 ? (h0 < 64 ? h0 : 64) : 0);
        lo[y] = l;
        span[y] = jok && hh > l ? hh - l : 0;
        full = full && span[y] == 64;
        nc[y] = 0;
    }
    auto body = [&](auto check) {
        // x outer, then the row groups g: a group's terms (4 rows) are read from LDS once for
        // the four column tiles (r04: inside the (y, x) loop they were read four times, 64
        // ds_read_b128 per lane per block); the rare exact path re-reads them
        auto test2 = [&](int x, int y, int k, const float *rs, const float *uu, float wjj, float vjj, float a0,
                         float a1, bool &c0, bool &c1) {
            const f2 c = __builtin_elementwise_fma(f2{rs[0], rs[1]}, f2{wjj, wjj}, f2{a0, a1});
            const f2 tt = __builtin_elementwise_fma(f2{uu[0], uu[1]}, f2{vjj, vjj}, f2{negE, negE});
            c0 = fabsf(c.x) >= tt.x;
            c1 = fabsf(c.y) >= tt.y;
            if (decltype(check)::value) {
                const int row = 32 * x + 8 * (k >> 2) + 4 * h + (k & 3);
                c0 = c0 & ((unsigned)(row - lo[y]) < (unsigned)span[y]);
                c1 = c1 & ((unsigned)(row + 1 - lo[y]) < (unsigned)span[y]);
            }
        };
#pragma unroll
        for (int x = 0; x < 2; x++) {
            bool any[4] = {false, false, false, false};
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int lr = wi * 64 + 32 * x + 8 * g + 4 * h;
                const float4 a4 = *reinterpret_cast<const float4 *>(rsf + lr);
                const float4 u4 = *reinterpret_cast<const float4 *>(ru + lr);
                const float rsg[4] = {a4.x, a4.y, a4.z, a4.w}, uug[4] = {u4.x, u4.y, u4.z, u4.w};
#pragma unroll
                for (int y = 0; y < 4; y++)
#pragma unroll
                    for (int e2 = 0; e2 < 4; e2 += 2) {
                        const int k = 4 * g + e2;
                        bool c0, c1;
                        test2(x, y, k, rsg + e2, uug + e2, wv[y], vj[y], acc[x][y][k], acc[x][y][k + 1], c0, c1);
                        any[y] = any[y] | c0 | c1;
                        __builtin_amdgcn_sched_barrier(0);  // keep the pairs' temporaries short-lived
                    }
            }
#pragma unroll
            for (int y = 0; y < 4; y++) {
                // only lanes holding a candidate: exact fp64 r^2 (out of line)
                if (any[y]) {
                    // recomputed from laundered operands and re-read terms: sharing the test's
                    // temporaries would keep them live (and spilled) across it for this rare path
                    float wjj = wv[y], vjj = vj[y];
                    asm volatile("" : "+v"(wjj), "+v"(vjj));
#pragma unroll
                    for (int k = 0; k < 16; k += 2) {
                        float a0 = acc[x][y][k], a1 = acc[x][y][k + 1];
                        asm volatile("" : "+v"(a0), "+v"(a1));
                        const int lr = wi * 64 + 32 * x + 8 * (k >> 2) + 4 * h + (k & 3);
                        const float rs2[2] = {rsf[lr], rsf[lr + 1]}, uu2[2] = {ru[lr], ru[lr + 1]};
                        bool c[2];
                        test2(x, y, k, rs2, uu2, wjj, vjj, a0, a1, c[0], c[1]);
#pragma unroll
                        for (int e = 0; e < 2; e++)
                            if (c[e])
                                nc[y] += ld_exact_pass(fv, chrom_id, a.max_dist, a.threshold,
                                                       i0 + 32 * x + 8 * ((k + e) >> 2) + 4 * h + ((k + e) & 3), jv[y],
                                                       (int)(e ? a1 : a0), dn);
                    }
                }
            }
        }
    };
    if (__all(full)) body(std::integral_constant<bool, false>{});
    else body(std::integral_constant<bool, true>{});
#pragma unroll
    for (int y = 0; y < 4; y++) {
        const int tot = nc[y] + __shfl_xor(nc[y], 32);
        const uint64_t bJ = 4ull * J4 + 2 * wj + (y >> 1);
        const uint64_t jrow0 = bJ * kLdBlock;
        const uint64_t ifirst = jrow0 > a.window ? (jrow0 - a.window) / kLdBlock : 0;
        const int64_t j = jv[y];
        const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
        if (h == 0 && jok && bI >= ifirst && bI <= bJ)
            cnt[(uint64_t)(j - (int64_t)a.j_lo) * a.nb + (bI - ifirst)] = (uint16_t)tot;
        nc[y] = h == 0 && jok && bI >= ifirst && bI <= bJ ? tot : 0;
    }
    qtot[0] = wave_sum(nc[0] + nc[1]);  // quarter hy = columns of tiles 2hy, 2hy+1
    qtot[1] = wave_sum(nc[2] + nc[3]);
}

// ---- the sparse-missing epilogue (kSp) ------------------------------------------------------
// computeRsqSIMD (VCFX_ld_calculator.cpp:352-393) sums over the samples valid in BOTH variants.
// With a missing call coded 0 in the FP4 plane, the k-loop's X_i . X_j is already Sxy over them;
// the other five sums differ from the per-variant ones only at the few missing samples
// (M_i: the samples variant i misses, |M_i| <= kLdSparseMax in these groups):
//   n   = ns - |M_i| - |M_j| + |M_i n M_j|
//   Sx  = SX_i - sum_{s in M_j} x_is       Sxx = SQ_i - sum_{s in M_j} x_is^2
//   Sy  = SX_j - sum_{s in M_i} x_js       Syy = SQ_j - sum_{s in M_i} x_js^2
// (x = 0 where missing).  Per column half hp (128 columns) the block adds, for every missing
// entry (i, s) of its rows, the 128 contributions gt16[s][J-half] into R[i][.] and, for every
// entry (j, s) of the half's columns, the 256 contributions gt16[s][I] into C[j][.]: packed u16
// c = x | x^2 << 5 | missing << 11, whose sums stay in their fields for <= 15 entries (LDS
// atomic adds of u16 pairs).  So R[i][j] = (Sum x_js, Sum x_js^2, |M_i n M_j|) over s in M_i and
// C[j][i] = (Sum x_is, Sum x_is^2, .) over s in M_j.  Then the half's waves run the exact
// prefilter and fp64 sequence of k_ld_mask on each pair.
#ifndef VCFXG_LD_SP_ROWU
#define VCFXG_LD_SP_ROWU 8
#endif
#ifndef VCFXG_LD_SP_COLU
#define VCFXG_LD_SP_COLU 4
#endif
constexpr int kSpRowU = VCFXG_LD_SP_ROWU, kSpColU = VCFXG_LD_SP_COLU;
// VCFXG_LD_SP_TABLES=1: the R / C tables (every missing entry's plane row gathered into LDS by
// atomic adds, for every half holding a candidate); 0 (default, r05): each candidate's two
// corrections summed straight from the CSR and the plane (sp_corr)
#ifndef VCFXG_LD_SP_TABLES
#define VCFXG_LD_SP_TABLES 0
#endif
constexpr bool kSpTables = VCFXG_LD_SP_TABLES != 0;
// VCFXG_LD_SP_R2CACHE=1 (default, r05): the emit writes a passing pair with the r^2 its decision
// computed, kept in the staging ring (dead in the epilogue when no R / C tables overlay it):
// kSpR2Cap doubles per wave, by the pair's position in the wave's list sequence; a wave with
// more candidates recomputes them.  0: the emit recomputes every pair
#ifndef VCFXG_LD_SP_R2CACHE
#define VCFXG_LD_SP_R2CACHE 1
#endif
constexpr bool kSpR2Cache = VCFXG_LD_SP_R2CACHE != 0 && !kSpTables;

// sum over s in M_u (variant u's missing samples, CSR) of the plane's packed c(x_vs): (Sum x,
// Sum x^2, the count of s where v misses too) in their u16 fields; mu = |M_u| (<= kLdSparseMax).
// The sample indices of a step of 4 are loaded together, then their plane entries: two round trips
// per step, the steps up to the active lanes' largest count
__device__ __forceinline__ uint32_t sp_corr(const LdSparse &sp, uint64_t u, uint64_t v, int mu) {
    // u's missing samples from its padded 16-entry list (two 16 B loads), then their plane entries
    const uint4 *ml = reinterpret_cast<const uint4 *>(sp.midx16 + u * 16);
    const uint4 m0 = ml[0];
    const uint4 m1 = mu > 8 ? ml[1] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t w[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    uint32_t acc = 0;
#pragma unroll
    for (int b = 0; b < 16; b += 4) {
        if (!__ballot(b < mu)) break;  // (the active lanes' largest count reached)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t si = (w[(b + q) >> 1] >> (16 * ((b + q) & 1))) & 0xFFFFu;
            acc += b + q < mu ? (uint32_t)sp.gt16[(uint64_t)si * sp.mp + v] : 0u;
        }
    }
    return acc;
}
constexpr int kSpR = 0;                           // R: [256 rows][128 cols] u16
constexpr int kSpCStride = 260;                   // C: [128 cols][256 rows + 4 pad] u16
constexpr int kSpC = 256 * 128 * 2;
constexpr int kSpRC = kSpC + 128 * kSpCStride * 2;  // 132,096 B (the ring and the dense terms)
constexpr int kSpInts = kRing + kFB * 32;         // per row / column packed sums (the records' area)
static_assert(kSpRC <= kSpInts, "R and C must not reach the packed sums");
// (the tile's 512 LdSpRec records, 16 B each: 8 KiB, DMA'd with the first k-slices as the dense
// kernel's LdFast records, so the epilogue starts without a global load)
constexpr int kSpRecBytes = 2 * kFB * (int)sizeof(LdSpRec);
static_assert(kSpRecBytes == 8 * 1024, "one 1 KiB piece per wave");
// the prefilter's per-row (5) and per-column (3) fp32 terms and the block maxima, after them
constexpr int kSpTerms = kSpInts + kSpRecBytes;
// the exact pass's per-wave work list over the terms once the prefilter is done: 4 waves per half,
// kSpList 8 B entries (then, for the emit, kSpList destinations after them)
constexpr int kSpList = 128;
constexpr int kSpR2Cap = kRing / (kWaves * 8);  // 2,048 cached r^2 per wave
static_assert(4 * kSpList * 16 <= 8 * kFB * 4, "the work lists fit the prefilter terms");
static_assert(kSpTerms + 8 * kFB * 4 + 16 <= kRing + kFB * 32 + 2 * kFvBytes, "prefilter terms fit the records' area");

// a row's / column's (missing count, Sx, Sx2) packed for one 64-bit LDS read
__device__ __forceinline__ uint64_t sp_pack(int m, int sx, int sx2) {
    return (uint64_t)(uint32_t)m | ((uint64_t)(uint32_t)sx << 8) | ((uint64_t)(uint32_t)sx2 << 32);
}

// The sparse epilogue's prefilter (every wave, on its own accumulators, before any table).
// Per variant, over its own present samples: N = ns - m, S, Q, V = N Q - S^2, xs its largest
// dosage (1 when Q == S).  The pair's common samples drop k_i <= m_j of variant i's, whose sums
// a_i <= min(k_i xs_i, S_i) and b_i <= min(k_i xs_i^2, Q_i) leave (MI / MJ the block's largest
// missing counts over its rows / columns, am = min(M_other xs, S), AI / AJ the largest am over
// the rows / columns):
//   |C| <= |N_i Sxy - S_i S_j| + MJ Sxy + AJ (S_i + am_i) + AI S_j + E
//   Vx  >= V_i - N_i min(MJ xs_i^2, Q_i) - MJ Q_i           (Vy alike, with MI)
// (C - (N_i Sxy - S_i S_j) = (m_ij - m_j) Sxy + S_i a_j + S_j a_i - a_i a_j with n = N_i - k_i,
// k_i = m_j - m_ij, Sx = S_i - a_i, Sy = S_j - a_j; E = 16 ulps of 4 ns^2 covers the fp32 roundings), so a
// pair whose exact r^2 reaches tm has |C| >= sqrt(tm' Vxmin Vymin): it is a candidate.  A
// variant that fails mask_r2's own-variance gate never is.  Per two rows of a column: five
// packed fp32 instructions and two compares (the dense register epilogue's form).
__device__ __forceinline__ void ld_sparse_prefilter(const v16f (&acc)[2][4], int8_t *lds, const LdWindowArgs &a,
                                                    const LdSparse &sp, uint32_t I4, uint32_t J4,
                                                    uint32_t (&cbm)[4][2]) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int wi = w >> 1, wj = w & 1;
    const int64_t M = (int64_t)a.m;
    const int64_t ibase = (int64_t)I4 * kFB, jbase = (int64_t)J4 * kFB;
    float *tS = reinterpret_cast<float *>(lds + kSpTerms);
    float *tN = tS + kFB, *tU = tN + kFB, *tM = tU + kFB, *tD = tM + kFB;
    float *cS = tD + kFB, *cV = cS + kFB, *cE = cV + kFB;
    int *mx = reinterpret_cast<int *>(cE + kFB);  // MI, MJ, AI, AJ
    if (t < 4) mx[t] = 0;
    __syncthreads();
    {
        const bool row = t < kFB;
        const int64_t v = row ? ibase + t : jbase + (t - kFB);
        const bool vok = v < M;
        const LdSpRec rc = reinterpret_cast<const LdSpRec *>(lds + kSpInts)[t];  // (zero past M)
        struct {
            int cnt, sx, sx2;
            double varx;
        } x;
        x.cnt = a.ns - (int)(rc.pk & 0xFF);
        x.sx = (int)((rc.pk >> 8) & 0xFFFFFF);
        x.sx2 = (int)(rc.pk >> 32);
        x.varx = rc.varx;
        const int mv = vok ? a.ns - x.cnt : 0;
        const int xs = x.sx2 != x.sx ? 2 : 1;
        atomicMax(&mx[row ? 0 : 1], mv);
        __syncthreads();
        const int Mo = row ? mx[1] : mx[0];  // the other side's largest missing count
        const int am = vok ? min(Mo * xs, x.sx) : 0;
        atomicMax(&mx[row ? 2 : 3], am);
        __syncthreads();
        const int AI = mx[2], AJ = mx[3];
        const double N = x.cnt, S = x.sx, Q = x.sx2;
        const double vmin = N * Q - S * S - N * fmin((double)(Mo * xs * xs), Q) - (double)Mo * Q;
        const bool live = vok && x.varx > 0.0;
        if (row) {
            const float tmf = (float)(a.tm * (1.0 - 1e-5));
            const float E = (float)(4.0 * a.ns * (double)a.ns * 0x1p-18);
            tS[t] = (float)x.sx;
            tN[t] = (float)x.cnt;
            tU[t] = live ? sqrtf(tmf * (float)fmax(vmin, 0.0)) : INFINITY;
            tM[t] = -(float)Mo;
            tD[t] = -((float)AJ * (float)(x.sx + am) + E);
        } else {
            const int c = t - kFB;
            cS[c] = (float)x.sx;
            cV[c] = live ? sqrtf((float)fmax(vmin, 0.0)) : INFINITY;
            cE[c] = -(float)AI * (float)x.sx;
        }
    }
    __syncthreads();
    const int64_t i0 = (int64_t)(4ull * I4 + wi) * kLdBlock;
    float Sj[4], Vj[4], Ej[4];
    int lo[4], span[4];
    bool full = true;
#pragma unroll
    for (int y = 0; y < 4; y++) {
        const int cj = 128 * wj + 32 * y + r;
        const int64_t j = jbase + cj;
        Sj[y] = cS[cj], Vj[y] = cV[cj], Ej[y] = cE[cj];
        const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
        // valid rows [lo, lo + span) of the wave's 64: i in [j - window, j)
        const int64_t l0 = j - (int64_t)a.window - i0, h0 = j - i0;
        const int lw = (int)(l0 > 0 ? (l0 < 64 ? l0 : 64) : 0);
        const int hw = (int)(h0 > 0 ? (h0 < 64 ? h0 : 64) : 0);
        lo[y] = lw;
        span[y] = jok && hw > lw ? hw - lw : 0;
        full = full && span[y] == 64;
#pragma unroll
        for (int x = 0; x < 2; x++) cbm[y][x] = a.all_pass ? 0xFFFFu : 0u;
    }
    if (!a.all_pass) {
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int lr = wi * 64 + 32 * x + 8 * g + 4 * h;
                const float4 S4 = *reinterpret_cast<const float4 *>(tS + lr);
                const float4 N4 = *reinterpret_cast<const float4 *>(tN + lr);
                const float4 U4 = *reinterpret_cast<const float4 *>(tU + lr);
                const float4 M4 = *reinterpret_cast<const float4 *>(tM + lr);
                const float4 D4 = *reinterpret_cast<const float4 *>(tD + lr);
#pragma unroll
                for (int e2 = 0; e2 < 4; e2 += 2) {
                    const f2 Si = e2 ? f2{S4.z, S4.w} : f2{S4.x, S4.y};
                    const f2 Ni = e2 ? f2{N4.z, N4.w} : f2{N4.x, N4.y};
                    const f2 Ui = e2 ? f2{U4.z, U4.w} : f2{U4.x, U4.y};
                    const f2 Mi = e2 ? f2{M4.z, M4.w} : f2{M4.x, M4.y};
                    const f2 Di = e2 ? f2{D4.z, D4.w} : f2{D4.x, D4.y};
                    const int k = 4 * g + e2;
#pragma unroll
                    for (int y = 0; y < 4; y++) {
                        const f2 A = f2{acc[x][y][k], acc[x][y][k + 1]};
                        const f2 Pp = Si * f2{Sj[y], Sj[y]};
                        const f2 C = __builtin_elementwise_fma(Ni, A, -Pp);
                        const f2 R = __builtin_elementwise_fma(Ui, f2{Vj[y], Vj[y]}, f2{Ej[y], Ej[y]});
                        const f2 T = __builtin_elementwise_fma(Mi, A, R) + Di;
                        cbm[y][x] |= (fabsf(C.x) >= T.x ? 1u << k : 0u) | (fabsf(C.y) >= T.y ? 2u << k : 0u);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // (one row group's terms live at a time)
            }
    }
    if (!__all(full)) {
#pragma unroll
        for (int y = 0; y < 4; y++)
#pragma unroll
            for (int x = 0; x < 2; x++) {
                uint32_t vm = 0;
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const int row = 32 * x + 8 * (k >> 2) + 4 * h + (k & 3);
                    vm |= (unsigned)(row - lo[y]) < (unsigned)span[y] ? 1u << k : 0u;
                }
                cbm[y][x] &= vm;
            }
    }
}

template <int P>
__device__ __forceinline__ void ld_sparse_epilogue(const v16f (&acc)[2][4], int8_t *lds, const LdWindowArgs &a,
                                                   const LdSparse &sp, const uint32_t *__restrict__ chrom_id,
                                                   uint32_t I4, uint32_t J4, uint16_t *__restrict__ cnt,
                                                   LdOffsets off, LdPair *__restrict__ pairs, const LdStage &st) {
    // (w wave-uniform: the CSR entry indices and their sample / variant loads are scalar)
    const int t = threadIdx.x, w = __builtin_amdgcn_readfirstlane(t >> 6), l = t & 63, r = l & 31, h = l >> 5;
    const int wi = w >> 1, wj = w & 1;
    const int64_t M = (int64_t)a.m;
    const int64_t ibase = (int64_t)I4 * kFB, jbase = (int64_t)J4 * kFB;
    // the tile's records ([256 rows][256 columns], DMA'd): packed sums and own variances
    const LdSpRec *rec = reinterpret_cast<const LdSpRec *>(lds + kSpInts);
    uint32_t *R32 = reinterpret_cast<uint32_t *>(lds + kSpR);
    uint32_t *C32 = reinterpret_cast<uint32_t *>(lds + kSpC);
    const uint16_t *R16 = reinterpret_cast<const uint16_t *>(lds + kSpR);
    const uint16_t *C16 = reinterpret_cast<const uint16_t *>(lds + kSpC);
    const uint64_t bI = 4ull * I4 + wi;
    // ---- the prefilter, on every wave's own accumulators (before the tables): a bound on the
    // pair's r^2 from the per-variant sums and the block's largest missing counts, in the
    // register epilogue's packed form; only halves holding a candidate build the tables
    uint32_t cbm[4][2];
    ld_sparse_prefilter(acc, lds, a, sp, I4, J4, cbm);
    // Sxy <= 4 ns < 2^16 (ns <= 16383, launch_ld_sparse): the accumulators as u16 pairs, half the
    // registers through the rest of the epilogue
    // (only a wave holding a candidate reads them: nearly every wave of a tile away from the
    // diagonal holds none and skips the packing, as it skips every per-pair step below)
    uint32_t accp[2][4][8];
    uint32_t cor = 0;
#pragma unroll
    for (int y = 0; y < 4; y++) cor |= cbm[y][0] | cbm[y][1];
    if (__builtin_amdgcn_ballot_w64(cor != 0u) != 0)
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int q = 0; q < 8; q++)
                    accp[x][y][q] = (uint32_t)(int)acc[x][y][2 * q] | ((uint32_t)(int)acc[x][y][2 * q + 1] << 16);
    // the row entries are contiguous in the CSR (rows ibase .. ibase + 255)
    const uint64_t re0 = sp.moff[ibase], re1 = sp.moff[ibase + kFB < M ? ibase + kFB : M];
    for (int hp = 0; hp < 2; hp++) {
        const int64_t jb = jbase + 128 * hp;  // this half's first column
        uint32_t anyc = 0;
        if (wj == hp)
#pragma unroll
            for (int y = 0; y < 4; y++) anyc |= cbm[y][0] | cbm[y][1];
        // (no candidate in the half: no tables; its counts are written as 0 below)
        const bool tables = __syncthreads_or(anyc != 0u) && kSpTables && !(VCFXG_LD_EXPT & (128 | 1024)) &&
                            !((VCFXG_LD_EXPT & 2048) && a.ns >= 0);
        if ((VCFXG_LD_EXPT & 256) && P == 1) {  // (diagnostic: halves, halves with tables, candidates)
            if (t == 0) {
                atomicAdd(st.ctr + 4, 1ull);
                if (tables) atomicAdd(st.ctr + 5, 1ull);
            }
            const int nca = wave_sum(wj == hp ? (int)(__popc(cbm[0][0]) + __popc(cbm[0][1]) + __popc(cbm[1][0]) +
                                                      __popc(cbm[1][1]) + __popc(cbm[2][0]) + __popc(cbm[2][1]) +
                                                      __popc(cbm[3][0]) + __popc(cbm[3][1])) : 0);
            if (l == 0 && nca) atomicAdd(st.ctr + 6, (unsigned long long)nca);
        }
        if (tables) {
        for (int k = t * 16; k < kSpRC; k += kWaves * kWave * 16) *reinterpret_cast<uint4 *>(lds + k) = make_uint4(0, 0, 0, 0);
        __syncthreads();
        // row side: entry (i, s) adds gt16[s][jb + 0..127] into R[i][.]: lane l, columns 2l, 2l + 1.
        // The gathers are latency-bound (one 256 / 512 B row piece per entry, gt16 is not L2-
        // resident): kSpRowU / kSpColU entries' loads in flight per wave
        if (!(VCFXG_LD_EXPT & 32)) {
            const uint16_t *col = sp.gt16 + jb + 2 * l;
            uint64_t e = re0 + w;
            for (; e + (kSpRowU - 1) * kWaves < re1; e += kSpRowU * kWaves) {
                uint32_t vv[kSpRowU], ii[kSpRowU];
#pragma unroll
                for (int u = 0; u < kSpRowU; u++) {
                    const uint64_t eu = e + u * kWaves;
                    ii[u] = sp.mvar[eu] - (uint32_t)ibase;
                    vv[u] = *reinterpret_cast<const uint32_t *>(col + (uint64_t)sp.midx[eu] * sp.mp);
                }
#pragma unroll
                for (int u = 0; u < kSpRowU; u++) atomicAdd(&R32[ii[u] * 64 + l], vv[u]);
            }
            for (; e < re1; e += kWaves) {
                const uint32_t ii = sp.mvar[e] - (uint32_t)ibase;
                atomicAdd(&R32[ii * 64 + l], *reinterpret_cast<const uint32_t *>(col + (uint64_t)sp.midx[e] * sp.mp));
            }
        }
        // column side: entry (j, s) adds gt16[s][ibase + 0..255] into C[j][.]: lane l, rows 4l..4l+3
        if (jb < M && !(VCFXG_LD_EXPT & 32)) {
            const uint64_t ce0 = sp.moff[jb], ce1 = sp.moff[jb + 128 < M ? jb + 128 : M];
            const uint16_t *col = sp.gt16 + ibase + 4 * l;
            uint64_t e = ce0 + w;
            for (; e + (kSpColU - 1) * kWaves < ce1; e += kSpColU * kWaves) {
                uint32_t jj[kSpColU];
                uint2 vv[kSpColU];
#pragma unroll
                for (int u = 0; u < kSpColU; u++) {
                    const uint64_t eu = e + u * kWaves;
                    jj[u] = sp.mvar[eu] - (uint32_t)jb;
                    vv[u] = *reinterpret_cast<const uint2 *>(col + (uint64_t)sp.midx[eu] * sp.mp);
                }
#pragma unroll
                for (int u = 0; u < kSpColU; u++) {
                    atomicAdd(&C32[jj[u] * (kSpCStride / 2) + 2 * l], vv[u].x);
                    atomicAdd(&C32[jj[u] * (kSpCStride / 2) + 2 * l + 1], vv[u].y);
                }
            }
            for (; e < ce1; e += kWaves) {
                const uint32_t jj = sp.mvar[e] - (uint32_t)jb;
                const uint2 vv = *reinterpret_cast<const uint2 *>(col + (uint64_t)sp.midx[e] * sp.mp);
                atomicAdd(&C32[jj * (kSpCStride / 2) + 2 * l], vv.x);
                atomicAdd(&C32[jj * (kSpCStride / 2) + 2 * l + 1], vv.y);
            }
        }
        __syncthreads();
        }
        if (wj == hp) {
            // the pairs of this wave: column j = jb + 32y + r, rows i0 + 32x + 8g + 4h + e; per
            // (y, x) the prefilter's 16-bit candidate mask over k = 4g + e.  The exact work (the six
            // sums from the tables, mask_r2's fp64 sequence) is spread over the wave's 64 lanes: a
            // lane's candidates are listed in LDS (row, column, Sxy) in rank order and every lane
            // takes every 64th entry, so a half whose candidates crowd a few columns (pairs inside an
            // LD block) costs total / 64 sequences, not the busiest lane's count
            uint2 *lst = reinterpret_cast<uint2 *>(lds + kSpTerms + wi * kSpList * 16);  // (the dead terms)
            int64_t jv[4];
            bool jokv[4];
#pragma unroll
            for (int y = 0; y < 4; y++) {
                jv[y] = jb + 32 * y + r;
                jokv[y] = jv[y] < M && jv[y] >= (int64_t)a.j_lo && jv[y] < (int64_t)a.j_hi;
            }
            // Sxy of (x, y, k) from the packed accumulators, all three run-time indices (a select tree
            // on their bits: a select chain on a value was once turned into an indexed load, the packed
            // accumulators moved to scratch -- 256 B per lane per block written to memory)
            auto sxy_of = [&](int x, int y, int k) -> uint32_t {
                const int q = k >> 1;
                uint32_t v4[2][4];
#pragma unroll
                for (int xx = 0; xx < 2; xx++)
#pragma unroll
                    for (int yy = 0; yy < 4; yy++) {
                        const uint32_t a0 = (q & 1) ? accp[xx][yy][1] : accp[xx][yy][0];
                        const uint32_t a1 = (q & 1) ? accp[xx][yy][3] : accp[xx][yy][2];
                        const uint32_t a2 = (q & 1) ? accp[xx][yy][5] : accp[xx][yy][4];
                        const uint32_t a3 = (q & 1) ? accp[xx][yy][7] : accp[xx][yy][6];
                        const uint32_t b0 = (q & 2) ? a1 : a0, b1 = (q & 2) ? a3 : a2;
                        v4[xx][yy] = (q & 4) ? b1 : b0;
                    }
                uint32_t vx[4];
#pragma unroll
                for (int yy = 0; yy < 4; yy++) vx[yy] = x ? v4[1][yy] : v4[0][yy];
                const uint32_t c0 = (y & 1) ? vx[1] : vx[0], c1 = (y & 1) ? vx[3] : vx[2];
                const uint32_t v = (y & 2) ? c1 : c0;
                return (v >> (16 * (k & 1))) & 0xFFFFu;
            };
            // a listed pair (il: row in the tile, jl: column in the half, Sxy): its r^2 (mask_r2) and
            // whether it is kept (max_dist, threshold)
            auto exact = [&](uint32_t d0, double &r2) -> bool {
                const int il = (int)(d0 & 0xFF), jl = (int)((d0 >> 8) & 0x7F), sxy = (int)(d0 >> 16);
                const int jt = kFB + 128 * hp + jl;
                const LdSpRec ri = rec[il], rj = rec[jt];
                uint32_t rv, cv;
                if constexpr (kSpTables) {
                    rv = R16[il * 128 + jl];
                    cv = C16[jl * kSpCStride + il];
                } else {  // R[i][j] = over M_i of c(x_js), C[j][i] = over M_j of c(x_is)
                    const uint64_t i = (uint64_t)(ibase + il), j = (uint64_t)(jb + jl);
                    rv = sp_corr(sp, i, j, (int)(ri.pk & 0xFF));
                    cv = sp_corr(sp, j, i, (int)(rj.pk & 0xFF));
                }
                const int n = a.ns - (int)(ri.pk & 0xFF) - (int)(rj.pk & 0xFF) + (int)(rv >> 11);
                const int sx = (int)((ri.pk >> 8) & 0xFFFFFF) - (int)(cv & 31);
                const int sxx = (int)(ri.pk >> 32) - (int)((cv >> 5) & 63);
                const int sy = (int)((rj.pk >> 8) & 0xFFFFFF) - (int)(rv & 31);
                const int syy = (int)(rj.pk >> 32) - (int)((rv >> 5) & 63);
                if (a.max_dist > 0) {
                    const int64_t i = ibase + il, j = jb + jl;
                    if (chrom_id[i] == chrom_id[j]) {
                        int d = sp.vars[j].pos - sp.vars[i].pos;
                        if (d < 0) d = -d;
                        if (d > a.max_dist) return false;
                    }
                }
                r2 = mask_r2(ri.varx, rj.varx, n, sx, sy, sxy, sxx, syy);
                return r2 >= a.threshold;
            };
            // (the row of bit k of mask (y, x) in the wave's 64)
            auto row_of = [&](int x, int k) { return 32 * x + 8 * (k >> 2) + 4 * h + (k & 3); };
            // Lane-parallel passes over per-lane pair sets, one 32-bit word per column y (bit b: x = b
            // >> 4, k = b & 15).  In rounds, every lane with a pair left lists its next one (slot from
            // a ballot), so the list fills kWave entries per round however unevenly the lanes hold
            // pairs; put(y, b, slot) lists a pair, run(e) handles entry e on lane e % 64, get(y, b,
            // slot) replays the rounds on the owning lanes to read the outcome back
            auto word_of = [&](const uint32_t (&W)[4], int y) {
                const uint32_t c0 = (y & 1) ? W[1] : W[0], c1 = (y & 1) ? W[3] : W[2];
                return (y & 2) ? c1 : c0;
            };
            auto adv_of = [&](const uint32_t (&W)[4], int &y, uint32_t &rm) {
                while (rm == 0u && y < 3) rm = word_of(W, ++y);
            };
            // one list's rounds from the state (y, rm): fn(y, b, e) per listed pair; returns the count
            auto rounds_of = [&](const uint32_t (&W)[4], int &y, uint32_t &rm, auto fn) {
                int n = 0;
#pragma unroll
                for (int rd = 0; rd < kSpList / kWave; rd++) {
                    const uint64_t bl = __builtin_amdgcn_ballot_w64(rm != 0u);
                    if (bl == 0) break;  // (wave-uniform)
                    if (rm != 0u) {
                        const int e = n + (int)__builtin_amdgcn_mbcnt_hi(
                                              (uint32_t)(bl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
                        fn(y, __builtin_ctz(rm), e);
                        rm &= rm - 1u;
                        adv_of(W, y, rm);
                    }
                    n += __popcll(bl);
                }
                return n;
            };
            auto spread = [&](const uint32_t (&W)[4], auto put, auto run, auto get) {
                if (__builtin_amdgcn_ballot_w64((W[0] | W[1] | W[2] | W[3]) != 0u) == 0) return;  // (usual)
                auto rounds = [&](int &y, uint32_t &rm, auto fn) { return rounds_of(W, y, rm, fn); };
                int y = 0;
                uint32_t rm = W[0];
                adv_of(W, y, rm);
                for (int base = 0;;) {
                    int yr = y;
                    uint32_t rr = rm;
                    const int n = rounds(y, rm, put);
                    if (n == 0) break;  // (wave-uniform)
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    for (int e = l; e < n; e += kWave) run(e, base + e);
                    base += n;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    rounds(yr, rr, get);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();  // (the list is rewritten by the next chunk)
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            };
            // the exact decision on every candidate; each listed pair's r^2 kept in the list's second
            // half (free until the emit), so when the wave's candidates fit one list -- the usual
            // case -- the emit writes the passing pairs from it instead of recomputing them
            double *const r2c = reinterpret_cast<double *>(lds + w * kSpR2Cap * 8);
            uint32_t passW[4];
            uint32_t candW[4];
            {
#pragma unroll
                for (int y = 0; y < 4; y++) {
                    candW[y] = (VCFXG_LD_EXPT & (128 | 512)) || ((VCFXG_LD_EXPT & 2048) && a.ns >= 0)
                                   ? 0u
                                   : cbm[y][0] | cbm[y][1] << 16;
                    passW[y] = 0;
                }
                spread(
                    candW,
                    [&](int y, int b, int e) {
                        const int x = b >> 4, k = b & 15;
                        lst[e] = make_uint2((uint32_t)(wi * 64 + row_of(x, k)) | (uint32_t)(32 * y + r) << 8 |
                                                sxy_of(x, y, k) << 16,
                                            0u);
                    },
                    [&](int e, int eg) {
                        double r2 = 0.0;
                        lst[e].y = exact(lst[e].x, r2) ? 1u : 0u;
                        if (kSpR2Cache && eg < kSpR2Cap) r2c[eg] = r2;
                    },
                    [&](int y, int b, int e) {
                        const uint32_t bit = lst[e].y ? 1u << b : 0u;
#pragma unroll
                        for (int yy = 0; yy < 4; yy++) passW[yy] |= yy == y ? bit : 0u;
                    });
            }
            uint32_t pass[4][2];
#pragma unroll
            for (int y = 0; y < 4; y++) {
                pass[y][0] = passW[y] & 0xFFFFu;
                pass[y][1] = passW[y] >> 16;
            }
            // the column's 64-row mask (both lanes h of column r hold it): row = 32x + 8g + 4h + e
            auto full_of = [&](int y) {
                uint64_t m64 = 0;
#pragma unroll
                for (int x = 0; x < 2; x++)
#pragma unroll
                    for (int k = 0; k < 16; k++)
                        if ((pass[y][x] >> k) & 1u) m64 |= 1ull << row_of(x, k);
                return m64 | (uint64_t)__shfl_xor((long long)m64, 32);
            };
            auto slot_of = [&](int y, uint64_t &slot) {  // the count-table slot of (bI, column j's 64-block)
                const uint64_t bJ = 4ull * J4 + 2 * hp + (y >> 1);
                const uint64_t jrow0 = bJ * kLdBlock;
                const uint64_t ifirst = jrow0 > a.window ? (jrow0 - a.window) / kLdBlock : 0;
                slot = bI - ifirst;
                return bI >= ifirst && bI <= bJ;
            };
            // each passing pair's destination: dst[y] + its rank among the column's passing rows
            int nc[4];
            LdPair *dst[4] = {nullptr, nullptr, nullptr, nullptr};
            uint64_t fmv[4];
            uint32_t por = 0;
#pragma unroll
            for (int y = 0; y < 4; y++) por |= pass[y][0] | pass[y][1];
            const bool wpass = __builtin_amdgcn_ballot_w64(por != 0u) != 0;  // (wave-uniform)
#pragma unroll
            for (int y = 0; y < 4; y++) {
                uint64_t slot;
                const bool in = jokv[y] && slot_of(y, slot);
                fmv[y] = wpass ? full_of(y) : 0ull;
                nc[y] = in ? __popcll(fmv[y]) : 0;
                if (P == 1 && h == 0 && in) cnt[(uint64_t)(jv[y] - (int64_t)a.j_lo) * a.nb + slot] = (uint16_t)nc[y];
                if (P == 2 && nc[y]) dst[y] = pairs + off.at((uint64_t)(jv[y] - (int64_t)a.j_lo), a.nb, slot);
            }
            if (P == 1 && st.temp) {
                // quarters (64 columns: y = 2hy, 2hy + 1) holding pairs, staged as k_ld_fast's count
                // pass stages them: lane l <-> column l of the quarter (its own mask, y = 2hy + h)
#pragma unroll
                for (int hy = 0; hy < 2; hy++) {
                    const int qt = wave_sum(h == 0 ? nc[2 * hy] + nc[2 * hy + 1] : 0);
                    if (!qt) continue;  // wave-uniform
                    const uint32_t c = (uint32_t)(h ? nc[2 * hy + 1] : nc[2 * hy]);
                    const uint32_t incl = wave_incl_scan(c);
                    const uint32_t total = wave_bcast(incl, kWave - 1);
                    unsigned long long base = 0;
                    if (l == 0) base = atomicAdd(st.ctr, (unsigned long long)total);
                    base = __shfl(base, 0);
                    if (base + total > st.cap) {
                        if (l == 0) atomicOr(st.overflow, 1u);
                        continue;
                    }
#pragma unroll
                    for (int yy = 0; yy < 2; yy++) {
                        const int y = 2 * hy + yy;
                        const uint32_t run = (uint32_t)__shfl((int)(incl - c), 32 * yy + r);  // column 32yy + r
                        if (nc[y]) dst[y] = st.temp + base + run;
                    }
                    if (l == 0) {
                        const unsigned long long q = atomicAdd(st.ctr + 1, 1ull);
                        const uint32_t bJ = (uint32_t)(4ull * J4 + 2 * hp + hy);
                        if (q < st.qcap) st.quarters[q] = LdQuarter{(uint32_t)bI, bJ, (uint64_t)base};
                        else atomicOr(st.overflow, 1u);
                    }
                }
            }
            if (P == 2 || st.temp) {
                // the passing pairs with a destination, their r^2 recomputed lane-parallel and written
                uint32_t emitW[4];
                uint32_t ncand = 0;
#pragma unroll
                for (int y = 0; y < 4; y++) {
                    emitW[y] = dst[y] ? passW[y] : 0u;
                    ncand += (uint32_t)__builtin_popcount(candW[y]);
                }
                auto dest = [&](int y, int row) {
                    LdPair *const d0 = (y & 1) ? dst[1] : dst[0], *const d1 = (y & 1) ? dst[3] : dst[2];
                    const uint64_t f0 = (y & 1) ? fmv[1] : fmv[0], f1 = (y & 1) ? fmv[3] : fmv[2];
                    return ((y & 2) ? d1 : d0) + __popcll(((y & 2) ? f1 : f0) & ((1ull << row) - 1ull));
                };
                uint64_t *dl = reinterpret_cast<uint64_t *>(lst) + kSpList;  // (the list's second half)
                if (kSpR2Cache && wave_sum(ncand) <= (uint32_t)kSpR2Cap) {  // (wave-uniform)
                    // every candidate's r^2 is cached: replay the decision pass's list sequence (the
                    // same rounds from the same masks give every pair its position again); a pair
                    // that passed and has a destination is written from its owning lane
                    int y = 0;
                    uint32_t rm = candW[0];
                    adv_of(candW, y, rm);
                    for (int base = 0;;) {
                        const int n = rounds_of(candW, y, rm, [&](int yy, int b, int e) {
                            if (!((word_of(emitW, yy) >> b) & 1u)) return;
                            const int row = row_of(b >> 4, b & 15);
                            LdPair pr;
                            pr.i = (uint32_t)(ibase + wi * 64 + row);
                            pr.j = (uint32_t)(jb + 32 * yy + r);
                            pr.r2 = r2c[base + e];
                            *dest(yy, row) = pr;
                        });
                        if (n == 0) break;  // (wave-uniform)
                        base += n;
                    }
                } else
                spread(
                    emitW,
                    [&](int y, int b, int e) {
                        const int x = b >> 4, k = b & 15;
                        const int row = row_of(x, k);
                        LdPair *const d = dest(y, row);
                        lst[e] = make_uint2((uint32_t)(wi * 64 + row) | (uint32_t)(32 * y + r) << 8 |
                                                sxy_of(x, y, k) << 16,
                                            0u);
                        dl[e] = (uint64_t)(uintptr_t)d;
                    },
                    [&](int e, int) {
                        const uint32_t d0 = lst[e].x;
                        double r2 = 0.0;
                        (void)exact(d0, r2);
                        LdPair pr;
                        pr.i = (uint32_t)(ibase + (d0 & 0xFF));
                        pr.j = (uint32_t)(jb + ((d0 >> 8) & 0x7F));
                        pr.r2 = r2;
                        *reinterpret_cast<LdPair *>((uintptr_t)dl[e]) = pr;
                    },
                    [&](int, int, int) {});
            }
        }
        __syncthreads();  // R and C are zeroed again for the next half
    }
}

template <int P, bool kSp>
__global__ __launch_bounds__(kWaves * kWave) void k_ld_fast(const uint8_t *__restrict__ Gp,
                                                            const LdFast *__restrict__ fv,
                                                            const uint32_t *__restrict__ chrom_id, LdWindowArgs a,
                                                            const uint32_t *__restrict__ blocks, uint32_t nblocks,
                                                            uint16_t *__restrict__ cnt,
                                                            LdOffsets off,
                                                            LdPair *__restrict__ pairs, LdStage st, LdSparse sp) {
    // ONE LDS array (a second __shared__ object makes hipcc drain vmcnt before the k-loop's
    // ds_reads): the staging ring during the k-loop, then the waves' epilogue tiles over it;
    // the per-row prefilter terms after that
    // ... and the tile's raw per-variant records (rows I, columns J), DMA'd in with the first
    // stages so no global-load latency sits before the k-loop or the epilogue
    __shared__ __attribute__((aligned(16))) int8_t lds[kRing + kFB * (8 + 4 + 4 + 4 + 4 + 4 + 4) + 2 * kFvBytes];
    double *rvx = reinterpret_cast<double *>(lds + kRing);
    int *rsx = reinterpret_cast<int *>(lds + kRing + kFB * 8);
    float *rvxf = reinterpret_cast<float *>(lds + kRing + kFB * 12);
    float *ru = reinterpret_cast<float *>(lds + kRing + kFB * 16);  // register epilogue: sqrt(tm' Vx) / n
    float *rsf = reinterpret_cast<float *>(lds + kRing + kFB * 20);  // and Sx as fp32
    float *cw = reinterpret_cast<float *>(lds + kRing + kFB * 24);   // columns: -Sy / n
    float *cv = reinterpret_cast<float *>(lds + kRing + kFB * 28);   // and sqrt(Vy)
    const LdFast *fI = reinterpret_cast<const LdFast *>(lds + kRing + kFB * 32);
    const LdFast *fJ = reinterpret_cast<const LdFast *>(lds + kRing + kFB * 32 + kFvBytes);
    const uint32_t b = xcd_remap(blockIdx.x, nblocks);
    const uint32_t I4 = blocks[2 * b], J4 = blocks[2 * b + 1];
    const int t = threadIdx.x, w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int wi = w >> 1, wj = w & 1;  // output rows wi*64.., columns wj*128..
    const int64_t M = (int64_t)a.m;
    const int64_t ibase = (int64_t)I4 * kFB, jbase = (int64_t)J4 * kFB;
    // count-table slot of 64-block pair (bI, bJ); false outside the window triangle
    auto sub = [&](uint64_t bI, uint64_t bJ, uint64_t &slot) {
        const uint64_t jrow0 = bJ * kLdBlock;
        const uint64_t ifirst = jrow0 > a.window ? (jrow0 - a.window) / kLdBlock : 0;
        slot = bI - ifirst;
        return bI >= ifirst && bI <= bJ;
    };
    if (P == 2) {  // emit pass: skip blocks without a counted pair (16 quarters x 64 columns)
        uint32_t any = 0;
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const int idx = t + e * kWaves * kWave;  // 0..1023
            const int qi = idx >> 8, qj = (idx >> 6) & 3, col = idx & 63;
            const uint64_t bI = 4ull * I4 + qi, bJ = 4ull * J4 + qj;
            uint64_t slot;
            const int64_t jj = (int64_t)(bJ * kLdBlock) + col;
            if (sub(bI, bJ, slot) && jj < M && jj >= (int64_t)a.j_lo && jj < (int64_t)a.j_hi)
                any |= cnt[(uint64_t)(jj - (int64_t)a.j_lo) * a.nb + slot];
        }
        if (!__syncthreads_or(any != 0)) return;
    }
    if (!kSp) {  // the I and J records: kFvBytes each, 1 KiB per wave-instruction.  A lane whose 16 B
        // start past the array re-reads its last 16 B (rows / columns outside the matrix, never
        // used); a lane straddling the end reads < 16 B past it, inside the M + 1 records the
        // array is allocated with (vcfxg_ld_prepare)
        const char *fv_end = reinterpret_cast<const char *>(fv + M);
        for (int q = w; q < 2 * kFvGlds; q += kWaves) {
            const int side = q / kFvGlds, part = q - side * kFvGlds;
            const char *s = reinterpret_cast<const char *>(fv + (side ? jbase : ibase)) + part * 1024 + l * 16;
            glds16(s < fv_end ? s : fv_end - 16, lds + kRing + kFB * 32 + side * kFvBytes + part * 1024);
        }
    }
    if (kSp) {  // the I and J sparse records: 8 KiB, one 1 KiB piece per wave (clamped to the zero
        // record at M: rows / columns outside the matrix)
        const int side = w >> 2, part = w & 3;
        const int64_t v = (side ? jbase : ibase) + part * 64 + l;
        glds16(reinterpret_cast<const char *>(sp.rec + (v < M ? v : M)), lds + kSpInts + w * 1024);
    }
    const int kpad = a.kp4;  // FP4 row bytes
    // staging: 32 wave-instructions of 1 KiB per stage, kGlds per wave; instruction q of
    // wave w fills LDS [(kGlds*w+q) KiB, +1 KiB) = 16 rows x 64 B; lane l -> row (l>>2),
    // physical slot l&3 holding logical 16 B slot (l&3) ^ ((row>>2)&3)
    const uint8_t *src[kGlds];
#pragma unroll
    for (int q = 0; q < kGlds; q++) {
        const int idx = kGlds * w + q;                // 0..31: A rows for 0..15, B rows after
        const int lrow = (idx & 15) * 16 + (l >> 2);  // row within the A or B tile
        int64_t g = (VCFXG_LD_EXPT & 16) ? lrow : (idx < 16 ? ibase : jbase) + lrow;
        if (g >= M) g = M - 1;
        const int logical = (l & 3) ^ ((lrow >> 2) & 3);
        src[q] = Gp + g * (int64_t)kpad + logical * 16;
    }
    auto stage = [&](int ks, int buf) {
#pragma unroll
        for (int q = 0; q < kGlds; q++) glds16(src[q] + ((VCFXG_LD_EXPT & 8) ? 0 : ks * kBK), lds + buf * kStage + (kGlds * w + q) * 1024);
    };
    v16f acc[2][4];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) acc[x][y] = v16f{};
    const int nk = kpad / kBK;
    // fragments of k-half s (32 k-bytes) of the k-slice in buffer `base`
    auto frag = [&](const int8_t *base, int s, v4i(&fa)[2], v4i(&fb)[4]) {
        const int lg = 2 * s + h;
#pragma unroll
        for (int x = 0; x < 2; x++) {
            const int ra = wi * 64 + x * 32 + r;
            fa[x] = *reinterpret_cast<const v4i *>(base + ra * kBK + ((lg ^ ((ra >> 2) & 3)) << 4));
        }
#pragma unroll
        for (int y = 0; y < 4; y++) {
            const int rb = wj * 128 + y * 32 + r;
            fb[y] = *reinterpret_cast<const v4i *>(base + kFB * kBK + rb * kBK + ((lg ^ ((rb >> 2) & 3)) << 4));
        }
    };
    auto mfma8 = [&](const v4i(&fa)[2], const v4i(&fb)[4]) {
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
                acc[x][y] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                    v8i{fa[x].x, fa[x].y, fa[x].z, fa[x].w, 0, 0, 0, 0},
                    v8i{fb[y].x, fb[y].y, fb[y].z, fb[y].w, 0, 0, 0, 0}, acc[x][y], kFmtFp4, kFmtFp4, 0, kScaleOne,
                    0, kScaleOne);
    };
    // Software pipeline over a kNBuf-buffer ring, fragments one k-half ahead of the MFMAs:
    //   step ks: read F(ks, 1) | MFMAs (ks, 0) | wait stage ks+1, barrier, stage ks+3 into
    //   buffer (ks-1)%kNBuf (last read by F(ks-1, 1), consumed before this barrier), read
    //   F(ks+1, 0) | MFMAs (ks, 1)
    // so every fragment read overlaps 8 MFMAs and the barrier sits between two MFMA groups;
    // counted vmcnt + raw s_barrier (a __syncthreads fence would drain every glds)
    // the epilogue's pointer arguments, consumed here: left to itself the compiler hoists their
    // scalar loads over the loop, and a pending SMEM load (out of order within lgkmcnt) turns
    // every fragment wait in the loop into lgkmcnt(0)
    asm volatile("" ::"s"(cnt), "s"(chrom_id), "s"(pairs));
    for (int q = 0; q < kNBuf - 1; q++) stage(q < nk ? q : nk - 1, q);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    v4i a0[2], b0[4], a1[2], b1[4];
    frag(lds, 0, a0, b0);
    for (int ks = 0; ks < nk - 1; ks++) {  // (the last step peeled: no branch before MFMAs (ks, 1)
        frag(lds + (ks % kNBuf) * kStage, 1, a1, b1);  // lets the compiler count lgkmcnt exactly)
        mfma8(a0, b0);
        // one MFMA first: the compiler's wait before it (always lgkmcnt(0) here) then covers
        // only F(ks, 0), and F(ks, 1) loads behind the other 7
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 7, 0);
        // stage ks+1 landed (stage ks+2 may still load); every step issues a stage -- past
        // the end a re-read of the last (L2-hot) slice into the free buffer -- so the counts
        // are constant and the loop body has no branch
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        frag(lds + ((ks + 1) % kNBuf) * kStage, 0, a0, b0);
        stage(ks + kNBuf - 1 < nk ? ks + kNBuf - 1 : nk - 1, (ks + kNBuf - 1) % kNBuf);
        mfma8(a1, b1);
        // again one MFMA first (the compiler's wait before it, lgkmcnt(0), then covers only
        // the long-landed F(ks, 1)), the fragment reads, the staging loads between MFMAs
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
        for (int q = 0; q < kGlds; q++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 7 - kGlds, 0);
    }
    frag(lds + ((nk - 1) % kNBuf) * kStage, 1, a1, b1);
    mfma8(a0, b0);
    mfma8(a1, b1);
    if (VCFXG_LD_EXPT & 1) {
        int z = 0;
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int k = 0; k < 16; k++) z ^= (int)acc[x][y][k];
        if (z == 0x7fffffff) cnt[0] = 1;
        return;
    }
    if constexpr (kSp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // every wave is done with the ring
        ld_sparse_epilogue<P>(acc, lds, a, sp, chrom_id, I4, J4, cnt, off, pairs, st);
        return;
    }
    // the row and column terms from the DMA'd records (every wave's loads done, then visible)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t < kFB) {
        const LdFast f = fI[t];
        rvx[t] = f.vxp;
        rvxf[t] = (float)f.vxp;
        ru[t] = a.all_pass ? 0.f : sqrtf((float)(a.tm * (1.0 - 1e-5)) * (float)f.vxp) / (float)a.ns;
        rsf[t] = (float)f.sx;
        rsx[t] = f.sx;
    } else {
        const LdFast f = fJ[t - kFB];
        cw[t - kFB] = a.ns > 0 ? -(float)f.sx / (float)a.ns : 0.f;  // (n = 0: every r^2 is 0, no NaN)
        cv[t - kFB] = a.all_pass ? 0.f : sqrtf((float)f.vxp);
    }
    const int pad = 0;  // FP4 rows are zero-padded
    const double dn = (double)a.ns;
    const int64_t n = a.ns;
    // fp32 form of the prefilter while n*Sxy and Sx*Sy fit int32 (n <= 23170): C exact in
    // int32, C^2 and tm*Vx*Vy within ~1e-6 relative in fp32, so a further 1e-5 relative
    // slack keeps every pair that can reach the threshold
    const bool f32 = a.ns <= 23170;
    const uint64_t bI = 4ull * I4 + wi;
    const int64_t i0 = (int64_t)bI * kLdBlock;
    int *tile = reinterpret_cast<int *>(lds + w * kQuarter);
    // quarter hy (columns hy*64.. of the wave) through this wave's LDS tile: lane l walks
    // column j's rows and returns the mask of the rows whose pair passes (exact decision)
    auto walk = [&](int hy, int64_t j, bool jok, LdFast &fj) -> uint64_t {
        // the quarter's accumulators -> this wave's LDS tile [row][col] (no other wave uses
        // it, and the wave's own lanes are in lockstep: no barrier between quarters)
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int yy = 0; yy < 2; yy++)
#pragma unroll
                for (int k = 0; k < 16; k++)
                    tile[(32 * x + (k & 3) + 8 * (k >> 2) + 4 * h) * 64 + 32 * yy + r] = (int)acc[x][2 * hy + yy][k];
        uint64_t mask = 0;
        if (jok) {
            fj = fv[j];
            const uint32_t cj = a.max_dist > 0 ? chrom_id[j] : 0u;
            const double rhs_j = a.all_pass ? 0.0 : a.tm * fj.vxp;
            const float rhs_jf = (float)(a.tm * (1.0 - 1e-5)) * (float)fj.vxp;
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
        return mask;
    };
    auto write_pairs = [&](uint64_t mask, int64_t j, const LdFast &fj, LdPair *dst) {
        uint32_t rank = 0;
        while (mask) {
            const int row = __builtin_ctzll(mask);
            mask &= mask - 1;
            LdPair pr;
            pr.i = (uint32_t)(i0 + row);
            pr.j = (uint32_t)j;
            pr.r2 = ld_fast_r2(fv[i0 + row], fj, tile[row * 64 + l] - pad, dn);
            dst[rank++] = pr;
        }
    };
    if (P == 1 && a.ns <= 23170) {
        __syncthreads();  // the row and column terms are visible to every wave
        int qt[2];
        ld_count_regs(acc, a, fv, chrom_id, cnt, ru, rsf, cw, cv, I4, J4, wi, wj, h, r, qt);
        if (!st.temp) return;
        // quarters holding pairs: written now, column-major into a bump-allocated staging
        // area (ld_scatter later moves each column's run to its ordered offset), so the
        // emit pass needs no second MFMA sweep
#pragma unroll
        for (int hy = 0; hy < 2; hy++) {
            if (!qt[hy]) continue;  // wave-uniform
            const uint64_t bJ = 4ull * J4 + 2 * wj + hy;
            const int64_t j = (int64_t)(bJ * kLdBlock) + l;
            const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
            LdFast fj{};
            const uint64_t mask = walk(hy, j, jok, fj);
            const uint32_t c = (uint32_t)__popcll(mask);
            const uint32_t incl = wave_incl_scan(c);
            const uint32_t total = wave_bcast(incl, kWave - 1);
            unsigned long long base = 0;
            if (l == 0) base = atomicAdd(st.ctr, (unsigned long long)total);
            base = __shfl(base, 0);
            if (base + total > st.cap) {
                if (l == 0) atomicOr(st.overflow, 1u);
                continue;
            }
            write_pairs(mask, j, fj, st.temp + base + (incl - c));
            if (l == 0) {
                const unsigned long long q = atomicAdd(st.ctr + 1, 1ull);
                if (q < st.qcap) st.quarters[q] = LdQuarter{(uint32_t)bI, (uint32_t)bJ, (uint64_t)base};
                else atomicOr(st.overflow, 1u);
            }
        }
        return;
    }
    __syncthreads();  // every wave is done reading the ring; the epilogue tiles reuse it
#pragma unroll
    for (int hy = 0; hy < 2; hy++) {  // the wave's two 64x64 quarters (columns hy*64..)
        const uint64_t bJ = 4ull * J4 + 2 * wj + hy;
        uint64_t slot;
        if (!sub(bI, bJ, slot)) continue;  // wave-uniform: a quarter outside the window triangle
        const int64_t j = (int64_t)(bJ * kLdBlock) + l;
        const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
        LdFast fj{};
        const uint64_t mask = walk(hy, j, jok, fj);
        if (P == 1) {
            if (jok) cnt[(uint64_t)(j - (int64_t)a.j_lo) * a.nb + slot] = (uint16_t)__popcll(mask);
            continue;
        }
        if (!mask) continue;
        write_pairs(mask, j, fj, pairs + off.at((uint64_t)(j - (int64_t)a.j_lo), a.nb, slot));
    }
}

// staged pairs -> their ordered offsets: one wave per staged quarter, lane = column j; the
// column's run starts after the runs of the quarter's earlier columns (the same wave scan
// that laid them out) and goes to off[j][slot]
__global__ __launch_bounds__(256) void k_ld_scatter(const LdQuarter *__restrict__ quarters,
                                                    const unsigned long long *__restrict__ ctr, LdWindowArgs a,
                                                    const uint16_t *__restrict__ cnt, LdOffsets off,
                                                    const LdPair *__restrict__ temp, LdPair *__restrict__ pairs) {
    const uint64_t nq = ctr[1];
    const int l = threadIdx.x & 63;
    const int64_t M = (int64_t)a.m;
    for (uint64_t q = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64; q < nq;
         q += (uint64_t)gridDim.x * blockDim.x / 64) {
        const LdQuarter Q = quarters[q];
        const uint64_t jrow0 = (uint64_t)Q.bJ * kLdBlock;
        const uint64_t ifirst = jrow0 > a.window ? (jrow0 - a.window) / kLdBlock : 0;
        const int64_t j = (int64_t)jrow0 + l;
        const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
        const uint64_t jrel = jok ? (uint64_t)(j - (int64_t)a.j_lo) : 0, slot = Q.bI - ifirst;
        const uint32_t c = jok ? cnt[jrel * a.nb + slot] : 0u;
        const uint32_t incl = wave_incl_scan(c);
        const LdPair *src = temp + Q.base + (incl - c);
        LdPair *dst = pairs + (jok ? off.at(jrel, a.nb, slot) : 0);
        for (uint32_t k = 0; k < c; k++) dst[k] = src[k];
    }
}

hipError_t launch_ld_scatter(const LdQuarter *quarters, const unsigned long long *ctr, uint64_t nq_host,
                             const LdWindowArgs &a, const uint16_t *cnt, LdOffsets off, const LdPair *temp,
                             LdPair *pairs, hipStream_t s) {
    if (!nq_host) return hipSuccess;
    const uint64_t blocks = (nq_host + 3) / 4;
    hipLaunchKernelGGL(k_ld_scatter, dim3((unsigned)std::min<uint64_t>(blocks, 65536)), dim3(256), 0, s, quarters, ctr,
                       a, cnt, off, temp, pairs);
    return hipGetLastError();
}

hipError_t launch_ld_fast(int pass, const uint8_t *Gp, const LdFast *fv, const uint32_t *chrom_id,
                          const LdWindowArgs &a, const uint32_t *blocks, uint32_t nblocks, uint16_t *cnt,
                          LdOffsets off, LdPair *pairs, const LdStage &st, hipStream_t s) {
    if (!nblocks) return hipSuccess;
    if (a.kp4 % kBK || a.kp4 <= 0) return hipErrorInvalidValue;
    if (pass == 1)
        hipLaunchKernelGGL((k_ld_fast<1, false>), dim3(nblocks), dim3(kWaves * kWave), 0, s, Gp, fv, chrom_id, a, blocks,
                           nblocks, cnt, off, pairs, st, LdSparse{});
    else
        hipLaunchKernelGGL((k_ld_fast<2, false>), dim3(nblocks), dim3(kWaves * kWave), 0, s, Gp, fv, chrom_id, a, blocks,
                           nblocks, cnt, off, pairs, st, LdSparse{});
    return hipGetLastError();
}

hipError_t launch_ld_sparse(int pass, const uint8_t *Gp, const LdSparse &sp, const uint32_t *chrom_id,
                            const LdWindowArgs &a, const uint32_t *blocks, uint32_t nblocks, uint16_t *cnt,
                            LdOffsets off, LdPair *pairs, const LdStage &st, hipStream_t s) {
    if (!nblocks) return hipSuccess;
    if (a.kp4 % kBK || a.kp4 <= 0 || a.ns > 16383 || !sp.gt16 || !sp.vars || !sp.rec || sp.mp % kFB) return hipErrorInvalidValue;
    if (pass == 1)
        hipLaunchKernelGGL((k_ld_fast<1, true>), dim3(nblocks), dim3(kWaves * kWave), 0, s, Gp, nullptr, chrom_id, a,
                           blocks, nblocks, cnt, off, pairs, st, sp);
    else
        hipLaunchKernelGGL((k_ld_fast<2, true>), dim3(nblocks), dim3(kWaves * kWave), 0, s, Gp, nullptr, chrom_id, a,
                           blocks, nblocks, cnt, off, pairs, st, LdSparse(sp));
    return hipGetLastError();
}

// FP4 (e2m1) copy of the compacted genotype rows for the fast kernel: dosage 0/1/2 ->
// 0x0/0x2/0x4, two per byte (element 2b low nibble), zero from ns on; an incomplete row's
// missing code packs as 0 (such rows never reach k_ld_fast)
__global__ void k_ld_pack4(const int8_t *__restrict__ Gc, uint64_t m, int kpad, int ns, uint8_t *__restrict__ Gp,
                           int kp4, const LdVar *__restrict__ vars) {
    const int per = kp4 / 16;  // 16 output bytes per thread
    const uint64_t total = m * (uint64_t)per;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = t / per;
        const int c = (int)(t - v * per);
        const int8_t *row = Gc + (vars ? vars[v].line : v) * (uint64_t)kpad;
        uint32_t in[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // 32 codes, 4 per dword
        if (c * 32 + 32 <= kpad) {
            const uint4 u0 = reinterpret_cast<const uint4 *>(row)[2 * c];
            const uint4 u1 = reinterpret_cast<const uint4 *>(row)[2 * c + 1];
            in[0] = u0.x, in[1] = u0.y, in[2] = u0.z, in[3] = u0.w;
            in[4] = u1.x, in[5] = u1.y, in[6] = u1.z, in[7] = u1.w;
        }
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 32; e++) {
            const int g = (int8_t)(in[e >> 2] >> (8 * (e & 3)));
            const uint32_t code = c * 32 + e < ns ? (g == 1 ? 0x2u : g == 2 ? 0x4u : 0x0u) : 0x0u;
            w[e >> 3] |= code << (4 * (e & 7));
        }
        reinterpret_cast<uint4 *>(Gp + v * (uint64_t)kp4)[c] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

hipError_t launch_ld_pack4(const int8_t *Gc, uint64_t m, int kpad, int ns, uint8_t *Gp, int kp4, hipStream_t s,
                           const LdVar *vars) {
    if (!m) return hipSuccess;
    if (kp4 % 64 || 2 * (int64_t)kp4 < ns) return hipErrorInvalidValue;
    const uint64_t total = m * (uint64_t)(kp4 / 16);
    const unsigned grid = (unsigned)std::min<uint64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_ld_pack4, dim3(grid), dim3(256), 0, s, Gc, m, kpad, ns, Gp, kp4, vars);
    return hipGetLastError();
}

// self-test of the FP4 MFMA operand layout: C = A (32x64) . B^T over K = 64, dosages 0..2
__global__ void k_mfma_f4_selftest(const uint8_t *A, const uint8_t *B, float *C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    const v4i a = *reinterpret_cast<const v4i *>(A + r * 32 + 16 * h);
    const v4i b = *reinterpret_cast<const v4i *>(B + r * 32 + 16 * h);
    v16f c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v8i{a.x, a.y, a.z, a.w, 0, 0, 0, 0},
                                                        v8i{b.x, b.y, b.z, b.w, 0, 0, 0, 0}, c, kFmtFp4, kFmtFp4, 0,
                                                        kScaleOne, 0, kScaleOne);
    for (int k = 0; k < 16; k++) C[((k & 3) + 8 * (k >> 2) + 4 * h) * 32 + r] = c[k];
}

hipError_t launch_mfma_f4_selftest(const uint8_t *A, const uint8_t *B, float *C, hipStream_t s) {
    hipLaunchKernelGGL(k_mfma_f4_selftest, dim3(1), dim3(64), 0, s, A, B, C);
    return hipGetLastError();
}

// per-row scan of the pair-count table: one wave per output row j, the u16 counts of its
// window slots (column blocks ifirst(J) .. J, every one written by the count kernels; the
// table is not cleared; nb is a multiple of 8, so each lane reads 8 slots as one 16 B load)
// -> the row's total and the u32 offsets inside the row of the slots that HOLD pairs (the
// emit passes read no other slot's offset).  Almost every slot is empty: a 512-slot step
// whose counts are all zero costs its loads and one ballot, and writes nothing
__global__ __launch_bounds__(256) void k_ld_rowscan(const uint16_t *__restrict__ cnt, uint64_t rows, uint64_t nb,
                                                    uint64_t j_lo, uint64_t window, uint32_t *__restrict__ in_row,
                                                    uint64_t *__restrict__ rowtot) {
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
    const int l = threadIdx.x & 63;
    for (uint64_t j = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64; j < rows; j += nw) {
        const uint64_t J = (j_lo + j) / kLdBlock, jr0 = J * kLdBlock;
        const uint64_t I0 = jr0 > window ? (jr0 - window) / kLdBlock : 0;
        const uint32_t ns = (uint32_t)(J - I0 + 1 < nb ? J - I0 + 1 : nb);
        const uint16_t *c = cnt + j * nb;
        uint32_t *o = in_row + j * nb;
        uint32_t run = 0;
        for (uint32_t s0 = 0; s0 < ns; s0 += 512) {
            const uint32_t sl = s0 + 8u * (uint32_t)l;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (sl < ns) v = *reinterpret_cast<const uint4 *>(c + sl);
            // slots past the row's window (the table's padding, never written) read as 0
            const uint32_t past = sl + 8u > ns ? (sl < ns ? sl + 8u - ns : 8u) : 0u;
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int lo_e = 2 * q, hi_e = 2 * q + 1;  // elements of dword q
                if (8 - (int)past <= lo_e) w[q] = 0u;
                else if (8 - (int)past <= hi_e) w[q] &= 0xFFFFu;
            }
            const uint32_t t = (w[0] & 0xFFFFu) + (w[0] >> 16) + (w[1] & 0xFFFFu) + (w[1] >> 16) + (w[2] & 0xFFFFu) +
                               (w[2] >> 16) + (w[3] & 0xFFFFu) + (w[3] >> 16);
            if (!__ballot(t != 0u)) continue;
            const uint32_t incl = wave_incl_scan32(t);
            uint32_t acc = run + incl - t;
            if (t) {
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    const uint32_t x = (w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
                    if (x) o[sl + e] = acc;
                    acc += x;
                }
            }
            run += __builtin_amdgcn_readlane(incl, 63);
        }
        if (l == 0) rowtot[j] = run;
    }
}

hipError_t launch_ld_rowscan(const uint16_t *cnt, uint64_t rows, uint64_t nb, uint64_t j_lo, uint64_t window,
                             uint32_t *in_row, uint64_t *rowtot, hipStream_t s) {
    if (!rows) return hipSuccess;
    const uint64_t blocks = (rows + 3) / 4;
    hipLaunchKernelGGL(k_ld_rowscan, dim3((unsigned)std::min<uint64_t>(blocks, 65536)), dim3(256), 0, s, cnt, rows, nb,
                       j_lo, window, in_row, rowtot);
    return hipGetLastError();
}

// per kLdFastBlock-variant group: 1 if every variant of the group is complete; 2 (sparse) if
// every variant misses at most kLdSparseMax calls; else 0
__global__ void k_ld_groups(const LdVar *__restrict__ vars, uint64_t m, int ns, int sparse, uint8_t *__restrict__ gflag,
                            const uint64_t *m_dev) {
    if (m_dev) m = *m_dev;
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x / 64 + threadIdx.x / 64;
    const uint64_t ng = (m + kFB - 1) / kFB;
    if (g >= ng) return;
    const int l = threadIdx.x & 63;
    bool ok = true, sp = true;
    for (int k = l; k < kFB; k += 64) {
        const uint64_t v = g * kFB + k;
        if (v < m) {
            ok = ok && vars[v].complete;
            sp = sp && ns - vars[v].cnt <= kLdSparseMax;
        }
    }
    ok = __all(ok);
    sp = __all(sp);
    if (l == 0) gflag[g] = ok ? 1 : (sparse && sp) ? 2 : 0;
}

hipError_t launch_ld_groups(const LdVar *vars, uint64_t m, int ns, int sparse, uint8_t *gflag, hipStream_t s,
                            const uint64_t *m_dev) {
    const uint64_t ng = (m + kFB - 1) / kFB;
    if (!ng) return hipSuccess;
    hipLaunchKernelGGL(k_ld_groups, dim3((unsigned)((ng + 3) / 4)), dim3(256), 0, s, vars, m, ns, sparse, gflag, m_dev);
    return hipGetLastError();
}

// per variant (one wave each): its missing samples (codes < 0 among the first ns) in sample
// order into midx / mvar from moff[v] (16 codes per lane per step, ballot-free: a wave scan of
// the per-lane counts)
__global__ __launch_bounds__(256) void k_ld_miss_fill(const int8_t *__restrict__ Gc, uint64_t m, int kpad, int ns,
                                                      const uint64_t *__restrict__ moff, uint16_t *__restrict__ midx,
                                                      uint32_t *__restrict__ mvar, uint16_t *__restrict__ midx16) {
    const int l = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t v = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64; v < m; v += nw) {
        const int8_t *row = Gc + v * (uint64_t)kpad;
        const uint64_t at0 = moff[v];
        uint64_t at = at0;
        for (int s0 = 0; s0 < ns; s0 += 16 * 64) {
            const int b = s0 + 16 * l;
            uint32_t bits = 0;
            if (b < kpad) {
                const uint4 q = *reinterpret_cast<const uint4 *>(row + b);
                const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if ((int8_t)(w[k >> 2] >> (8 * (k & 3))) < 0 && b + k < ns) bits |= 1u << k;
            }
            const uint32_t c = (uint32_t)__popc(bits);
            const uint32_t incl = wave_incl_scan(c);
            uint64_t o = at + incl - c;
            while (bits) {
                const int k = __builtin_ctz(bits);
                bits &= bits - 1u;
                midx[o] = (uint16_t)(b + k);
                mvar[o] = (uint32_t)v;
                if (o - at0 < 16) midx16[v * 16 + (o - at0)] = (uint16_t)(b + k);  // (the first 16)
                o++;
            }
            at += wave_bcast(incl, 63);
        }
    }
}

hipError_t launch_ld_miss_fill(const int8_t *Gc, uint64_t m, int kpad, int ns, const uint64_t *moff, uint16_t *midx,
                               uint32_t *mvar, uint16_t *midx16, hipStream_t s) {
    if (!m) return hipSuccess;
    if (kpad % 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ld_miss_fill, dim3((unsigned)std::min<uint64_t>((m + 3) / 4, 16384)), dim3(256), 0, s, Gc, m,
                       kpad, ns, moff, midx, mvar, midx16);
    return hipGetLastError();
}

// the sample-major contribution plane: 64 variants x 64 samples per block through LDS (rows of
// Gc in, rows of gt16 out, both coalesced); variants past m and samples past ns are zero
__global__ __launch_bounds__(256) void k_ld_gt16(const int8_t *__restrict__ Gc, uint64_t m, int kpad, int ns,
                                                 uint64_t mp, uint16_t *__restrict__ gt16) {
    __shared__ int8_t tile[64][68];
    const uint64_t v0 = (uint64_t)blockIdx.x * 64;
    const int s0 = blockIdx.y * 64;
    const int t = threadIdx.x;
    // load: 64 rows x 64 codes, 16 B per thread
    {
        const int rr = t >> 2, cc = (t & 3) * 16;
        const uint64_t v = v0 + rr;
        uint4 q = make_uint4(0, 0, 0, 0);
        if (v < m && s0 + cc < kpad) q = *reinterpret_cast<const uint4 *>(Gc + v * (uint64_t)kpad + s0 + cc);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 16; k++) tile[rr][cc + k] = (int8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
    __syncthreads();
    // store: 64 sample rows x 64 variants as u16, 16 per thread (two 16 B stores)
    const int ss = t >> 2, vv = (t & 3) * 16;
    if (s0 + ss >= ns) return;
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        uint32_t pr = 0;
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const uint64_t v = v0 + vv + k + e;
            const int g = v < m ? (int)tile[vv + k + e][ss] : 0;
            const uint32_t c = g < 0 ? 2048u : g == 1 ? 33u : g == 2 ? 130u : 0u;
            pr |= c << (16 * e);
        }
        o[k >> 1] = pr;
    }
    uint4 *dst = reinterpret_cast<uint4 *>(gt16 + (uint64_t)(s0 + ss) * mp + v0 + vv);
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// the sparse kernel's per-variant records (entry m: zeros, the rows / columns past the matrix)
__global__ __launch_bounds__(256) void k_ld_sprec(const LdVar *__restrict__ vars, uint64_t m, int ns,
                                                  LdSpRec *__restrict__ rec) {
    for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v <= m; v += (uint64_t)gridDim.x * 256) {
        LdSpRec r{0, 0.0};
        if (v < m) {
            const LdVar x = vars[v];
            r.pk = sp_pack(ns - x.cnt, x.sx, x.sx2);
            r.varx = x.varx;
        }
        rec[v] = r;
    }
}

hipError_t launch_ld_sprec(const LdVar *vars, uint64_t m, int ns, LdSpRec *rec, hipStream_t s) {
    hipLaunchKernelGGL(k_ld_sprec, dim3((unsigned)std::min<uint64_t>(m / 256 + 1, 4096)), dim3(256), 0, s, vars, m, ns,
                       rec);
    return hipGetLastError();
}

hipError_t launch_ld_gt16(const int8_t *Gc, uint64_t m, int kpad, int ns, uint64_t mp, uint16_t *gt16, hipStream_t s) {
    if (!m || ns <= 0) return hipSuccess;
    if (mp % 256 || mp < m || kpad % 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ld_gt16, dim3((unsigned)(mp / 64), (unsigned)((ns + 63) / 64)), dim3(256), 0, s, Gc, m, kpad,
                       ns, mp, gt16);
    return hipGetLastError();
}

}  // namespace vcfxg
