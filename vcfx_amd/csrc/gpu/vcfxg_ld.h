// vcfxg_ld.h -- device layouts and launchers of the LD kernels (vcfxg_ld.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vcfxg {

constexpr int kLdBlock = 64;       // count-table granularity (64-variant blocks)
constexpr int kLdFastBlock = 256;  // complete-group tile of the X.X^T kernel (vcfxg_ld_fast.hip)
constexpr int kLdMaskTile = 128;   // tile of the missing-data kernel (vcfxg_ld_mask.hip)

struct LdParseArgs {
    int ns;            // numSamples from the #CHROM line (tabs - 8 when >= 9 tabs)
    int kpad;          // row stride of the genotype matrix (ns rounded up to 64)
    int has_region;
    int rstart, rend;
    int64_t rlen;
    const char *rchrom;  // device copy of the region chromosome
    int stoi_mode;       // stdin matrix mode: std::stoi POS, parseGenotype on the whole field
};

struct LdLine {  // per indexed line
    uint32_t valid;
    int pos;
    uint32_t cnt, sx, sx2;  // valid samples, sum x, sum x^2
    uint32_t chrom_len, id_len;
    uint64_t chrom, id;     // byte offsets in the input
};

struct LdVar {  // per variant (compact order)
    int pos;
    int cnt, sx, sx2;
    double varx;            // own variance (computeStats) for computeRsqFast's gate
    int complete;           // no missing genotype among the ns samples
    uint32_t chrom_len, id_len;
    uint64_t chrom, id, line;
};

// complete-variant terms of computeRsqSIMD (:352-393) with n = ns, computed once per variant
// with the reference's own operation order, plus the integer variance for the prefilter
struct LdFast {
    double mx;   // Sx / n
    double vx;   // Sx2 / n - mx*mx  (== computeStats varX for a complete variant)
    double sq;   // sqrt(vx)
    double vxp;  // n*Sx2 - Sx^2 as double (> 0), +inf for a monomorphic variant
    int sx, pos;
};

// r^2 of two complete variants from S_xy: the reference's fp64 sequence, bit-identical
__device__ __forceinline__ double ld_fast_r2(const LdFast &fi, const LdFast &fj, int sxy, double dn) {
    if (!(fi.vx > 0.0) || !(fj.vx > 0.0) || dn < 2.0) return 0.0;  // computeRsqFast gate / n < 2
    const double cov = __dsub_rn(__ddiv_rn((double)sxy, dn), __dmul_rn(fi.mx, fj.mx));
    const double r = __ddiv_rn(cov, __dmul_rn(fi.sq, fj.sq));
    return __dmul_rn(r, r);
}

// The prefilter.  With n, Sx, Sy, Sxy, Sxx, Syy exact integers (fp32 accumulators, < 2^24):
//   C = n Sxy - Sx Sy,  Vx = n Sxx - Sx^2,  Vy = n Syy - Sy^2,  exact r^2 = C^2 / (Vx Vy).
// c = fma(n, Sxy, -fl(Sx Sy)) errs from C by at most ulp(Sx Sy)/2 + ulp(c)/2 <= pe, where pe
// (host: 2^-23 * 4 ns^2 + 1, twice the ulp of the largest magnitude 4 ns^2, plus one) bounds
// both; the same for vx, vy.  So |C| <= |c| + pe, Vx >= vx - pe, Vy >= vy - pe, and a pair is a
// candidate when (|c| + pe)^2 >= tm' max(vx - pe, 0) max(vy - pe, 0), tm' = tm (1 - 1e-5)
// absorbing the fp32 roundings of these three products (< 1e-6 relative).  Every pair whose
// exact r^2 reaches tm (threshold less the fp64 sequence's error margin, LdWindowArgs::tm) is a
// candidate; candidates run the reference's fp64 sequence.
__device__ __forceinline__ bool mask_candidate(float n, float sx, float sy, float sxy, float sxx, float syy, float pe,
                                               float tmf) {
    const float c = fabsf(__builtin_fmaf(n, sxy, -(sx * sy))) + pe;
    const float vx = fmaxf(__builtin_fmaf(n, sxx, -(sx * sx)) - pe, 0.f);
    const float vy = fmaxf(__builtin_fmaf(n, syy, -(sy * sy)) - pe, 0.f);
    return c * c >= tmf * (vx * vy);
}

// computeRsqFast (:397-401) on the pair's sums: the own-variance gate of both variants, then
// computeRsqSIMD's fp64 sequence (:383-392) with correctly rounded operations
__device__ __forceinline__ double mask_r2(double gi, double gj, int n, int sx, int sy, int sxy, int sxx, int syy) {
    if (gi <= 0.0 || gj <= 0.0) return 0.0;
    if (n < 2) return 0.0;
    const double dn = (double)n;
    const double mx = __ddiv_rn((double)sx, dn), my = __ddiv_rn((double)sy, dn);
    const double cov = __dsub_rn(__ddiv_rn((double)sxy, dn), __dmul_rn(mx, my));
    const double vx = __dsub_rn(__ddiv_rn((double)sxx, dn), __dmul_rn(mx, mx));
    const double vy = __dsub_rn(__ddiv_rn((double)syy, dn), __dmul_rn(my, my));
    if (vx <= 0.0 || vy <= 0.0) return 0.0;
    const double r = __ddiv_rn(cov, __dmul_rn(__dsqrt_rn(vx), __dsqrt_rn(vy)));
    return __dmul_rn(r, r);
}

struct LdPair {
    uint32_t i, j;          // variant indices, i < j
    double r2;
};

struct LdWindowArgs {
    uint64_t m;             // variants
    int kpad, ns;
    uint64_t window;        // pairs (i, j) with j - window <= i < j
    double threshold;
    int max_dist;           // > 0: same-chrom pairs farther apart are skipped (mmap streaming)
    uint64_t j_lo, j_hi;    // rows of this chunk
    uint64_t nb;            // column blocks per row in the count table
    double tm;              // prefilter: exact r^2 < tm cannot reach threshold (tm = threshold - delta)
    int all_pass;           // tm <= 0: every pair is a candidate
    int kp4;                // FP4 row bytes of the fast kernel's operand copy (multiple of 64)
};

hipError_t launch_ld_parse(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, const LdParseArgs &a, int8_t *G, LdLine *lines, hipStream_t s);
hipError_t launch_ld_compact(const LdLine *lines, const uint64_t *vidx, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int kpad, int ns, const int8_t *G, int8_t *Gc, LdVar *vars,
                             LdFast *fv, hipStream_t s);
// the LD walk (the parse without vcfxg_index; n_samples <= 4096): walker wk's lines to slots
// wk * cap_w + n (LdLine + int8 row of kpad bytes in G); wcount / wvalid per walker; overflow
// when a walker has more than cap_w lines; then the lines off the walk's fast path (pend_n
// zeroed by the caller; pend: capacity nw * cap_w) parsed on their own (k_ld_pending)
hipError_t launch_ld_walk(const char *buf, int64_t lo, int64_t hi, int64_t chunk, int64_t span0, uint64_t cap_w,
                          const LdParseArgs &a, int8_t *G, LdLine *lines, uint64_t *wcount, uint64_t *wvalid,
                          unsigned *overflow, unsigned long long *pend_n, uint64_t *pend, hipStream_t s);
// slots -> compact variants (vbase: exclusive scan of wvalid, nw + 1 entries): vars (line = the
// slot), fv, prefix lengths plen; flags bit 0 = some variant incomplete; *m_out = M
hipError_t launch_ld_wcompact(int64_t nw, uint64_t cap_w, const uint64_t *wcount, const uint64_t *vbase,
                              const LdLine *lines, int ns, const char *buf, int id_dot_to_pos, LdVar *vars, LdFast *fv,
                              uint64_t *plen, unsigned *flags, uint64_t *m_out, hipStream_t s);
// Gc[v] = the walk row of variant v (vars[v].line = its slot)
hipError_t launch_ld_gather(const LdVar *vars, uint64_t m, const int8_t *G, int kpad, int8_t *Gc, hipStream_t s);
// ordered output offset of pair slot (row j - j_lo, column block slot): the row's first
// pair (exclusive scan over rows) + the slot's offset inside the row (per-row scan, u32)
struct LdOffsets {
    const uint64_t *row = nullptr;
    const uint32_t *in_row = nullptr;
    __device__ __forceinline__ uint64_t at(uint64_t jrel, uint64_t nb, uint64_t slot) const {
        return row[jrel] + in_row[jrel * nb + slot];
    }
};
hipError_t launch_ld_rowscan(const uint16_t *cnt, uint64_t rows, uint64_t nb, uint64_t j_lo, uint64_t window,
                             uint32_t *in_row, uint64_t *rowtot, hipStream_t s);

// count pass of the fast kernel staging the pairs of every quarter that holds some
// (quarters[] records where each went); overflow -> the emit pass recomputes them
struct LdQuarter {
    uint32_t bI, bJ;  // 64-blocks: column block (rows i) and row block (variants j)
    uint64_t base;    // first staged pair
};
struct LdStage {
    LdPair *temp = nullptr;               // nullptr: count only
    uint64_t cap = 0;                     // staged-pair capacity
    LdQuarter *quarters = nullptr;
    uint64_t qcap = 0;
    unsigned long long *ctr = nullptr;    // [0] staged pairs, [1] quarters
    unsigned *overflow = nullptr;
};
hipError_t launch_ld_scatter(const LdQuarter *quarters, const unsigned long long *ctr, uint64_t nq_host,
                             const LdWindowArgs &a, const uint16_t *cnt, LdOffsets off, const LdPair *temp,
                             LdPair *pairs, hipStream_t s);
hipError_t launch_ld_fast(int pass, const uint8_t *Gp, const LdFast *fv, const uint32_t *chrom_id,
                          const LdWindowArgs &a, const uint32_t *blocks, uint32_t nblocks, uint16_t *cnt,
                          LdOffsets off, LdPair *pairs, const LdStage &st, hipStream_t s);
// per 256-group: 1 = every variant complete; 2 = (sparse != 0) every variant has at most
// kLdSparseMax missing calls (the sparse-correction kernel's groups); 0 = other
constexpr int kLdSparseMax = 15;
// (m_dev: the variant count on the device, m its upper bound)
hipError_t launch_ld_groups(const LdVar *vars, uint64_t m, int ns, int sparse, uint8_t *gflag, hipStream_t s,
                            const uint64_t *m_dev = nullptr);

// the sparse-missing form of k_ld_fast (vcfxg_ld_fast.hip, kSp): per variant its missing samples
// (CSR: moff[v] .. moff[v + 1] into midx = sample, mvar = v) and the sample-major contribution
// plane gt16[s * mp + v] = c(code): x | x^2 << 5 | missing << 11 (x = 0 for a missing call)
struct LdSpRec {
    uint64_t pk;   // missing count | Sx << 8 | Sx2 << 32
    double varx;   // LdVar::varx
};
struct LdSparse {
    const LdVar *vars = nullptr;
    const uint16_t *gt16 = nullptr;
    uint64_t mp = 0;           // gt16 row stride (variants, a multiple of 256, zero past m)
    const uint64_t *moff = nullptr;
    const uint16_t *midx = nullptr;
    const uint32_t *mvar = nullptr;
    const uint16_t *midx16 = nullptr;  // per variant its first 16 missing samples ([v][16], the rest unset)
    float pe = 0.f;            // the fp32 prefilter's error bound (as k_ld_mask)
    // per variant (m + 1 entries, the last zero): the packed (missing count, Sx, Sx2) and the own
    // variance, DMA'd into LDS with the first k-slices (k_ld_sprec)
    const LdSpRec *rec = nullptr;
};
hipError_t launch_ld_miss_fill(const int8_t *Gc, uint64_t m, int kpad, int ns, const uint64_t *moff, uint16_t *midx,
                               uint32_t *mvar, uint16_t *midx16, hipStream_t s);
hipError_t launch_ld_sprec(const LdVar *vars, uint64_t m, int ns, LdSpRec *rec, hipStream_t s);
hipError_t launch_ld_gt16(const int8_t *Gc, uint64_t m, int kpad, int ns, uint64_t mp, uint16_t *gt16, hipStream_t s);
hipError_t launch_ld_sparse(int pass, const uint8_t *Gp, const LdSparse &sp, const uint32_t *chrom_id,
                            const LdWindowArgs &a, const uint32_t *blocks, uint32_t nblocks, uint16_t *cnt,
                            LdOffsets off, LdPair *pairs, const LdStage &st, hipStream_t s);
// (vars: the rows of variant v are Gc + vars[v].line * kpad -- the walk's slots -- instead of v * kpad)
hipError_t launch_ld_pack4(const int8_t *Gc, uint64_t m, int kpad, int ns, uint8_t *Gp, int kp4, hipStream_t s,
                           const LdVar *vars = nullptr);
hipError_t launch_mfma_f4_selftest(const uint8_t *A, const uint8_t *B, float *C, hipStream_t s);
// FP4 row bytes for ns samples: two per byte, whole 64-byte k-slices
inline int ld_kp4(int ns) { return ns > 0 ? ((ns + 127) / 128) * 64 : 64; }
// tiles (128 x 128, list of (I, J) tile indices) where a side holds a missing genotype: the six
// pair sums of computeRsqSIMD on the FP4 MFMA (Gx = the dosage plane = Gp, Gv the valid mask,
// Gq the squared dosage; vcfxg_ld_mask.hip)
hipError_t launch_ld_mask(int pass, const uint8_t *Gx, const uint8_t *Gv, const uint8_t *Gq, const LdVar *vars,
                          const uint32_t *chrom_id, const LdWindowArgs &a, const uint32_t *tiles, uint32_t ntiles,
                          uint16_t *cnt, LdOffsets off, LdPair *pairs, hipStream_t s);
hipError_t launch_ld_pack_vq(const int8_t *Gc, uint64_t m, int kpad, int ns, uint8_t *Gv, uint8_t *Gq, int kp4,
                             hipStream_t s);
hipError_t launch_ld_block(int pass, const int8_t *Gc, const LdVar *vars, const uint32_t *chrom_id,
                           const LdWindowArgs &a, const uint32_t *blocks, uint32_t nblocks, uint16_t *cnt,
                           LdOffsets off, LdPair *pairs, hipStream_t s);
hipError_t launch_ld_prefix(int which, const LdVar *vars, uint64_t m, const char *buf, int id_dot_to_pos,
                            uint64_t *len_or_off, char *out, hipStream_t s);
hipError_t launch_ld_pairtext(int which, const LdPair *pairs, uint64_t np, const uint64_t *poff, const char *prefix,
                              uint64_t *len_or_off, char *out, hipStream_t s);
hipError_t launch_ld_matrix(const int8_t *Gc, const LdVar *vars, uint64_t m, int kpad, int ns, int gate, int printf4,
                            const uint32_t *blocks, uint32_t nblocks, char *cells, hipStream_t s);
hipError_t launch_mfma_i8_selftest(const int8_t *A, const int8_t *B, int *C, hipStream_t s);


}  // namespace vcfxg
