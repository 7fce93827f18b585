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
hipError_t launch_ld_groups(const LdVar *vars, uint64_t m, uint8_t *gflag, hipStream_t s);
hipError_t launch_ld_pack4(const int8_t *Gc, uint64_t m, int kpad, int ns, uint8_t *Gp, int kp4, hipStream_t s);
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
