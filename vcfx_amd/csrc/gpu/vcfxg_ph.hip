// vcfxg_ph.hip -- VCFX_haplotype_phaser's per-record parse and consecutive-variant LD (SURVEY
// 8(f) rank 3: LD reuse in block phasing).
//
// The phaser groups variants into blocks by r^2 between a variant and the last variant of the
// current block, which is always the variant before it (groupVariants, VCFX_haplotype_phaser.cpp
// :1275-1322, and the streaming loops :757-965 / :1086-1259): so the device computes, for every
// parsed variant v > 0, calculateLDFast (:366-470) of the pair (v - 1, v) and the decision the
// reference takes on it (r^2 >= threshold, and r > 0 on chromosome "1"), plus whether the two
// share CHROM.  The host assembles the block lines from these flags and the variants' entry
// texts "idx:(chrom:pos)" formatted here.
//
//   k_ph_lines  wave per line: the line rules of both input modes (status), POS, the FORMAT's
//               GT index and one genotype code per sample (parseGenotypeFast :312-357: the
//               allele sum as int8, -1 missing) into row `line` of G (kpad bytes per row): the
//               fixed-stride sweep (gt_fast) for GT-only records, else a lane per sample start;
//   k_ph_pairs  wave per variant: the pair sums over min(ns) samples (valid = both >= 0), the
//               reference's fp64 sequence in correctly rounded operations, the decision, the
//               CHROM compare and the entry length;
//   k_ph_fmt    the entries at their scanned offsets.
#include <algorithm>

#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

constexpr int kPhThreads = 256;
constexpr int kPhWaves = kPhThreads / kWave;
constexpr int kPhLdsRow = 4096;
constexpr int kPhUnroll = 4;     // k_ph_pairs: 16 B loads of each row in flight per lane  // samples per record composed in LDS (more: byte stores to HBM)

// parseGenotypeFast on [g, g + n)
__device__ __forceinline__ int ph_gt(const char *__restrict__ buf, int64_t g, int64_t n) {
    if (n <= 0) return -1;
    if (n == 3) {
        const uint32_t c0 = byte_at(buf, g), c1 = byte_at(buf, g + 1), c2 = byte_at(buf, g + 2);
        if (c1 == '/' || c1 == '|') {
            if (c0 == '.' || c2 == '.') return -1;
            if (c0 - '0' < 10u && c2 - '0' < 10u) return (int)(int8_t)((c0 - '0') + (c2 - '0'));
        }
    }
    int64_t k = 0;
    while (k < n && byte_at(buf, g + k) != '/' && byte_at(buf, g + k) != '|') k++;
    if (k == n) return -1;
    const int64_t n1 = k, n2 = n - k - 1;
    if (!n1 || !n2 || byte_at(buf, g) == '.' || byte_at(buf, g + k + 1) == '.') return -1;
    uint32_t i1 = 0, i2 = 0;
    for (int64_t j = 0; j < n1; j++) {
        const uint32_t c = byte_at(buf, g + j);
        if (c - '0' >= 10u) return -1;
        i1 = i1 * 10u + (c - '0');
    }
    for (int64_t j = 0; j < n2; j++) {
        const uint32_t c = byte_at(buf, g + k + 1 + j);
        if (c - '0' >= 10u) return -1;
        i2 = i2 * 10u + (c - '0');
    }
    return (int)(int8_t)(i1 + i2);
}

// the sample at st (ends at the next tab or E): its gi-th ':' sub-field (extractNthField)
__device__ __forceinline__ int ph_sample(const char *__restrict__ buf, int64_t st, int64_t E, int gi) {
    int cur = 0;
    int64_t fs = st;
    for (int64_t q = st;; q++) {
        const uint32_t c = q < E ? byte_at(buf, q) : (uint32_t)'\t';
        if (c == '\t' || c == ':') {
            if (cur == gi) return ph_gt(buf, fs, q - fs);
            if (c == '\t') return -1;
            cur++;
            fs = q + 1;
        }
    }
}

// fixed-stride reducer: the code of every sample into its row
struct PhOp {
    int8_t *row;
    int64_t S;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {
        if (!v.real) return;
        const uint32_t a = v.f & 0xFFu, b = (v.f >> 16) & 0xFFu;
        row[(v.p - S) >> 2] = (int8_t)(v.dig == 0x01000100u ? (int)(a + b) : -1);
    }
    __device__ void finish() {}
};

// the same codes into the wave's LDS row (an LDS-address-space pointer: ds_write_b8, not flat)
struct PhOpL {
    __attribute__((address_space(3))) int8_t *row;
    int64_t S;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {
        if (!v.real) return;
        const uint32_t a = v.f & 0xFFu, b = (v.f >> 16) & 0xFFu;
        row[(v.p - S) >> 2] = (int8_t)(v.dig == 0x01000100u ? (int)(a + b) : -1);
    }
    __device__ void finish() {}
};

struct PhLine {
    uint64_t chrom;  // CHROM start
    uint32_t clen;   // CHROM bytes
    int32_t pos;
    uint32_t ns;     // samples (fields after the 9th)
    uint32_t pad;
};

// kFast: the first pass -- fixed-stride records composed in LDS (and every head-only status);
// any other record is left kPhPend for the second pass (kFast = false, which skips every other
// line), so the first pass carries none of the per-sample-start parser's registers
constexpr uint8_t kPhPend = 0xFE;
template <bool kFast>
__global__ __launch_bounds__(kPhThreads) void k_ph_lines(const char *__restrict__ buf, int64_t data_start,
                                                         const uint64_t *__restrict__ line_end,
                                                         const uint64_t *n_lines_p, int mode, uint32_t kpad,
                                                         int8_t *__restrict__ G, uint8_t *__restrict__ status,
                                                         uint32_t *__restrict__ isvar, PhLine *__restrict__ info,
                                                         unsigned long long *__restrict__ counters,
                                                         const LineMeta *__restrict__ wmeta, unsigned *__restrict__ bad) {
    __shared__ int64_t scratch[kPhWaves][16];
    // a GT-only fixed-stride record's codes are composed in the wave's LDS row (byte writes)
    // and leave in 16 B stores: a byte store per sample to HBM would be 4 store instructions
    // per lane per KiB of record
    __shared__ __attribute__((aligned(16))) int8_t lrows[kPhWaves][kPhLdsRow];
    int64_t *lds = scratch[threadIdx.x / kWave];
    int8_t *lrow = lrows[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        if (!kFast && status[li] != kPhPend) continue;  // (wave-uniform)
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start, le = (int64_t)line_end[li];
        const LineMeta wm = wmeta ? wmeta[li] : LineMeta{};
        uint8_t st = kPhSkip;
        bool swept_fixed = false;
        PhLine m{};
        if (!(mode == 1 && le == ls)) {  // stdin: an empty line before the '\r' strip
            int64_t ae = le;
            if (ae > ls && byte_at(buf, ae - 1) == '\r') ae--;
            if (ae == ls) st = mode == 0 ? kPhSkip : kPhFew;  // (stdin: a lone '\r' is a 1-field line)
            else if (byte_at(buf, ls) == '#') st = kPhHeader;
            else {
                int64_t t0 = 0, t8 = 0;
                int nt = 0, gi = -1;
                bool ok = true;  // POS: every byte a digit (an empty POS is 0), int accumulation
                uint32_t pos = 0;
                bool head = false;
                if (kFast && wmeta && wm.kind == kMetaGt && (int64_t)wm.S > ls) {
                    // a record of the head walk: its 9 tabs were found (S = the 9th + 1) and its
                    // FORMAT starts "GT" (index 0), so CHROM and POS come from one 64-byte load --
                    // no head sweep, no byte-by-byte POS loop of dependent loads
                    const int64_t q = ls + lane();
                    const uint32_t c = q < ae ? byte_at(buf, q) : 0u;
                    const uint64_t tb = __ballot(c == '\t');
                    if (__popcll(tb) >= 2) {
                        t0 = ls + __builtin_ctzll(tb);
                        const int64_t t1 = ls + __builtin_ctzll(tb & (tb - 1));
                        t8 = (int64_t)wm.S - 1;
                        nt = 9;
                        gi = 0;
                        head = true;
                        // POS = sum of digit * 10^(place), mod 2^32 like the serial accumulation
                        const bool in = q > t0 && q < t1;
                        ok = !__any(in && c - '0' >= 10u);
                        uint32_t pw = 1;
                        for (int64_t k = t1 - 1 - q; in && k > 0; k--) pw *= 10u;
                        pos = wave_sum(in && ok ? (c - '0') * pw : 0u);
                        if (!ok) gi = -1;
                    }
                }
                if (!head) {
                    int64_t t[9];
                    nt = head_tabs(buf, ls, ae, 9, t, lds);
                    if (nt >= 9) {
                        t0 = t[0];
                        t8 = t[8];
                        for (int64_t q = t[0] + 1; q < t[1]; q++) {
                            const uint32_t c = byte_at(buf, q);
                            if (c - '0' >= 10u) {
                                ok = false;
                                break;
                            }
                            pos = pos * 10u + (c - '0');
                        }
                        gi = ok ? gt_index(buf, t[7] + 1, t[8]) : -1;
                    }
                }
                if (nt < 9) st = kPhFew;
                else {
                    if (!ok) st = kPhPos;
                    else if (gi < 0) st = kPhNoGt;
                    else {
                        st = kPhVar;
                        m.chrom = (uint64_t)ls;
                        m.clen = (uint32_t)(t0 - ls);
                        m.pos = (int32_t)pos;
                        const int64_t S = t8 + 1;
                        int8_t *row = G + li * (uint64_t)kpad;
                        const int64_t L = ae - S;
                        const bool fixed = gi == 0 && L >= 3 && ((L + 1) & 3) == 0 && (uint64_t)((L + 1) / 4) <= kpad;
                        bool swept = false;
                        if (fixed && (L + 1) / 4 <= kPhLdsRow) {
                            PhOpL op{(__attribute__((address_space(3))) int8_t *)lrow, S};
                            swept = gt_fast(buf, S, ae, op);
                            if (swept) {
                                const uint32_t ns = (uint32_t)((L + 1) / 4);
                                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                                __builtin_amdgcn_wave_barrier();
                                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                                for (uint32_t o = (uint32_t)lane() * 16; o < ns; o += kWave * 16) {
                                    if (o + 16 <= ns)
                                        *reinterpret_cast<uint4 *>(row + o) = *reinterpret_cast<const uint4 *>(lrow + o);
                                    else
                                        for (uint32_t q = o; q < ns; q++) row[q] = lrow[q];
                                }
                                // the next line's byte writes must not pass these reads
                                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                                __builtin_amdgcn_wave_barrier();
                            }
                        } else if (!kFast && fixed) {
                            PhOp op{row, S};
                            swept = gt_fast(buf, S, ae, op);
                        }
                        swept_fixed = swept;
                        if (swept)
                            m.ns = (uint32_t)((L + 1) / 4);
                        else if (kFast)
                            st = kPhPend;
                        else {
                            // a lane per sample start; sample k = its rank among the starts
                            uint32_t cnt = 0;
                            for (int64_t w = S & ~(int64_t)15; w <= ae; w += kWaveStep) {
                                const int64_t blk = w + (int64_t)lane() * kBlockBytes;
                                uint32_t starts = 0;
                                if (blk <= ae) {
                                    const uint32_t tm = eq_mask16(load16(buf, blk), kRepTab);
                                    starts = (tm << 1) & 0xFFFFu;
                                    if (blk > 0 && byte_at(buf, blk - 1) == '\t') starts |= 1u;
                                    starts &= range_mask16(blk, S + 1, ae + 1);  // (a trailing tab: a sample at ae)
                                    if (S >= blk && S < blk + 16) starts |= 1u << (S - blk);
                                }
                                const uint32_t c = (uint32_t)__popc(starts);
                                const uint32_t incl = wave_incl_scan(c);
                                uint32_t k = cnt + incl - c;
                                while (starts) {
                                    const int j = __builtin_ctz(starts);
                                    starts &= starts - 1u;
                                    if (k < kpad) row[k] = (int8_t)ph_sample(buf, blk + j, ae, gi);
                                    k++;
                                }
                                cnt += wave_bcast(incl, kWave - 1);
                            }
                            m.ns = cnt;
                            if (cnt > kpad && lane() == 0) atomicMax(&counters[3], (unsigned long long)cnt);
                        }
                    }
                }
            }
        }
        // a record the head walk took on its predicted end: its bounds hold only if the fixed-stride
        // sweep validated [S, ae) (no '\n' inside); any other outcome redoes the call on the index
        if (wmeta && st != kPhPend && !(st == kPhVar && swept_fixed) && (wm.pad & kWalkUnswept) &&
            wm.kind == kMetaGt && lane() == 0)
            atomicOr(bad, 1u);
        if (lane() == 0) {
            status[li] = st;
            isvar[li] = st == kPhVar;
            info[li] = m;
        }
    }
}

__device__ __forceinline__ uint32_t ph_digits(uint64_t v) {  // (compares, no 64-bit division)
    uint32_t d = 1;
    for (uint64_t p = 10; d < 20 && v >= p; p *= 10) d++;
    return d;
}
__device__ __forceinline__ uint32_t ph_int_len(int64_t v) { return v < 0 ? 1u + ph_digits((uint64_t)-v) : ph_digits((uint64_t)v); }

// 16 codes per lane of two rows (x, y; a negative code is missing) into the six sums' lane parts:
// four codes per dword, valid where both are >= 0 (bit 7 clear) and the sample is below n; the
// sums by byte dot products of the codes masked to the valid bytes (v_dot4_u32_u8, v_sad_u8),
// not a loop over the 16 codes.  Fields: (valid, Sx) | (Sy, Sxy) | (Sx2, Sy2), 32 bits each.
__device__ __forceinline__ void ph_acc16(const uint4 &va, const uint4 &vb, uint32_t k0, uint32_t n, uint64_t &p0,
                                         uint64_t &p1, uint64_t &p2) {
    const uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
    uint32_t vn = 0, sx = 0, sy = 0, sxy = 0, sx2 = 0, sy2 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int rem = (int)n - (int)(k0 + 4 * i);
        const uint32_t lim = rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u;
        const uint32_t m = ~(wa[i] | wb[i]) & 0x80808080u & lim;
        const uint32_t mb = (m - (m >> 7)) | m;  // 0xFF per valid byte
        const uint32_t xs = wa[i] & mb, ys = wb[i] & mb;
        vn += __popc(m);
        sx = __builtin_amdgcn_sad_u8(xs, 0u, sx);
        sy = __builtin_amdgcn_sad_u8(ys, 0u, sy);
        sxy = __builtin_amdgcn_udot4(xs, ys, sxy, false);
        sx2 = __builtin_amdgcn_udot4(xs, xs, sx2, false);
        sy2 = __builtin_amdgcn_udot4(ys, ys, sy2, false);
    }
    p0 += (uint64_t)vn | (uint64_t)sx << 32;
    p1 += (uint64_t)sy | (uint64_t)sxy << 32;
    p2 += (uint64_t)sx2 | (uint64_t)sy2 << 32;
}

// calculateLDFast's fp64 tail (:440-470) on the pair's six sums, correctly rounded, and the block
// rule (r^2 >= thr, and r > 0 on CHROM "1"); flags as k_ph_pairs writes them
__device__ __forceinline__ uint8_t ph_pair_flags(const PhLine &, const PhLine &, bool one, bool same, int64_t N,
                                                 int64_t SX, int64_t SY, int64_t SXY, int64_t SX2, int64_t SY2,
                                                 double thr, double &r2v) {
    double r = 0.0;
    r2v = 0.0;
    if (N > 0) {
        const double dn = (double)N;
        const double mx = __ddiv_rn((double)SX, dn), my = __ddiv_rn((double)SY, dn);
        const double cov = __dsub_rn(__ddiv_rn((double)SXY, dn), __dmul_rn(mx, my));
        const double vx = __dsub_rn(__ddiv_rn((double)SX2, dn), __dmul_rn(mx, mx));
        const double vy = __dsub_rn(__ddiv_rn((double)SY2, dn), __dmul_rn(my, my));
        if (vx > 0.0 && vy > 0.0) {
            r = __ddiv_rn(cov, __dmul_rn(__dsqrt_rn(vx), __dsqrt_rn(vy)));
            r2v = __dmul_rn(r, r);
        }
    }
    const bool pass = one ? (r2v >= thr && r > 0.0) : (r2v >= thr);
    return (uint8_t)((pass ? 1u : 0u) | (same ? 2u : 0u));
}

// k_ph_pairs for rows of at most kU KiB: a wave takes kPhRun consecutive variants, each row
// loaded once into registers (the next two rows' loads in flight while a pair reduces) and kept
// as the next pair's first row -- every code read once, not twice
constexpr uint64_t kPhRun = 32;
template <int kU>
__global__ __launch_bounds__(kPhThreads) void k_ph_pairs_run(const char *__restrict__ buf,
                                                             const uint64_t *__restrict__ vline,
                                                             const uint64_t *n_var_p, const PhLine *__restrict__ info,
                                                             const int8_t *__restrict__ G, uint32_t kpad, double thr,
                                                             uint8_t *__restrict__ flags, uint64_t *__restrict__ len,
                                                             double *__restrict__ r2_out) {
    const uint64_t nv = *n_var_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    auto load_row = [&](uint64_t line, uint4(&r)[kU]) {
#pragma unroll
        for (int u = 0; u < kU; u++) {
            uint32_t k0 = 16u * (lane() + kWave * u);
            k0 = k0 < kpad ? k0 : kpad - 16u;  // (bytes past the row are masked by n)
            r[u] = *reinterpret_cast<const uint4 *>(G + line * (uint64_t)kpad + k0);
        }
    };
    // a PhLine field of variant lane k of the run (preloaded by lane k), wave-uniform
    // (readlane returns int: each half goes through uint32_t, or the low half would sign-extend
    // into the high one -- offsets past 2 GiB)
    auto rd64 = [](uint64_t x, int k) {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), k) << 32) |
               (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)x, k);
    };
    for (uint64_t v0 = wid * kPhRun; v0 < nv; v0 += nw * kPhRun) {
        const uint64_t v1 = std::min<uint64_t>(nv, v0 + kPhRun);
        // lane k < run length: variant v0 - 1 + k's line and PhLine (one load each, all lanes at
        // once, instead of a dependent chain per variant)
        const int64_t vk = (int64_t)v0 - 1 + lane();
        uint64_t mline = 0, mchrom = 0;
        uint32_t mclen = 0, mns = 0;
        int32_t mpos = 0;
        if (vk >= 0 && (uint64_t)vk < v1) {
            mline = vline[vk];
            const PhLine q = info[mline];
            mchrom = q.chrom, mclen = q.clen, mns = q.ns, mpos = q.pos;
        }
        auto line_of = [&](uint64_t v) { return rd64(mline, (int)(v + 1 - v0)); };
        auto info_of = [&](uint64_t v) {
            const int k = (int)(v + 1 - v0);
            PhLine q{};
            q.chrom = rd64(mchrom, k);
            q.clen = __builtin_amdgcn_readlane(mclen, k);
            q.ns = __builtin_amdgcn_readlane(mns, k);
            q.pos = (int32_t)__builtin_amdgcn_readlane((uint32_t)mpos, k);
            return q;
        };
        // a CHROM's bytes, one per lane (CHROMs of up to 64 bytes; longer ones compared in a loop)
        auto chrom_bytes = [&](const PhLine &q) {
            return (uint32_t)lane() < q.clen ? (uint32_t)(uint8_t)buf[q.chrom + lane()] : 0u;
        };
        uint4 ra[kU], rb[kU];
        PhLine a{};
        uint32_t ca = 0;
        if (v0 > 0) {
            a = info_of(v0 - 1);
            ca = chrom_bytes(a);
            load_row(line_of(v0 - 1), ra);
        }
        uint64_t lb = line_of(v0);
        load_row(lb, rb);
        // the next two rows in flight while a pair reduces (one ahead left every iteration waiting
        // on its row)
        uint4 rn[kU], rm[kU];
        if (v0 + 1 < v1) load_row(line_of(v0 + 1), rn);
        // lane j keeps variant v0 + j's six sums and CHROM flags; the fp64 tails, the entry
        // lengths and the stores then run once for the whole run, a variant per lane
        uint64_t s0 = 0, s1 = 0, s2 = 0;
        uint32_t sf = 0;  // bit 0: a pair, bit 1: CHROM "1", bit 2: same CHROM
        for (uint64_t v = v0; v < v1; v++) {
            const PhLine b = info_of(v);
            const uint32_t cb = chrom_bytes(b);
            if (v + 2 < v1) load_row(line_of(v + 2), rm);
            if (v > 0) {
                const uint32_t n = min(a.ns, b.ns);
                uint64_t p0 = 0, p1 = 0, p2 = 0;
#pragma unroll
                for (int u = 0; u < kU; u++) ph_acc16(ra[u], rb[u], 16u * (lane() + kWave * u), n, p0, p1, p2);
                const uint64_t q0 = (uint64_t)wave_sum((int64_t)p0), q1 = (uint64_t)wave_sum((int64_t)p1),
                               q2 = (uint64_t)wave_sum((int64_t)p2);
                const bool one = b.clen == 1 && __builtin_amdgcn_readfirstlane(cb) == '1';
                bool same = a.clen == b.clen && !__any(ca != cb);
                for (uint32_t k = kWave; same && k < a.clen; k++) same = buf[a.chrom + k] == buf[b.chrom + k];
                if ((uint64_t)lane() == v - v0) {
                    s0 = q0, s1 = q1, s2 = q2;
                    sf = 1u | (one ? 2u : 0u) | (same ? 4u : 0u);
                }
            }
#pragma unroll
            for (int u = 0; u < kU; u++) ra[u] = rb[u], rb[u] = rn[u], rn[u] = rm[u];
            a = b;
            ca = cb;
        }
        const uint64_t v = v0 + lane();
        // variant v0 + j's CHROM length and POS: lane j + 1's preloaded ones
        const uint32_t vclen = (uint32_t)__shfl_down((int)mclen, 1);
        const int32_t vpos = __shfl_down(mpos, 1);
        if (v < v1) {
            uint8_t f = 0;
            double r2v = 0.0;
            if (sf & 1u)
                f = ph_pair_flags(a, a, (sf & 2u) != 0, (sf & 4u) != 0, (uint32_t)s0, s0 >> 32, (uint32_t)s1,
                                  s1 >> 32, (uint32_t)s2, s2 >> 32, thr, r2v);
            flags[v] = f;
            r2_out[v] = r2v;
            len[v] = ph_digits(v) + 2u + vclen + 1u + ph_int_len(vpos) + 1u;
        }
    }
}

// per variant v: vline[v] = its line.  flags: bit 0 the pair (v - 1, v) passes the block rule,
// bit 1 the two share CHROM.  len: bytes of the entry "v:(chrom:pos)".
__global__ __launch_bounds__(kPhThreads) void k_ph_pairs(const char *__restrict__ buf, const uint64_t *__restrict__ vline,
                                                         const uint64_t *n_var_p, const PhLine *__restrict__ info,
                                                         const int8_t *__restrict__ G, uint32_t kpad, double thr,
                                                         uint8_t *__restrict__ flags, uint64_t *__restrict__ len,
                                                         double *__restrict__ r2_out) {
    const uint64_t nv = *n_var_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t v = wid; v < nv; v += nw) {
        const PhLine b = info[vline[v]];
        uint8_t f = 0;
        double r2v = 0.0;
        if (v > 0) {
            const PhLine a = info[vline[v - 1]];
            const int8_t *ga = G + vline[v - 1] * (uint64_t)kpad, *gb = G + vline[v] * (uint64_t)kpad;
            const uint32_t n = min(a.ns, b.ns);
            // per lane and pass: (valid, Sx) | (Sy, Sxy) | (Sx2, Sy2) as two 32-bit fields of
            // one 64-bit word each, so a pass reduces three 64-bit sums instead of six (a pass
            // covers 16 * 64 * kPhUnroll codes: a field stays below 127^2 * 4096 < 2^32)
            int64_t N = 0, SX = 0, SY = 0, SXY = 0, SX2 = 0, SY2 = 0;
            // 16 codes per lane per load, kPhUnroll loads of each row in flight (rows are 16-byte
            // aligned and kpad long; bytes past n are masked, a load past the row re-reads its
            // last 16 bytes)
            for (uint32_t b0 = 0; b0 < n; b0 += 16u * kWave * kPhUnroll) {
                uint4 va[kPhUnroll], vb[kPhUnroll];
#pragma unroll
                for (int u = 0; u < kPhUnroll; u++) {
                    uint32_t k0 = b0 + 16u * (lane() + kWave * u);
                    k0 = k0 < kpad ? k0 : kpad - 16u;
                    va[u] = *reinterpret_cast<const uint4 *>(ga + k0);
                    vb[u] = *reinterpret_cast<const uint4 *>(gb + k0);
                }
                uint64_t p0 = 0, p1 = 0, p2 = 0;
#pragma unroll
                for (int u = 0; u < kPhUnroll; u++) ph_acc16(va[u], vb[u], b0 + 16u * (lane() + kWave * u), n, p0, p1, p2);
                const uint64_t q0 = (uint64_t)wave_sum((int64_t)p0), q1 = (uint64_t)wave_sum((int64_t)p1),
                               q2 = (uint64_t)wave_sum((int64_t)p2);
                N += (uint32_t)q0;
                SX += q0 >> 32;
                SY += (uint32_t)q1;
                SXY += q1 >> 32;
                SX2 += (uint32_t)q2;
                SY2 += q2 >> 32;
            }
            const bool one = b.clen == 1 && byte_at(buf, (int64_t)b.chrom) == '1';
            bool same = a.clen == b.clen;
            for (uint32_t k = 0; same && k < a.clen; k++) same = buf[a.chrom + k] == buf[b.chrom + k];
            f = ph_pair_flags(a, b, one, same, N, SX, SY, SXY, SX2, SY2, thr, r2v);
        }
        if (lane() == 0) {
            flags[v] = f;
            r2_out[v] = r2v;
            len[v] = ph_digits(v) + 2u + b.clen + 1u + ph_int_len(b.pos) + 1u;
        }
    }
}

__device__ __forceinline__ void ph_put_int(char *o, int64_t v, uint32_t nb) {
    uint64_t x = v < 0 ? (uint64_t)-v : (uint64_t)v;
    if (v < 0) o[0] = '-';
    for (uint32_t k = nb; k-- > (v < 0 ? 1u : 0u);) {
        o[k] = (char)('0' + x % 10);
        x /= 10;
    }
}

__global__ __launch_bounds__(kPhThreads) void k_ph_fmt(const char *__restrict__ buf, const uint64_t *__restrict__ vline,
                                                       const uint64_t *n_var_p, const PhLine *__restrict__ info,
                                                       const uint64_t *__restrict__ off, char *__restrict__ out) {
    const uint64_t nv = *n_var_p;
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < nv; v += gridDim.x * (uint64_t)blockDim.x) {
        const PhLine b = info[vline[v]];
        char *o = out + off[v];
        uint32_t nb = ph_digits(v);
        ph_put_int(o, (int64_t)v, nb);
        o += nb;
        *o++ = ':';
        *o++ = '(';
        for (uint32_t k = 0; k < b.clen; k++) *o++ = buf[b.chrom + k];
        *o++ = ':';
        nb = ph_int_len(b.pos);
        ph_put_int(o, b.pos, nb);
        o += nb;
        *o = ')';
    }
}

// variant number -> line (the lines with isvar set, in order)
__global__ void k_ph_compact(const uint32_t *__restrict__ isvar, const uint64_t *__restrict__ vnum,
                             const uint64_t *n_lines_p, uint64_t *__restrict__ vline, uint64_t *__restrict__ n_var) {
    const uint64_t n = *n_lines_p;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gridDim.x * (uint64_t)blockDim.x) {
        if (isvar[i]) vline[vnum[i]] = i;
        if (i == n - 1) *n_var = vnum[i] + isvar[i];
    }
}

size_t ph_line_bytes() { return sizeof(PhLine); }

hipError_t launch_ph_lines(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, int mode, uint32_t kpad, int8_t *G, uint8_t *status, uint32_t *isvar,
                           void *info, unsigned long long *counters, hipStream_t s, const void *walk_meta,
                           unsigned *bad) {
    if (!n_lines_host) return hipSuccess;
    if (walk_meta && !bad) return hipErrorInvalidValue;
    const LineMeta *wm = static_cast<const LineMeta *>(walk_meta);
    int64_t g = ((int64_t)n_lines_host + kPhWaves - 1) / kPhWaves;
    if (g > 4096) g = 4096;
    // (a record's sweep with 8 KiB-steps in flight per wave measured the same as 4: r02)
    hipLaunchKernelGGL(k_ph_lines<true>, dim3((unsigned)g), dim3(kPhThreads), 0, s, buf, data_start, line_end,
                       n_lines_dev, mode, kpad, G, status, isvar, static_cast<PhLine *>(info), counters, wm, bad);
    hipLaunchKernelGGL(k_ph_lines<false>, dim3((unsigned)std::min<int64_t>(g, 2048)), dim3(kPhThreads), 0, s, buf,
                       data_start, line_end, n_lines_dev, mode, kpad, G, status, isvar,
                       static_cast<PhLine *>(info), counters, wm, bad);
    return hipGetLastError();
}

hipError_t launch_ph_compact(const uint32_t *isvar, const uint64_t *vnum, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, uint64_t *vline, uint64_t *n_var, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    int64_t g = ((int64_t)n_lines_host + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_ph_compact, dim3((unsigned)g), dim3(256), 0, s, isvar, vnum, n_lines_dev, vline, n_var);
    return hipGetLastError();
}

hipError_t launch_ph_pairs(const char *buf, const uint64_t *vline, const uint64_t *n_var_dev, uint64_t n_var_host,
                           const void *info, const int8_t *G, uint32_t kpad, double thr, uint8_t *flags, uint64_t *len,
                           double *r2, hipStream_t s) {
    if (!n_var_host) return hipSuccess;
    int64_t g = ((int64_t)n_var_host + kPhWaves - 1) / kPhWaves;
    if (g > 4096) g = 4096;
    const PhLine *in = static_cast<const PhLine *>(info);
    // rows of up to 4 KiB: consecutive variants per wave, each row read once
    const int ku = (int)((kpad + 1023) / 1024);
    const unsigned gr = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(4096, (n_var_host + kPhWaves * kPhRun - 1) /
                                                                                      (kPhWaves * kPhRun)));
    if (ku == 1)
        hipLaunchKernelGGL(k_ph_pairs_run<1>, dim3(gr), dim3(kPhThreads), 0, s, buf, vline, n_var_dev, in, G, kpad, thr,
                           flags, len, r2);
    else if (ku == 2)
        hipLaunchKernelGGL(k_ph_pairs_run<2>, dim3(gr), dim3(kPhThreads), 0, s, buf, vline, n_var_dev, in, G, kpad, thr,
                           flags, len, r2);
    else if (ku == 3)
        hipLaunchKernelGGL(k_ph_pairs_run<3>, dim3(gr), dim3(kPhThreads), 0, s, buf, vline, n_var_dev, in, G, kpad, thr,
                           flags, len, r2);
    else if (ku == 4)
        hipLaunchKernelGGL(k_ph_pairs_run<4>, dim3(gr), dim3(kPhThreads), 0, s, buf, vline, n_var_dev, in, G, kpad, thr,
                           flags, len, r2);
    else
        hipLaunchKernelGGL(k_ph_pairs, dim3((unsigned)g), dim3(kPhThreads), 0, s, buf, vline, n_var_dev, in, G, kpad,
                           thr, flags, len, r2);
    return hipGetLastError();
}

hipError_t launch_ph_fmt(const char *buf, const uint64_t *vline, const uint64_t *n_var_dev, uint64_t n_var_host,
                         const void *info, const uint64_t *off, char *out, hipStream_t s) {
    if (!n_var_host) return hipSuccess;
    int64_t g = ((int64_t)n_var_host + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_ph_fmt, dim3((unsigned)g), dim3(256), 0, s, buf, vline, n_var_dev,
                       static_cast<const PhLine *>(info), off, out);
    return hipGetLastError();
}

}  // namespace vcfxg
