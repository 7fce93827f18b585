// vcfxg_af_walk.hip -- VCFX_allele_freq_calc's record pass without a separate line index.
//
// The data region is cut into C-byte chunks, one wave ("walker") each.  A line belongs to
// the chunk holding its first byte.  A walker finds the first line start of its chunk (the
// byte after the first '\n' at or after chunk start - 1: a short scan over the tail of the
// previous chunk's last line) and then walks its lines one after the other:
//
//   1. one 1 KiB window at the line start (16 B per lane) gives the first '\n' if the line
//      is short, the first 9 tabs and the FORMAT bytes (ballots + a wave scan);
//   2. the line end E: the window's '\n'; or, for a GT-only record (FORMAT == "GT"), the
//      PREDICTED end S + span (span = the '\n' distance from the sample start of the
//      walker's previous fixed-stride record, first the header's 4 * samples - 1), accepted
//      when the byte at E is '\n' (or E is the end of an input without a final '\n'); or
//      else a wave scan for the '\n';
//   3. the fixed-stride sample sweep (vcfxg_gt.h gt_fast, the reference's
//      parseGenotypeAndCount :262-293 on single-digit diploid records) over [S, E).  It
//      validates every byte of [S, E) as a digit, '.', separator or tab, so a predicted
//      end that it accepts has no '\n' before it: the bounds are exact.  If the sweep
//      rejects a predicted line, the '\n' is searched for and the line is re-swept with
//      its true bounds;
//   4. the line's end offset, counts, status and head record go to the walker's region;
//      the next line starts at E + 1 (its window is loaded before this line's sweep).
//
// So every input byte is read from HBM about once (the tail of each chunk's last line is
// read twice, the second time mostly from the Infinity Cache), against twice for the
// separate index sweep.  k_walk_compact concatenates the regions in file order and
// k_af_complex runs the exact per-line path for everything that is not a fixed-stride
// GT-first record (kMetaFull lines, kAfPending lines), exactly as after the two-sweep
// schedule.  A walker over its line capacity raises `overflow` and the caller reruns the
// two-sweep schedule.  Head semantics follow vcfxg_meta.h head_meta (processMmap :355-470 /
// processStdin :490-556): '\r' stripped in file mode, '#' lines, empty lines, GT-first
// FORMAT, row prefix = CHROM..ALT and its tab.
#include <algorithm>

#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

namespace {

constexpr int kWalkThreads = 256;
constexpr int kWalkWaves = kWalkThreads / kWave;

// first '\n' in [p, hi), else hi (wave-uniform; 4 KiB per step)
__device__ __forceinline__ int64_t scan_nl(const char *__restrict__ buf, int64_t p, int64_t hi) {
    constexpr int kU = 4;
    for (int64_t w = p & ~(int64_t)15; w < hi; w += kU * kWaveStep) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int64_t blk = w + (int64_t)u * kWaveStep + 16 * (int64_t)lane();
            v[u] = blk < hi ? load16(buf, blk) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int64_t blk = w + (int64_t)u * kWaveStep + 16 * (int64_t)lane();
            const uint32_t m = eq_mask16(v[u], kRepNl) & range_mask16(blk, p, hi);
            const uint64_t any = __ballot(m != 0u);
            if (any) {
                const int k = __builtin_ctzll(any);
                const uint32_t mk = (uint32_t)__shfl((int)m, k);
                return uniform64(w + (int64_t)u * kWaveStep + 16 * k + __builtin_ctz(mk));
            }
        }
    }
    return hi;
}

// dword `comp` (uniform) of a uint4
__device__ __forceinline__ uint32_t comp4(const uint4 &v, int comp) {
    return comp == 0 ? v.x : comp == 1 ? v.y : comp == 2 ? v.z : v.w;
}
// byte x of the window whose lane k holds [A + 16k, A + 16k + 16); A <= x < A + 1024
__device__ __forceinline__ uint32_t win_byte(const uint4 &W, int64_t A, int64_t x) {
    const int o = (int)(x - A);
    const uint32_t d = (uint32_t)__shfl((int)comp4(W, (o >> 2) & 3), o >> 4);
    return (d >> (8 * (o & 3))) & 0xFFu;
}

// the window at line start L: lane k holds [A + 16k, +16), A = L & ~15 (zeros past hi)
__device__ __forceinline__ uint4 load_window(const char *__restrict__ buf, int64_t L, int64_t hi) {
    const int64_t blk = (L & ~(int64_t)15) + 16 * (int64_t)lane();
    return blk < hi ? load16(buf, blk) : make_uint4(0, 0, 0, 0);
}

// position of the tab with 0-based rank r (< total) given per-lane tab masks and their
// exclusive per-lane counts (wave-uniform result)
__device__ __forceinline__ int64_t tab_at(uint32_t tm, uint32_t excl, uint32_t c, int r, int64_t blk) {
    const bool mine = (uint32_t)r >= excl && (uint32_t)r < excl + c;
    const uint64_t who = __ballot(mine);
    const int k = __builtin_ctzll(who);
    const int64_t p = mine ? blk + nth_bit(tm, r - (int)excl) : 0;
    return uniform64(__shfl(p, k));
}

}  // namespace

__global__ __launch_bounds__(kWalkThreads) void k_af_walk(const char *__restrict__ buf, int64_t lo, int64_t hi,
                                                          int64_t chunk, int64_t n_walkers, int mode, int64_t span0,
                                                          uint64_t cap_w, uint64_t *__restrict__ le_o,
                                                          int32_t *__restrict__ alt_o, int32_t *__restrict__ tot_o,
                                                          uint32_t *__restrict__ rowpre_o,
                                                          uint8_t *__restrict__ status_o,
                                                          LineMeta *__restrict__ meta_o, uint64_t *__restrict__ wcount,
                                                          uint32_t *__restrict__ wgt, unsigned *overflow) {
    const int64_t wk = uniform64((int64_t)blockIdx.x * kWalkWaves + threadIdx.x / kWave);
    if (wk >= n_walkers) return;
    const int strip_cr = mode == 0 ? 1 : 0;
    const int64_t cs = lo + wk * chunk;
    const int64_t ce = std::min<int64_t>(cs + chunk, hi);
    int64_t L = wk == 0 ? lo : scan_nl(buf, cs - 1, hi) + 1;
    int64_t span = span0;  // predicted '\n' distance from the sample start
    uint64_t n = 0;
    uint32_t ngt = 0;
    const uint64_t base = (uint64_t)wk * cap_w;
    uint4 W = make_uint4(0, 0, 0, 0);
    if (L < ce) W = load_window(buf, L, hi);
    while (L < ce) {
        if (n >= cap_w) {
            if (lane() == 0) atomicOr(overflow, 1u);
            break;
        }
        // ---- 1. window analysis
        const int64_t A = L & ~(int64_t)15;
        const int64_t blk = A + 16 * (int64_t)lane();
        const int64_t wend = std::min<int64_t>(A + kWaveStep, hi);
        const uint32_t nlm = eq_mask16(W, kRepNl) & range_mask16(blk, L, hi);
        const uint64_t anyn = __ballot(nlm != 0u);
        int64_t N1 = -1;
        if (anyn) {
            const int k = __builtin_ctzll(anyn);
            N1 = uniform64(A + 16 * k + __builtin_ctz((uint32_t)__shfl((int)nlm, k)));
        }
        const int64_t lim = N1 >= 0 ? N1 : wend;
        const uint32_t tm = eq_mask16(W, kRepTab) & range_mask16(blk, L, lim);
        const uint32_t tc = __popc(tm);
        const uint32_t tinc = wave_incl_scan(tc);
        const uint32_t ntab = (uint32_t)__shfl((int)tinc, kWave - 1);
        const uint32_t first = win_byte(W, A, L);
        int64_t t4 = -1, t7 = -1, t8 = -1;
        bool gt_head = false, gt_only = false;
        if (ntab >= 9 && first != '#') {
            t4 = tab_at(tm, tinc - tc, tc, 4, blk);
            t7 = tab_at(tm, tinc - tc, tc, 7, blk);
            t8 = tab_at(tm, tinc - tc, tc, 8, blk);
            if (t8 - t7 >= 3 && win_byte(W, A, t7 + 1) == 'G' && win_byte(W, A, t7 + 2) == 'T') {
                gt_only = t8 - t7 == 3;
                gt_head = gt_only || win_byte(W, A, t7 + 3) == ':';
            }
        }
        // ---- 2. line end
        int64_t E;
        bool predicted = false;
        if (N1 >= 0) {
            E = N1;
        } else if (gt_only && span > 0) {
            E = t8 + 1 + span;
            const bool ok = E < hi ? byte_at(buf, E) == '\n' : E == hi;
            if (ok) predicted = true;
            else E = scan_nl(buf, wend, hi);
        } else {
            E = scan_nl(buf, wend, hi);
        }
        // the next line's window, loaded before this line's sweep
        uint4 Wn = make_uint4(0, 0, 0, 0);
        if (E + 1 < ce) Wn = load_window(buf, E + 1, hi);
        // ---- 3. kind (head_meta) and the sweep
        uint8_t st = 0, kind, cr = 0, sep = 0;
        uint32_t alt = 0, tot = 0, rowpre = 0;
        int64_t S = 0;
        for (int pass = 0;; pass++) {
            int64_t ae = E;
            cr = 0;
            if (strip_cr && E > L && byte_at(buf, E - 1) == '\r') {
                ae = E - 1;
                cr = 1;
            }
            if (ae <= L) kind = kMetaEmpty;
            else if (first == '#') kind = kMetaHeader;
            else if (gt_head && t8 < ae) kind = kMetaGt;
            else kind = kMetaFull;
            if (kind != kMetaGt) {
                st = 0;
                break;
            }
            S = t8 + 1;
            rowpre = (uint32_t)(t4 - L + 1);
            sep = t8 + 2 < ae ? (uint8_t)byte_at(buf, t8 + 2) : 0;
            AfOp op{buf, ae, 0};
            if (gt_fast(buf, S, ae, op, sep)) {
                st = 1;
                alt = op.alt;
                tot = op.tot;
                span = E - S;
                break;
            }
            st = kAfPending;  // not fixed-stride: k_af_complex runs the general sweep
            if (!predicted || pass > 0) break;
            // a rejected prediction: the true end, then the line again with it
            const int64_t Et = scan_nl(buf, wend, hi);
            predicted = false;
            if (Et == E) break;
            E = Et;
            Wn = make_uint4(0, 0, 0, 0);
            if (E + 1 < ce) Wn = load_window(buf, E + 1, hi);
        }
        // ---- 4. outputs
        if (lane() == 0) {
            const uint64_t o = base + n;
            LineMeta m{};
            m.kind = kind;
            m.cr = cr;
            if (kind == kMetaGt) {
                m.S = (uint64_t)S;
                m.rowpre = rowpre;
                m.sep = sep;
            }
            le_o[o] = (uint64_t)E;
            alt_o[o] = (int32_t)alt;
            tot_o[o] = (int32_t)tot;
            rowpre_o[o] = kind == kMetaGt ? rowpre : 0u;
            status_o[o] = st;
            meta_o[o] = m;
        }
        ngt += kind == kMetaGt ? 1u : 0u;
        n++;
        L = E + 1;
        W = Wn;
    }
    if (lane() == 0) {
        wcount[wk] = n;
        wgt[wk] = ngt;
    }
}

// walker regions -> dense per-line arrays in file order (offs = exclusive scan of wcount);
// the rows / data-line counters (every GT-first record counts as both) are reduced per block
__global__ __launch_bounds__(256) void k_walk_compact(int64_t n_walkers, uint64_t cap_w,
                                                      const uint64_t *__restrict__ offs,
                                                      const uint32_t *__restrict__ wgt,
                                                      const uint64_t *__restrict__ le_b,
                                                      const int32_t *__restrict__ alt_b,
                                                      const int32_t *__restrict__ tot_b,
                                                      const uint32_t *__restrict__ rowpre_b,
                                                      const uint8_t *__restrict__ status_b,
                                                      const LineMeta *__restrict__ meta_b, uint64_t *line_end,
                                                      int32_t *alt, int32_t *tot, uint32_t *rowpre, uint8_t *status,
                                                      LineMeta *meta, uint64_t *n_lines,
                                                      unsigned long long *counters) {
    __shared__ uint32_t red[256 / kWave];
    // one wave per walker, lanes over its lines
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);
    uint32_t g = 0;
    for (int64_t w = (int64_t)blockIdx.x * (256 / kWave) + threadIdx.x / kWave; w < n_walkers; w += nw) {
        const uint64_t d0 = offs[w], n = offs[w + 1] - d0, s0 = (uint64_t)w * cap_w;
        for (uint64_t i = lane(); i < n; i += kWave) {
            const uint64_t s = s0 + i, d = d0 + i;
            line_end[d] = le_b[s];
            alt[d] = alt_b[s];
            tot[d] = tot_b[s];
            rowpre[d] = rowpre_b[s];
            status[d] = status_b[s];
            meta[d] = meta_b[s];
        }
        if (lane() == 0) g += wgt[w];
    }
    g = wave_sum(g);
    if (lane() == 0) red[threadIdx.x / kWave] = g;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < 256 / kWave; k++) t += red[k];
        if (t) {
            atomicAdd(&counters[0], (unsigned long long)t);
            atomicAdd(&counters[1], (unsigned long long)t);
        }
        if (blockIdx.x == 0) *n_lines = offs[n_walkers];
    }
}

int64_t af_walkers(int64_t lo, int64_t hi, int64_t chunk) { return hi > lo ? (hi - lo + chunk - 1) / chunk : 0; }

hipError_t launch_af_walk(const char *buf, int64_t lo, int64_t hi, int64_t chunk, int mode, int64_t span0,
                          uint64_t cap_w, uint64_t *le_b, int32_t *alt_b, int32_t *tot_b, uint32_t *rowpre_b,
                          uint8_t *status_b, void *meta_b, uint64_t *wcount, uint32_t *wgt, unsigned *overflow,
                          hipStream_t s) {
    const int64_t nw = af_walkers(lo, hi, chunk);
    if (!nw) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((nw + kWalkWaves - 1) / kWalkWaves);
    hipLaunchKernelGGL(k_af_walk, dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, mode, span0, cap_w,
                       le_b, alt_b, tot_b, rowpre_b, status_b, static_cast<LineMeta *>(meta_b), wcount, wgt, overflow);
    return hipGetLastError();
}

hipError_t launch_walk_compact(int64_t n_walkers, uint64_t cap_w, const uint64_t *offs, const uint32_t *wgt,
                               const uint64_t *le_b, const int32_t *alt_b, const int32_t *tot_b,
                               const uint32_t *rowpre_b, const uint8_t *status_b, const void *meta_b,
                               uint64_t *line_end, int32_t *alt, int32_t *tot, uint32_t *rowpre, uint8_t *status,
                               void *meta, uint64_t *n_lines, unsigned long long *counters, hipStream_t s) {
    const int64_t blocks = std::min<int64_t>((n_walkers + 3) / 4, 2048);
    hipLaunchKernelGGL(k_walk_compact, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s, n_walkers, cap_w,
                       offs, wgt, le_b, alt_b, tot_b, rowpre_b, status_b, static_cast<const LineMeta *>(meta_b),
                       line_end, alt, tot, rowpre, status, static_cast<LineMeta *>(meta), n_lines, counters);
    return hipGetLastError();
}

}  // namespace vcfxg
