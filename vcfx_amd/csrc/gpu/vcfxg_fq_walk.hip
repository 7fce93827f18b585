// vcfxg_fq_walk.hip -- VCFX_record_filter, VCFX_genotype_query and the fused
// `record_filter | genotype_query` pipeline (BASELINE config 3) without a separate line
// index: the walk of vcfxg_af_walk.hip (one wave per chunk walks the chunk's lines, a
// line's head analysed out of an LDS window fetched while the previous line was swept) with
// the per-line work of the two tools:
//
//   * record_filter (kRF): the walk stores each line's first 8 tab offsets (found in its head
//     window); k_fq_finish then runs evaluateLine (VCFX_record_filter.cpp:383-401, rf_eval in
//     vcfxg_rf.h) thread-per-line from them.  A line whose first 8 tabs are not inside the
//     1 KiB window gets status kRfPending and k_fq_finish finds its tabs itself.
//   * genotype_query (kGQ): checkAnySampleMatches (VCFX_genotype_query.cpp:322-345) on a
//     GT-first record as the fixed-stride sweep with the early exit at the first match
//     (gt_fast + GqOp, vcfxg_gt.h); everything else goes to k_gq_complex (kGqPending: the
//     general sweep of a GT-first record; kGqFull: gq_line, the whole per-line path).
//
// A GT-only record's end may be PREDICTED from the walker's previous fixed-stride record
// (as in the AF walk).  The prediction holds iff the byte at E is the '\n' (or E is the
// input end), the '\r' state matches, and no '\n' lies in [S, E): the sweep validates every
// byte it examines, and after an early exit (a match) the unswept rest is scanned for '\n'.
// A rejected prediction re-runs the line with the '\n' found by a scan.
//
// Final statuses (the same arrays vcfxg_index + vcfxg_record_filter / vcfxg_genotype_query /
// vcfxg_filter_query produce): RF 0 empty, 4 header, 1 kept, 2 dropped; GQ 1 match, 2 no
// match, 3 "<9 fields" warning, 4 header, 0 empty; the pipeline maps the GQ verdicts of the
// lines RF kept to 1 / 6 / 7 (gq_gated).  strip_cr: record_filter (and so the pipeline)
// strips a trailing '\r' (:454-456 / :509-511); genotype_query alone does not.
#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"
#include "vcfxg_rf.h"
#include "vcfxg_walk.h"

namespace vcfxg {

#ifndef VCFXG_FQ_UNROLL
#define VCFXG_FQ_UNROLL 6
#endif
constexpr int kFqUnroll = VCFXG_FQ_UNROLL;
// The filter does not run in the walk: the walk stores each data line's first 8 tab offsets
// (u16 from the line start, 0xFFFF past the last tab) and k_fq_finish evaluates rf_eval
// thread-per-line from them (the bytes through a 16-byte block cache per thread).  Evaluated
// in the walk itself, wave-uniformly, the filter's scalar code serialised every line behind
// it (and its state spilled the walk's SGPRs).
struct BlockBytes {  // byte source: the 16-byte aligned block of the last byte read (per lane)
    const char *__restrict__ buf;
    mutable int64_t base;
    mutable uint4 v;
    __device__ __forceinline__ uint32_t operator[](int64_t p) const {
        const int64_t b = p & ~(int64_t)15;
        if (b != base) {  // the input is padded, so the block is always readable
            v = *reinterpret_cast<const uint4 *>(buf + b);
            base = b;
        }
        const int o = (int)(p & 15), q = o >> 2;
        const uint32_t w = q == 0 ? v.x : (q == 1 ? v.y : (q == 2 ? v.z : v.w));
        return (w >> ((o & 3) * 8)) & 0xFFu;
    }
};
struct PoolBytes {
    const char *__restrict__ p;
    __device__ __forceinline__ uint32_t operator[](int64_t i) const { return (uint8_t)p[i]; }
};

// kNR (with kGQ, without kRF): VCFX_nonref_filter -- the same walk with NrOp ("some sample
// is not hom-ref", early exit) in place of the query; k_nr_complex takes the rest.
// kMD (with kGQ): VCFX_missing_detector -- MdOp ("some sample's GT has a '.' allele", early
// exit): status kMdFlag / 1 on the fixed-stride records; k_md_lines takes the rest
template <bool kRF, bool kGQ, bool kNR = false, bool kMD = false>
__global__ __launch_bounds__(kWalkThreads) void k_fq_walk(const char *__restrict__ buf, int64_t lo, int64_t hi,
                                                          int64_t chunk, int64_t n_walkers, int strip_cr,
                                                          int64_t span0, uint64_t cap_w, RfArgs rf, GqQuery Q,
                                                          uint64_t *__restrict__ le_o, uint8_t *__restrict__ status_o,
                                                          LineMeta *__restrict__ meta_o, uint4 *__restrict__ tabs_o,
                                                          uint64_t *__restrict__ wcount, unsigned *overflow) {
    __shared__ uint4 win[kWalkWaves][2][kWave];  // two window slots per wave (double buffer)
    const int wv = threadIdx.x / kWave;
    if (blockIdx.x == 0 && threadIdx.x == 0) wcount[n_walkers] = 0;  // the scan's last entry (no memset)
    const int64_t wk = uniform64((int64_t)walk_block() * kWalkWaves + wv);
    if (wk >= n_walkers) return;
    const int64_t cs = lo + wk * chunk;
    const int64_t ce = std::min<int64_t>(cs + chunk, hi);
    int64_t L, ce2;  // this walker's lines start in [L, ce2)
    walker_lines(buf, lo, hi, cs, ce, L, ce2, chunk);
    int64_t span = kGQ ? span0 : 0;  // predicted '\n' distance from the sample start
    uint8_t cr_prev = 0;             // and the '\r' state of that record
    uint64_t n = 0;
    const uint64_t base = (uint64_t)wk * cap_w;
    // per-line results held by lane (n & 63), written out 64 lines at a time
    uint64_t r_le = 0, r_S = 0;
    uint32_t r_k = 0;  // kind | sep << 8 | cr << 16 | status << 24
    uint32_t r_t[4] = {0, 0, 0, 0};  // kRF: tabs 0-7, u16 offsets from the line start
    auto flush = [&](uint64_t first, uint32_t cnt) {
        if ((uint32_t)lane() < cnt) {
            const uint64_t o = base + first + lane();
            le_o[o] = r_le;
            status_o[o] = (uint8_t)(r_k >> 24);
            if (kRF) tabs_o[o] = make_uint4(r_t[0], r_t[1], r_t[2], r_t[3]);
            if (kGQ) {
                LineMeta m{};
                m.kind = (uint8_t)r_k;
                m.cr = (uint8_t)(r_k >> 16);
                if (m.kind == kMetaGt) {
                    m.S = r_S;
                    m.sep = (uint8_t)(r_k >> 8);
                }
                meta_o[o] = m;
            }
        }
    };
    int cur = 0;
    int64_t A = L & ~(int64_t)15;  // window base of the current line (L - A < 16)
    if (L < ce2) prefetch_window(buf, A, hi, win[wv][cur]);
    while (L < ce2) {
        if (n >= cap_w) {
            if (lane() == 0) atomicOr(overflow, 1u);
            break;
        }
        // ---- 1. window analysis (offsets relative to A): the first '\n', the first 9 tabs
        const int Lr = (int)(L - A);
        const uint4 *cw = win[wv][cur];
        int hr, N1r, rt[9] = {};
        uint32_t ntab, first;
        // the kWin window, four bytes per lane (vcfxg_walk.h first_tabs; the lane's dword stays
        // in w4 for the byte reads below)
        uint32_t w4 = 0;
        bool long_head = false;
        {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            w4 = reinterpret_cast<const uint32_t *>(cw)[lane()];
            hr = (int)std::min<int64_t>(hi - A, kWin);
            const uint32_t rg = range4(Lr, hr);
            N1r = first_match<4>(zero_bytes(w4 ^ kRepNl) & rg);
            ntab = first_tabs<4>(zero_bytes(w4 ^ kRepTab) & rg, N1r >= 0 ? N1r : hr, rt);
            first = dword_byte(w4, Lr);
        }
        if (N1r < 0 && ntab < 9 && first != '#' && hr == kWin) {  // (rare) a long head: the 1 KiB window
            prefetch_window(buf, A, hi, win[wv][cur], kWaveStep);
            long_head = true;
            const uint4 W = read_window(cw);
            const int b = 16 * lane();
            hr = (int)std::min<int64_t>(hi - A, kWaveStep);
            N1r = first_match<16>(eq_mask16(W, kRepNl) & range16(b, Lr, hr));
            ntab = first_tabs<16>(eq_mask16(W, kRepTab) & range16(b, Lr, hr), N1r >= 0 ? N1r : hr, rt);
        }
        // window byte o (wave-uniform, < hr)
        auto wbyte = [&](int o) { return long_head ? slot_byte(cw, o) : dword_byte(w4, o); };
        const int64_t wend = A + hr;
        const int64_t t8 = ntab >= 9 ? A + rt[8] : -1;
        bool gt_head = false, gt_only = false;
        if (ntab >= 9 && first != '#') {
            const int r7 = rt[7], r8 = rt[8];
            if (r8 - r7 >= 3 && wbyte(r7 + 1) == 'G' && wbyte(r7 + 2) == 'T') {
                gt_only = r8 - r7 == 3;
                gt_head = gt_only || wbyte(r7 + 3) == ':';
            }
        }
        // fields 0-7 inside the window: the whole line, or its first 8 tabs (and criteria and
        // pool small enough for the registers)
        const bool rf_here = N1r >= 0 || ntab >= 8;
        // ---- 2. line end (and its '\r' when stripped)
        int64_t E;
        uint8_t cr = 0;
        bool predicted = false;
        if (N1r >= 0) {
            E = A + N1r;
            cr = strip_cr && E > L && wbyte(N1r - 1) == '\r';
        } else if (kGQ && gt_only && span > 0 && t8 + 1 + span <= hi) {
            E = t8 + 1 + span;  // checked after the sweep (its end bytes come with the next window)
            cr = cr_prev;
            predicted = true;
        } else {
            E = scan_nl(buf, wend, hi);
            cr = strip_cr && E > L && __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r';
        }
        const uint32_t sep_w = gt_head && t8 + 2 < wend ? wbyte((int)(t8 + 2 - A)) : 0u;
        // ---- 3. kind and the query sweep; the next
        // window's prefetch is issued right after the sweep's first loads
        const int nxt = cur ^ 1;
        int64_t An = std::max<int64_t>(E - 1, 0) & ~(int64_t)15;
        bool pending = true;  // pre() still to run
        uint8_t kind = 0, sep = 0;
        int64_t ae = E - cr, S = 0, swept = 0;
        auto pre = [&]() {
            prefetch_window(buf, An, hi, win[wv][nxt]);
            pending = false;
        };
        bool ok = false, found = false;
        auto sweep = [&]() {
            ae = E - cr;
            if (ae <= L) kind = kMetaEmpty;
            else if (first == '#') kind = kMetaHeader;
            else if (gt_head && t8 < ae) kind = kMetaGt;
            else kind = kMetaFull;
            ok = found = false;
            swept = ae;
            if (kGQ && kind == kMetaGt) {
                S = t8 + 1;
                sep = t8 + 2 >= ae ? 0
                      : t8 + 2 < wend ? (uint8_t)sep_w
                                      : (uint8_t)__builtin_amdgcn_readfirstlane(byte_at(buf, t8 + 2));
                if constexpr (kMD) {
                    MdOp op{};
                    ok = gt_fast<kFqUnroll>(buf, S, ae, op, sep, pre, &swept);
                    found = op.found;
                } else if constexpr (kNR) {
                    NrOp op{buf, ae, 0, strip_cr ? 0 : 1};
                    ok = gt_fast<kFqUnroll>(buf, S, ae, op, sep, pre, &swept);
                    found = op.found;
                } else {
                    GqOp op{buf, ae, 0, Q};
                    ok = gt_fast<kFqUnroll>(buf, S, ae, op, sep, pre, &swept);
                    found = op.found;
                }
            }
            if (pending) pre();
        };
        sweep();
        if (predicted) {
            const uint4 *nw = win[wv][nxt];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t be = slot_byte(nw, (int)(E - An)), be1 = slot_byte(nw, (int)(E - 1 - An));
            const bool endok = (E < hi ? be == '\n' : true) && ((strip_cr && be1 == '\r') == (cr != 0));
            // after an early exit the bytes past the sweep hold no '\n' only once scanned
            const bool good = ok && endok && (swept >= ae || nl_free(buf, swept, E));
            if (!good) {
                const int64_t Et = scan_nl(buf, wend, hi);
                if (Et != E || !endok) {  // the line again with its true bounds
                    E = Et;
                    cr = strip_cr && E > L && __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r';
                    An = std::max<int64_t>(E - 1, 0) & ~(int64_t)15;
                    pending = true;
                    sweep();
                }
                // else: true bounds, not fixed-stride
            }
        }
        if (kGQ && kind == kMetaGt && ok) {  // the next prediction
            span = E - S;
            cr_prev = cr;
        }
        // ---- 4. status
        uint8_t st;
        if (kind == kMetaEmpty) st = 0;
        else if (kind == kMetaHeader) st = 4;
        else if (kRF && !rf_here) {
            st = kRfPending;  // k_fq_finish evaluates the filter (then k_gq_complex the query)
            kind = kMetaFull;
        } else if (!kGQ) st = 1;  // (k_fq_finish drops the lines the filter rejects)
        else if (kind == kMetaGt && ok) st = kMD ? (found ? kMdFlag : 1) : found ? 1 : (kRF ? 6 : 2);
        else st = kind == kMetaGt ? kGqPending : kGqFull;
        if ((uint32_t)lane() == (uint32_t)(n & 63)) {
            r_le = (uint64_t)E;
            r_S = (uint64_t)S;
            r_k = (uint32_t)kind | ((uint32_t)sep << 8) | ((uint32_t)cr << 16) | ((uint32_t)st << 24);
            if (kRF) {
                const int Lr = (int)(L - A);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t a0 = (uint32_t)(2 * k) < ntab ? (uint32_t)(rt[2 * k] - Lr) : 0xFFFFu;
                    const uint32_t a1 = (uint32_t)(2 * k + 1) < ntab ? (uint32_t)(rt[2 * k + 1] - Lr) : 0xFFFFu;
                    r_t[k] = a0 | a1 << 16;
                }
            }
        }
        n++;
        if ((n & 63) == 0) flush(n - 64, 64);
        L = E + 1;
        A = An;
        cur = nxt;
    }
    if (n & 63) flush(n & ~(uint64_t)63, (uint32_t)(n & 63));
    if (lane() == 0) wcount[wk] = n;
}

// walker regions -> dense per-line arrays in file order (offs = exclusive scan of wcount),
// one wave per walker region
template <bool kMeta, bool kTabs>
__global__ __launch_bounds__(256) void k_fq_compact(int64_t n_walkers, uint64_t cap_w, const uint64_t *__restrict__ offs,
                                                    const uint64_t *__restrict__ le_b,
                                                    const uint8_t *__restrict__ status_b,
                                                    const LineMeta *__restrict__ meta_b,
                                                    const uint4 *__restrict__ tabs_b, uint64_t *line_end,
                                                    uint8_t *status, LineMeta *meta, uint4 *tabs, uint64_t *n_lines) {
    const int64_t w = (int64_t)blockIdx.x * (256 / kWave) + threadIdx.x / kWave;  // one wave per walker
    if (w < n_walkers) {
        const uint64_t d0 = offs[w], cnt = offs[w + 1] - d0, s0 = (uint64_t)w * cap_w;
        for (uint64_t i = lane(); i < cnt; i += kWave) {
            const uint64_t sl = s0 + i, d = d0 + i;
            line_end[d] = le_b[sl];
            status[d] = status_b[sl];
            if (kMeta) meta[d] = meta_b[sl];
            if (kTabs) tabs[d] = tabs_b[sl];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *n_lines = offs[n_walkers];
}

// per dense line: the filter (from the tabs the walk stored, or with its own tab scan for the
// lines whose head outgrew the window: kRfPending), then the counters the tools report --
// record_filter: kept, data lines; genotype_query: the GT-first lines it matched and examined
// (k_gq_complex adds the ones it takes)
template <bool kRF, bool kGQ>
#ifdef VCFXG_FIN_WAVES  // (A/B knob: a minimum occupancy for the latency-bound filter pass)
__attribute__((amdgpu_waves_per_eu(VCFXG_FIN_WAVES, 8)))
#endif
__global__ __launch_bounds__(256) void k_fq_finish(const char *__restrict__ buf, int64_t data_start,
                                                   const uint64_t *__restrict__ line_end, const uint64_t *n_lines_p,
                                                   RfArgs rf, uint8_t *__restrict__ status, LineMeta *__restrict__ meta,
                                                   const uint4 *__restrict__ tabs, unsigned long long *rf_cnt,
                                                   unsigned long long *gq_cnt) {
    __shared__ uint32_t red[4][256 / kWave];
    const uint64_t n = *n_lines_p;
    uint32_t c[4] = {0, 0, 0, 0};  // rf kept, rf data lines, gq matched, gq data lines
    for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < n; li += gridDim.x * (uint64_t)blockDim.x) {
        uint8_t st = status[li];
        if (kRF && st != 0 && st != 4) {  // a data line: its 8 tabs stored by the walk, or
            // (kRfPending: a head longer than the walk's window) found here
            const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
            int64_t ae = (int64_t)line_end[li];
            const BlockBytes B{buf, -1, {}};
            int64_t t[8];
            int nt = 0;
            if (st == kRfPending) {
                if (ae > ls && B[ae - 1] == '\r') ae--;
#pragma unroll
                for (int k = 0; k < 8; k++) t[k] = 0;
                for (int64_t p = ls; p < ae && nt < 8; p++)
                    if (B[p] == '\t') {  // (register selects: no scratch array)
#pragma unroll
                        for (int k = 0; k < 8; k++) t[k] = k == nt ? p : t[k];
                        nt++;
                    }
            } else {
                const uint4 tv = tabs[li];
                const uint32_t tw[4] = {tv.x, tv.y, tv.z, tv.w};
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t o = (tw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                    t[k] = ls + o;
                    nt += o != 0xFFFFu;
                }
                // the line end only bounds a field past the last tab (fewer than 8 tabs)
                if (nt < 8 && ae > ls && B[ae - 1] == '\r') ae--;
            }
            const bool keep = rf_eval(B, t, nt, ls, ae, rf.crit, rf.ncrit, rf.and_logic, PoolBytes{rf.pool});
            const uint8_t st0 = st;
            if (!keep) {
                st = 2;
                if (kGQ) meta[li].kind = kMetaGated;
            } else if (st == kRfPending) st = kGQ ? kGqFull : 1;
            if (st != st0) status[li] = st;
        }
        if (kRF) {
            c[0] += st != 0 && st != 4 && st != 2;
            c[1] += st != 0 && st != 4;
        }
        if (kGQ) {
            const uint8_t kind = meta[li].kind;
            c[2] += kind == kMetaGt && st == 1;
            c[3] += kind == kMetaGt;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t s = wave_sum(c[k]);
        if (lane() == 0) red[k][threadIdx.x / kWave] = s;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        uint32_t t = 0;
        for (int w = 0; w < 256 / kWave; w++) t += red[threadIdx.x][w];
        unsigned long long *dst = threadIdx.x < 2 ? (kRF ? rf_cnt + threadIdx.x : nullptr)
                                                  : (kGQ ? gq_cnt + (threadIdx.x - 2) : nullptr);
        if (t && dst) atomicAdd(dst, (unsigned long long)t);
    }
}

template <bool kRF, bool kGQ, bool kNR = false, bool kMD = false>
static hipError_t fq_walk_launch(const char *buf, int64_t lo, int64_t hi, int64_t chunk, int strip_cr, int64_t span0,
                                 uint64_t cap_w, const RfArgs &rf, const GqQuery &Q, uint64_t *le_b,
                                 uint8_t *status_b, LineMeta *meta_b, uint4 *tabs_b, uint64_t *wcount,
                                 unsigned *overflow, hipStream_t s) {
    const int64_t nw = af_walkers(lo, hi, chunk);
    const unsigned grid = (unsigned)((nw + kWalkWaves - 1) / kWalkWaves);
    hipLaunchKernelGGL((k_fq_walk<kRF, kGQ, kNR, kMD>), dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, strip_cr,
                       span0, cap_w, rf, Q, le_b, status_b, meta_b, tabs_b, wcount, overflow);
    return hipGetLastError();
}

hipError_t launch_fq_walk(int what, const char *buf, int64_t lo, int64_t hi, int64_t chunk, int strip_cr,
                          int64_t span0, uint64_t cap_w, const RfArgs &rf, const char *q_dev, int qlen, int strict,
                          int qa, int qb, uint64_t *le_b, uint8_t *status_b, void *meta_b, void *tabs_b,
                          uint64_t *wcount, unsigned *overflow, hipStream_t s) {
    if (!af_walkers(lo, hi, chunk)) return hipErrorInvalidValue;
    const GqQuery Q{q_dev, qlen, strict, qa, qb};
    LineMeta *m = static_cast<LineMeta *>(meta_b);
    uint4 *t = static_cast<uint4 *>(tabs_b);
    if (what == kFqRF)
        return fq_walk_launch<true, false>(buf, lo, hi, chunk, strip_cr, span0, cap_w, rf, Q, le_b, status_b, m, t,
                                           wcount, overflow, s);
    if (what == kFqGQ)
        return fq_walk_launch<false, true>(buf, lo, hi, chunk, strip_cr, span0, cap_w, rf, Q, le_b, status_b, m, t,
                                           wcount, overflow, s);
    if (what == kFqNR)
        return fq_walk_launch<false, true, true>(buf, lo, hi, chunk, strip_cr, span0, cap_w, rf, Q, le_b, status_b, m,
                                                 t, wcount, overflow, s);
    if (what == kFqMD)
        return fq_walk_launch<false, true, false, true>(buf, lo, hi, chunk, strip_cr, span0, cap_w, rf, Q, le_b,
                                                        status_b, m, t, wcount, overflow, s);
    return fq_walk_launch<true, true>(buf, lo, hi, chunk, strip_cr, span0, cap_w, rf, Q, le_b, status_b, m, t, wcount,
                                      overflow, s);
}

hipError_t launch_fq_compact(int what, int64_t n_walkers, uint64_t cap_w, const uint64_t *offs, const uint64_t *le_b,
                             const uint8_t *status_b, const void *meta_b, const void *tabs_b, uint64_t *line_end,
                             uint8_t *status, void *meta, void *tabs, uint64_t *n_lines, hipStream_t s) {
    const int64_t blocks = std::max<int64_t>((n_walkers + 256 / kWave - 1) / (256 / kWave), 1);
    const LineMeta *mb = static_cast<const LineMeta *>(meta_b);
    LineMeta *m = static_cast<LineMeta *>(meta);
    const uint4 *tb = static_cast<const uint4 *>(tabs_b);
    uint4 *t = static_cast<uint4 *>(tabs);
    if (what == kFqRF)
        hipLaunchKernelGGL((k_fq_compact<false, true>), dim3((unsigned)blocks), dim3(256), 0, s, n_walkers, cap_w, offs,
                           le_b, status_b, mb, tb, line_end, status, m, t, n_lines);
    else if (what == kFqGQ || what == kFqNR || what == kFqMD)
        hipLaunchKernelGGL((k_fq_compact<true, false>), dim3((unsigned)blocks), dim3(256), 0, s, n_walkers, cap_w, offs,
                           le_b, status_b, mb, tb, line_end, status, m, t, n_lines);
    else
        hipLaunchKernelGGL((k_fq_compact<true, true>), dim3((unsigned)blocks), dim3(256), 0, s, n_walkers, cap_w, offs,
                           le_b, status_b, mb, tb, line_end, status, m, t, n_lines);
    return hipGetLastError();
}

// the call's counters, line count and overflow flag into mapped host memory (out[0..7],
// out[8], out[9]), each zeroed once read: the next call needs no memset or copy
__global__ void k_fq_done(unsigned long long *cnt, const uint64_t *n_lines, uint64_t *ovf, uint64_t *out) {
    const int t = threadIdx.x;
    if (t < 8) {
        out[t] = cnt[t];
        cnt[t] = 0;
    } else if (t == 8) {
        out[8] = *n_lines;
    } else if (t == 9) {
        out[9] = *ovf;
        *ovf = 0;
    }
}
hipError_t launch_fq_done(unsigned long long *cnt, const uint64_t *n_lines, uint64_t *ovf, uint64_t *out,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_fq_done, dim3(1), dim3(64), 0, s, cnt, n_lines, ovf, out);
    return hipGetLastError();
}

hipError_t launch_fq_finish(int what, const char *buf, int64_t data_start, const uint64_t *line_end,
                            const uint64_t *n_lines_dev, uint64_t n_lines_host, const RfArgs &rf, uint8_t *status,
                            void *meta, const void *tabs, unsigned long long *rf_cnt, unsigned long long *gq_cnt,
                            hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    // up to one line per thread: the filter is a latency chain (line end, tabs, field bytes),
    // so lines get their own threads rather than grid-stride shares; the kernel still grid-
    // strides past 65535 * 256 lines (the loop keeps it correct at any count).  n_lines_host
    // is the caller's line capacity, an upper bound of the count the kernel reads on the device
    const unsigned grid = (unsigned)std::min<uint64_t>((n_lines_host + 255) / 256, 65535);
    LineMeta *m = static_cast<LineMeta *>(meta);
    const uint4 *t = static_cast<const uint4 *>(tabs);
    if (what == kFqRF)
        hipLaunchKernelGGL((k_fq_finish<true, false>), dim3(grid), dim3(256), 0, s, buf, data_start, line_end,
                           n_lines_dev, rf, status, m, t, rf_cnt, gq_cnt);
    else if (what == kFqGQ)
        hipLaunchKernelGGL((k_fq_finish<false, true>), dim3(grid), dim3(256), 0, s, buf, data_start, line_end,
                           n_lines_dev, rf, status, m, t, rf_cnt, gq_cnt);
    else
        hipLaunchKernelGGL((k_fq_finish<true, true>), dim3(grid), dim3(256), 0, s, buf, data_start, line_end,
                           n_lines_dev, rf, status, m, t, rf_cnt, gq_cnt);
    return hipGetLastError();
}

}  // namespace vcfxg
