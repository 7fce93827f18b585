// vcfxg_af_walk.hip -- VCFX_allele_freq_calc's record pass without a separate line index.
//
// The data region is cut into C-byte chunks, one wave ("walker") each.  A walker's lines are
// those starting in [b(chunk start), b(chunk end)), b(x) the byte after the last '\n' before x
// (vcfxg_walk.h walker_lines: two short backward scans; the line across a chunk boundary goes
// to the walker after it, which reads it first).  It walks its lines one after the other:
//
//   1. one kWin (256 B) window at the line start (4 B per lane, LDS-DMA'd during the previous
//      line's sweep) gives the first '\n' if the line is short, the first 9 tabs and the
//      FORMAT bytes (SWAR masks, one ballot, then scalar code over the matching lanes; a head
//      longer than the window gets a 1 KiB one);
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
// So every input byte is read from HBM about once (the backward scans' bytes are the next
// walker's first line, read right after them), against twice for the separate index sweep.  k_walk_compact concatenates the regions in file order and
// k_af_complex runs the exact per-line path for everything that is not a fixed-stride
// GT-first record (kMetaFull lines, kAfPending lines), exactly as after the two-sweep
// schedule.  A walker over its line capacity raises `overflow` and the caller reruns the
// two-sweep schedule.  Head semantics follow vcfxg_meta.h head_meta (processMmap :355-470 /
// processStdin :490-556): '\r' stripped in file mode, '#' lines, empty lines, GT-first
// FORMAT, row prefix = CHROM..ALT and its tab.
#include <algorithm>
#include <type_traits>

#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"
#include "vcfxg_walk.h"

namespace vcfxg {

#ifndef VCFXG_WALK_UNROLL
#define VCFXG_WALK_UNROLL 6
#endif
constexpr int kWalkUnroll = VCFXG_WALK_UNROLL;  // wave-steps (KiB) of a record in flight per sweep step
// the HWE walk's sweep: 5 wave-steps (its clean-step genotype classes need the registers of the
// sixth under the 96-VGPR bound; at 6 the record loop spilled)
#ifndef VCFXG_HWE_UNROLL
#define VCFXG_HWE_UNROLL 5
#endif
constexpr int kHweUnroll = VCFXG_HWE_UNROLL;
// the GT-first walk's allele counts on per-byte flags (gt_first_af) rather than gt_first's loop
// over each lane's sample starts (VCFXG_GF_FLAGS=0: the loop, for A/B)
#ifndef VCFXG_GF_FLAGS
#define VCFXG_GF_FLAGS 1
#endif
constexpr bool kGfFlags = VCFXG_GF_FLAGS != 0;
// wave-steps in flight in the GT-first walk's sweeps (its flags take more registers per step)
#ifndef VCFXG_GF_UNROLL
#define VCFXG_GF_UNROLL 4
#endif
constexpr int kGfUnroll = VCFXG_GF_UNROLL;
// VCFXG_AF_XREC=1: the GT-only AF walk carries the next record's first wave-steps across
// records (af_fixed_x).  Measured slower (r04 A/B: af_walk 1.010-1.016 ms at 6 steps, 1.001 at
// 3, against 0.896-0.904 for the default, 112 VGPRs / occupancy 4 against 95 / 5): the
// per-record gap it hides is smaller than the occupancy it costs.  Default 0: each record's
// sweep issues its own first loads after its head's analysis
#ifndef VCFXG_AF_XREC
#define VCFXG_AF_XREC 0
#endif
// VCFXG_AF_EXPT (diagnostic builds only, rows invalid): bit 0 skips the rows' staging, bit 1
// only their frequency text
#ifndef VCFXG_AF_EXPT
#define VCFXG_AF_EXPT 0
#endif
// VCFXG_AF_EARLY=1: the GT-only AF walk issues a record's first sweep batch from its line start
// (16-aligned) before analysing its head, so the batch's latency overlaps the analysis (the
// head bytes ride along and are masked like the bytes before S)
#ifndef VCFXG_AF_EARLY
#define VCFXG_AF_EARLY 0
#endif
#define VCFXG_STR2(x) #x
#define VCFXG_STR(x) VCFXG_STR2(x)

// the walk's per-record reducer: AF allele counts (alt, total) or, for VCFX_hwe_tester, the
// genotype classes (hom-ref, het, hom-alt; the third in aux_o)
template <class Op>
struct WalkRed;
template <>
struct WalkRed<AfOp> {
    static constexpr bool kAux = false;
    __device__ static AfOp make(const char *buf, int64_t ae) { return AfOp{buf, ae, 0}; }
    __device__ static void out(const AfOp &op, uint32_t &a, uint32_t &b, uint32_t &) {
        a = op.alt;
        b = op.tot;
    }
};
template <>
struct WalkRed<HweOp> {
    static constexpr bool kAux = true;
    __device__ static HweOp make(const char *buf, int64_t ae) { return HweOp{buf, ae}; }
    __device__ static void out(const HweOp &op, uint32_t &a, uint32_t &b, uint32_t &c) {
        a = op.c0;
        b = op.c1;
        c = op.c2;
    }
};

template <>
struct WalkRed<DoseWalkOp> {  // samples and "NA" samples of the record (alt_o / tot_o)
    static constexpr bool kAux = false;
    __device__ static DoseWalkOp make(const char *buf, int64_t ae) { return DoseWalkOp{buf, ae}; }
    __device__ static void out(const DoseWalkOp &op, uint32_t &a, uint32_t &b, uint32_t &) {
        a = op.ns;
        b = op.na;
    }
};

template <>
struct WalkRed<DoseHeadOp> : WalkRed<DoseWalkOp> {
    __device__ static DoseHeadOp make(const char *buf, int64_t ae) { return DoseHeadOp{{buf, ae}}; }
};

// kGF: the GT-first walk (records "GT:AD:DP"-like, no fixed stride to predict): a GT-first
// record whose '\n' is past the window is swept by gt_first from its sample start, which finds
// the record's end in the same pass (and issues the next window as soon as it does); a separate
// instantiation, so the GT-only walk keeps its registers
template <class Op, bool kGF = false>
__global__ __launch_bounds__(kWalkThreads)
#ifdef VCFXG_WALK_MAXW
__attribute__((amdgpu_waves_per_eu(1, VCFXG_WALK_MAXW)))
#else
// the GT-first walk at <= 128 VGPRs (4 waves per SIMD; it needs 129 unconstrained, which
// rounds to 136 and 3 waves); the others at <= 96 (5 waves: the HWE walk took 100 without
// the bound, 4 waves; no spills at 96)
#ifndef VCFXG_AF_MINW
#define VCFXG_AF_MINW 5
#endif
__attribute__((amdgpu_waves_per_eu(kGF ? 4 : VCFXG_AF_MINW)))
#endif
void k_af_walk(const char *__restrict__ buf, int64_t lo, int64_t hi, int64_t chunk, int64_t n_walkers, int mode,
               int64_t span0, uint64_t cap_w, uint64_t *__restrict__ le_o, int32_t *__restrict__ alt_o,
               int32_t *__restrict__ tot_o, int32_t *__restrict__ aux_o, uint32_t *__restrict__ rowpre_o,
               uint8_t *__restrict__ status_o, LineMeta *__restrict__ meta_o, uint64_t *__restrict__ wcount,
               uint32_t *__restrict__ wgt, unsigned *overflow, WalkTail tail) {
    typedef WalkRed<Op> R;
    __shared__ uint4 win[kWalkWaves][2][kWave];  // two window slots per wave (double buffer)
    // (AfOp) each walker's rows composed in LDS and copied to its global stage once, at the end:
    // stored per record, their completion held up the next record's window wait (r05 ablation:
    // af_walk 0.889 -> 0.839 ms without the per-record stores)
    constexpr bool kStageLds = std::is_same<Op, AfOp>::value;
    constexpr uint32_t kStgCap = kStageLds ? 2048u : 16u;
    __shared__ __attribute__((aligned(16))) char stg[kStageLds ? kWalkWaves : 1][kStgCap];
    const int wv = threadIdx.x / kWave;
    const int64_t wk = uniform64((int64_t)walk_block() * kWalkWaves + wv);
    if (wk >= n_walkers) return;
    const int strip_cr = mode == 0 ? 1 : 0;
    const int64_t cs = lo + wk * chunk;
    const int64_t ce = std::min<int64_t>(cs + chunk, hi);
    int64_t L, ce2;  // this walker's lines start in [L, ce2)
    walker_lines(buf, lo, hi, cs, ce, L, ce2, chunk);
    const int64_t L0 = L;
    uint64_t wtext = 0;  // region tail (tail.wtext): bytes of this walker's GT-line rows
    int64_t span = span0;  // predicted '\n' distance from the sample start
    uint8_t cr_prev = 0;   // and the '\r' state of that record
    uint64_t n = 0;
    uint32_t ngt = 0, ngf = 0;  // GT-first lines; of them, swept whole by gt_first (kGF)
    bool dirty = false;         // AfOp staged rows: some row of this walker is not in its stage
    const uint64_t base = (uint64_t)wk * cap_w;
    // per-line results held by lane (n & 63), written out 64 lines at a time (no stores --
    // and no waits for their completion -- on the per-record path)
    uint64_t r_le = 0, r_S = 0;
    uint32_t r_alt = 0, r_tot = 0, r_aux = 0, r_pre = 0, r_k = 0;  // r_k: kind | sep << 8 | cr << 16 | status << 24
    uint32_t r_h = 0;  // HWE: the CHROM..ALT flags (LineMeta::pad)
    auto flush = [&](uint64_t first, uint32_t cnt) {
        if ((uint32_t)lane() < cnt) {
            const uint64_t o = base + first + lane();
            const uint8_t kind = (uint8_t)r_k;
            LineMeta m{};
            m.kind = kind;
            m.cr = (uint8_t)(r_k >> 16);
            m.pad = (R::kAux || std::is_same<Op, DoseHeadOp>::value) ? (uint8_t)r_h : 0;
            if (kind == kMetaGt) {
                m.S = r_S;
                m.rowpre = r_pre;
                m.sep = (uint8_t)(r_k >> 8);
            }
            le_o[o] = r_le;
            alt_o[o] = (int32_t)r_alt;
            tot_o[o] = (int32_t)r_tot;
            if (R::kAux) aux_o[o] = (int32_t)r_aux;
            rowpre_o[o] = kind == kMetaGt ? r_pre : 0u;
            status_o[o] = (uint8_t)(r_k >> 24);
            meta_o[o] = m;
        }
    };
    // (AfOp, GT-only walk) the next record's first wave-steps, issued during this record's sweep
    constexpr bool kXrec = VCFXG_AF_XREC && std::is_same<Op, AfOp>::value && !kGF;
    uint4 xv[kXrec ? kWalkUnroll : 1];
    int64_t xvb = -1;  // their base (-1: none)
    int cur = 0;
    int64_t A = L & ~(int64_t)15;  // window base of the current line (L - A < 32)
    if (L < ce2) prefetch_window(buf, A, hi, win[wv][cur]);
    constexpr bool kEarly = VCFXG_AF_EARLY && std::is_same<Op, AfOp>::value && !kGF && !kXrec;
    uint4 ev[kEarly ? kWalkUnroll : 1];
    const int64_t hlast = (hi - 1) & ~(int64_t)15;
    while (L < ce2) {
        if (n >= cap_w) {
            if (lane() == 0) atomicOr(overflow, 1u);
            break;
        }
        if constexpr (kEarly) {  // the first batch from the line start (= the window base A)
#pragma unroll
            for (int u = 0; u < kWalkUnroll; u++) {
                const int64_t g = A + u * kWaveStep + kBlockBytes * lane();
                ev[u] = load16(buf, g < hi ? g : hlast);
            }
        }
        int64_t eA = kEarly ? A : -1;  // the early batch's base (-1: used or none)
        // ---- 1. window analysis (offsets relative to A); a head that does not fit the short
        // window (no '\n' and fewer than 9 tabs in it) gets the 1 KiB window
        const int Lr = (int)(L - A);
        const uint4 *cw = win[wv][cur];
        int hr, N1r, r4 = 0, r7 = 0, r8 = 0;
        uint32_t ntab, first, hflags = 0;
        // the tab positions -> r4, r7, r8 (and HWE's row rules on CHROM..ALT,
        // VCFX_hwe_tester.cpp:497-506: an ALT with a comma, an empty CHROM / POS / ALT)
        auto take = [&](const int(&rt)[9], bool comma) {
            r4 = rt[4];
            r7 = rt[7];
            r8 = rt[8];
            if (R::kAux) {
                const bool empty = rt[0] == Lr || rt[1] == rt[0] + 1 || r4 == rt[3] + 1;
                hflags = (comma ? kHweAltComma : 0u) | (empty ? kHweEmptyField : 0u);
            }
        };
        // the kWin window, four bytes per lane (the lane's dword stays in w4 for the byte reads
        // below: a v_readlane each instead of an LDS round trip)
        uint32_t w4 = 0;
        bool long_head = false;
        {
            // the window's LDS-DMA landed (kEarly: all but the early batch, issued after it)
            if constexpr (kEarly) asm volatile("s_waitcnt vmcnt(" VCFXG_STR(VCFXG_WALK_UNROLL) ")" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            w4 = reinterpret_cast<const uint32_t *>(cw)[lane()];
            hr = (int)std::min<int64_t>(hi - A, kWin);
            const uint32_t rg = range4(Lr, hr);
            N1r = first_match<4>(zero_bytes(w4 ^ kRepNl) & rg);
            int rt[9] = {};
            ntab = first_tabs<4>(zero_bytes(w4 ^ kRepTab) & rg, N1r >= 0 ? N1r : hr, rt);
            first = dword_byte(w4, Lr);
            if (ntab >= 9) take(rt, R::kAux && __ballot((zero_bytes(w4 ^ 0x2C2C2C2Cu) & range4(rt[3] + 1, rt[4])) != 0u));
        }
        if (N1r < 0 && ntab < 9 && first != '#' && hr == kWin) {  // (rare) a long head: the 1 KiB window
            prefetch_window(buf, A, hi, win[wv][cur], kWaveStep);
            long_head = true;
            const uint4 W = read_window(cw);
            const int b = 16 * lane();
            hr = (int)std::min<int64_t>(hi - A, kWaveStep);
            N1r = first_match<16>(eq_mask16(W, kRepNl) & range16(b, Lr, hr));
            int rt[9] = {};
            ntab = first_tabs<16>(eq_mask16(W, kRepTab) & range16(b, Lr, hr), N1r >= 0 ? N1r : hr, rt);
            if (ntab >= 9) take(rt, R::kAux && __ballot((eq_mask16(W, 0x2C2C2C2Cu) & range16(b, rt[3] + 1, rt[4])) != 0u));
        }
        // window byte o (wave-uniform, < hr)
        auto wbyte = [&](int o) { return long_head ? slot_byte(cw, o) : dword_byte(w4, o); };
        const int64_t wend = A + hr;
        int64_t t4 = -1, t8 = -1;
        bool gt_head = false, gt_only = false;
        if (ntab >= 9 && first != '#') {
            t4 = A + r4;
            t8 = A + r8;
            if (r8 - r7 >= 3 && wbyte(r7 + 1) == 'G' && wbyte(r7 + 2) == 'T') {
                gt_only = r8 - r7 == 3;
                gt_head = gt_only || wbyte(r7 + 3) == ':';
            }
        }
        // ---- 2. line end (and its '\r' in file mode)
        int64_t E;
        uint8_t cr = 0;
        bool predicted = false;
        const bool gf = kGF && N1r < 0 && gt_head && !gt_only;  // the end comes with the sweep
        if (N1r >= 0) {
            E = A + N1r;
            cr = strip_cr && E > L && wbyte(N1r - 1) == '\r';
        } else if (gf) {
            E = hi;  // (until gt_first finds the '\n')
        } else if (gt_only && span > 0 && t8 + 1 + span <= hi) {
            // predicted from the previous fixed-stride record; its end bytes come with the
            // next window (which starts at E - 1) and are checked after the sweep
            E = t8 + 1 + span;
            cr = cr_prev;
            predicted = true;
        } else {
            E = scan_nl(buf, wend, hi);
            cr = strip_cr && E > L && __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r';
        }
        // every read of the current slot happens before the next prefetch is issued (an LDS
        // read after it would make the compiler wait for the LDS-DMA)
        const uint32_t sep_w = gt_head && t8 + 2 < wend ? wbyte((int)(t8 + 2 - A)) : 0u;
        // the next window (the next line's head, and bytes E - 1 and E): issued right after
        // the sweep's first loads (issued before them, the sweep loop's head wait would
        // hold its loads back until the window landed)
        const int nxt = cur ^ 1;
        int64_t An = std::max<int64_t>(E - 1, 0) & ~(int64_t)15;
        bool pending = true;  // the prefetch for An is still to be issued
        auto pre = [&]() {
            prefetch_window(buf, An, hi, win[wv][nxt]);
            pending = false;
        };
        // ---- 3. kind (head_meta) and the sweep
        uint8_t st = 0, kind = 0, sep = 0;
        uint32_t alt = 0, tot = 0, aux = 0, rowpre = 0;
        int64_t S = 0;
        bool ok = false;
        // DoseHeadOp: a predicted GT-only record is not swept (k_dose_fmt checks its bytes)
        bool skip = std::is_same<Op, DoseHeadOp>::value && predicted;
        // the carried wave-steps are this record's only if its sweep is the first af_fixed_x call
        // since they were issued (any other record or a re-sweep drops them)
        int64_t xuse = xvb;
        xvb = -1;
        auto sweep = [&]() {
            if constexpr (kGF) {
              if (gf) {  // gt_first from the sample start: the counts and the record end
                S = t8 + 1;
                Op op = R::make(buf, hi);
                int64_t Eo = hi;
                uint8_t cro = 0;
                auto pre_e = [&](int64_t e) {
                    An = std::max<int64_t>(e - 1, 0) & ~(int64_t)15;
                    pre();
                };
                if constexpr (std::is_same<Op, AfOp>::value && kGfFlags)
                    ok = gt_first_af<kGfUnroll>(buf, S, hi, strip_cr, op, pre_e, Eo, cro);
                else
                    ok = gt_first<kWalkUnroll>(buf, S, hi, strip_cr, op, pre_e, Eo, cro);
                E = Eo;
                cr = cro;
                const int64_t ae = E - cr;
                kind = t8 < ae ? kMetaGt : kMetaFull;
                ok = ok && kind == kMetaGt;
                if (kind == kMetaGt) {
                    rowpre = (uint32_t)(t4 - L + 1);
                    sep = t8 + 2 >= ae ? 0
                          : t8 + 2 < wend ? (uint8_t)sep_w
                                          : (uint8_t)__builtin_amdgcn_readfirstlane(byte_at(buf, t8 + 2));
                    R::out(op, alt, tot, aux);
                }
                return;
              }
            }
            const int64_t ae = E - cr;
            if (ae <= L) kind = kMetaEmpty;
            else if (first == '#') kind = kMetaHeader;
            else if (gt_head && t8 < ae) kind = kMetaGt;
            else kind = kMetaFull;
            ok = false;
            if (kind == kMetaGt) {
                S = t8 + 1;
                rowpre = (uint32_t)(t4 - L + 1);
                sep = t8 + 2 >= ae ? 0
                      : t8 + 2 < wend ? (uint8_t)sep_w
                                      : (uint8_t)__builtin_amdgcn_readfirstlane(byte_at(buf, t8 + 2));
                Op op = R::make(buf, ae);
                if constexpr (kXrec) {
                    const int64_t use = xuse >= 0 && xuse <= S ? xuse : -1;
                    xuse = -1;
                    const int64_t nb = E + 1 < ce2 ? (E + 1) & ~(int64_t)15 : -1;  // this walker's next line
                    int64_t vbo;
                    ok = af_fixed_x<kWalkUnroll>(buf, S, ae, hi, op, sep, pre, xv, use, nb, vbo);
                    xvb = vbo;
                } else if constexpr (kEarly) {
                    // the early batch is this sweep's first when it covers S's block (a re-sweep
                    // after a failed prediction loads its own)
                    const bool mine = eA >= 0 && eA <= S;
                    ok = af_fixed<kWalkUnroll>(buf, S, ae, op, sep, pre, mine ? ev : nullptr, mine ? eA : -1);
                    eA = -1;
                } else if constexpr (std::is_same<Op, AfOp>::value)
                    ok = af_fixed < kGF ? kGfUnroll : kWalkUnroll > (buf, S, ae, op, sep, pre);
                else if constexpr (std::is_same<Op, DoseHeadOp>::value) {
                    if (skip) {  // samples (ae - S + 1) / 4, none "NA" (checked by k_dose_fmt)
                        ok = (sep == '/' || sep == '|') && ae - S >= 3 && ((ae - S + 1) & 3) == 0;
                        op.ns = ok ? (uint32_t)((ae - S + 1) >> 2) : 0u;
                        op.na = 0;
                    } else {
                        ok = gt_fast<kWalkUnroll>(buf, S, ae, op, sep, pre);
                    }
                } else ok = gt_fast < std::is_same<Op, HweOp>::value ? kHweUnroll : kWalkUnroll > (buf, S, ae, op, sep, pre);
                R::out(op, alt, tot, aux);
            }
        };
        sweep();
        if (pending) pre();  // (no sweep ran)
        if (predicted) {
            // the prediction holds iff the sweep accepted every byte of [S, ae) and the end
            // bytes are the '\n' (or the input end) and the predicted '\r' state
            const uint4 *nw = win[wv][nxt];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t be = slot_byte(nw, (int)(E - An)), be1 = slot_byte(nw, (int)(E - 1 - An));
            const bool endok = (E < hi ? be == '\n' : true) && ((strip_cr && be1 == '\r') == (cr != 0));
            if (!(ok && endok)) {
                const int64_t Et = scan_nl(buf, wend, hi);
                if (Et != E || !endok) {  // the line again with its true bounds
                    skip = false;
                    E = Et;
                    cr = strip_cr && E > L && __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r';
                    An = std::max<int64_t>(E - 1, 0) & ~(int64_t)15;
                    pending = true;
                    sweep();
                    if (pending) pre();
                }
                // else: true bounds, not fixed-stride
            }
        }
        // DoseHeadOp: a record taken on its predicted end without a sweep (its interior bytes are
        // unread: the consumer checks them, k_dose_fmt / k_ph_lines)
        if constexpr (std::is_same<Op, DoseHeadOp>::value)
            if (skip && kind == kMetaGt) hflags |= kWalkUnswept;
        if (kind == kMetaGt) {
            if (ok) {
                st = 1;
                span = E - S;
                cr_prev = cr;
            } else {
                st = kAfPending;  // not fixed-stride: k_af_complex runs the general sweep
            }
        }
        // ---- 4. results into lane n & 63
        if ((uint32_t)lane() == (uint32_t)(n & 63)) {
            r_le = (uint64_t)E;
            r_S = (uint64_t)S;
            r_alt = alt;
            r_tot = tot;
            r_aux = aux;
            r_h = hflags;
            r_pre = rowpre;
            r_k = (uint32_t)kind | ((uint32_t)sep << 8) | ((uint32_t)cr << 16) | ((uint32_t)st << 24);
        }
        if constexpr (std::is_same<Op, AfOp>::value) {
            // the row's text into the walker's stage (lanes = bytes): CHROM..ALT and its tab from
            // the head window, which still holds the line (the next window went to the other slot),
            // then the frequency; a line left to k_af_cx (or a stage too small) marks the walker
            if (tail.stage && !(VCFXG_AF_EXPT & 1)) {
                if (kind == kMetaGt && ok && wtext + rowpre + 7u <= std::min<uint32_t>(tail.stage_cap, kStgCap)) {
                    uint32_t flo = 0x30303030u, fhi = 0x0A3030u;
                    if (!(VCFXG_AF_EXPT & 2)) af_freq_text(mode, (int32_t)alt, (int32_t)tot, flo, fhi);
                    auto *dst = reinterpret_cast<__attribute__((address_space(3))) char *>(
                                    reinterpret_cast<__attribute__((address_space(3))) char *>(
                                        (__attribute__((address_space(3))) void *)stg[kStageLds ? wv : 0])) +
                                wtext;
                    const unsigned char *src = reinterpret_cast<const unsigned char *>(cw) + (L - A);
                    for (uint32_t j0 = 0; j0 < rowpre + 7u; j0 += kWave) {
                        const uint32_t j = j0 + (uint32_t)lane();
                        if (j < rowpre) dst[j] = (char)src[j];
                        else if (j < rowpre + 7u) {
                            const uint32_t q = j - rowpre;
                            dst[j] = (char)((q < 4u ? flo >> (8u * q) : fhi >> (8u * (q - 4u))) & 0xFFu);
                        }
                    }
                } else if (kind == kMetaGt || kind == kMetaFull) {
                    dirty = true;
                }
            }
        }
        ngt += kind == kMetaGt ? 1u : 0u;
        if constexpr (kGF) ngf += gf && kind == kMetaGt && ok ? 1u : 0u;
        if (tail.wtext) {
            // the row (CHROM..ALT + "\t" + 4 digits... "x.xxxx\n") of a GT line; lines off the
            // fixed-stride sweep go to the leftover list (rare: one atomic each)
            if (kind == kMetaGt) wtext += (uint64_t)rowpre + 7u;
            if (kind == kMetaFull || (kind == kMetaGt && !ok)) {
                if (lane() == 0) {
                    const unsigned long long e = atomicAdd(tail.cx_n, 1ull);
                    if (e < tail.cx_cap) tail.cx_list[e] = base + n;
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
    if constexpr (kStageLds) {
        if (tail.stage && wtext) {  // the walker's rows to its global stage, 16 B stores
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t wt = (uint32_t)std::min<uint64_t>(wtext, kStgCap);
            char *gs = tail.stage + (uint64_t)wk * tail.stage_cap;
            for (uint32_t o = (uint32_t)lane() * 16u; o < wt; o += kWave * 16u)
                *reinterpret_cast<uint4 *>(gs + o) = *reinterpret_cast<const uint4 *>(stg[wv] + o);
        }
    }
    if (lane() == 0) {
        wcount[wk] = n;
        if (tail.wtext) {
            tail.wtext[wk] = wtext;
            tail.wstart[wk] = (uint64_t)L0;
        }
        wgt[wk] = ngt | (ngf << 16);
        if (tail.wdirty) tail.wdirty[wk] = dirty || n >= cap_w ? 1 : 0;
    }
}

// walker regions -> dense per-line arrays in file order (offs = exclusive scan of wcount):
// kCompactSub walker regions per wave at a time, one per group of 64 / kCompactSub lanes (r05: a
// region holds ~13 lines on the 10 KB-record shards, so one region per wave left 51 of 64 lanes
// idle through every round trip), so no slot division and no work for the unused slots; the
// rows / data-line counters (every GT-first record counts as both) are reduced per block (few
// blocks: few atomics)
#ifndef VCFXG_COMPACT_SUB
#define VCFXG_COMPACT_SUB 4
#endif
constexpr int kCompactSub = VCFXG_COMPACT_SUB, kCompactLanes = kWave / kCompactSub;
__global__ __launch_bounds__(256) void k_walk_compact(int64_t n_walkers, uint64_t cap_w,
                                                      const uint64_t *__restrict__ offs,
                                                      const uint32_t *__restrict__ wgt,
                                                      const uint64_t *__restrict__ le_b,
                                                      const int32_t *__restrict__ alt_b,
                                                      const int32_t *__restrict__ tot_b,
                                                      const int32_t *__restrict__ aux_b,
                                                      const uint32_t *__restrict__ rowpre_b,
                                                      const uint8_t *__restrict__ status_b,
                                                      const LineMeta *__restrict__ meta_b, uint64_t *line_end,
                                                      int32_t *alt, int32_t *tot, int32_t *aux, uint32_t *rowpre,
                                                      uint8_t *status, LineMeta *meta, uint64_t *n_lines,
                                                      unsigned long long *counters, const uint64_t *__restrict__ bpre) {
    __shared__ uint32_t red[256 / kWave];
    uint32_t g = 0;
    const int64_t nwaves = (int64_t)gridDim.x * (256 / kWave);
    const int sub = lane() / kCompactLanes, sl = lane() % kCompactLanes;
    for (int64_t w0 = ((int64_t)blockIdx.x * (256 / kWave) + threadIdx.x / kWave) * kCompactSub; w0 < n_walkers;
         w0 += nwaves * kCompactSub) {
        const int64_t w = w0 + sub;
        if (w >= n_walkers) continue;
        // (bpre: block-local offsets of k_walker_scan)
        const uint64_t d0 = offs[w] + (bpre ? bpre[w / kWalkerScanBlock] : 0),
                       cnt = offs[w + 1] + (bpre ? bpre[(w + 1) / kWalkerScanBlock] : 0) - d0, s0 = (uint64_t)w * cap_w;
        g += sl == 0 ? (wgt[w] & 0xFFFFu) : 0u;
        for (uint64_t i = sl; i < cnt; i += kCompactLanes) {
            const uint64_t sl = s0 + i, d = d0 + i;
            line_end[d] = le_b[sl];
            alt[d] = alt_b[sl];
            tot[d] = tot_b[sl];
            if (aux_b) aux[d] = aux_b[sl];
            rowpre[d] = rowpre_b[sl];
            status[d] = status_b[sl];
            meta[d] = meta_b[sl];
        }
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
        if (blockIdx.x == 0) *n_lines = offs[n_walkers] + (bpre ? bpre[n_walkers / kWalkerScanBlock] : 0);
    }
}

int64_t af_walkers(int64_t lo, int64_t hi, int64_t chunk) { return hi > lo ? (hi - lo + chunk - 1) / chunk : 0; }

hipError_t launch_af_walk(const char *buf, int64_t lo, int64_t hi, int64_t chunk, int mode, int64_t span0,
                          uint64_t cap_w, uint64_t *le_b, int32_t *alt_b, int32_t *tot_b, uint32_t *rowpre_b,
                          uint8_t *status_b, void *meta_b, uint64_t *wcount, uint32_t *wgt, unsigned *overflow,
                          hipStream_t s, int32_t *hwe_aux_b, const WalkTail *tail, bool dose, bool gt_first_walk,
                          bool dose_head) {
    const WalkTail t = tail ? *tail : WalkTail{};
    const int64_t nw = af_walkers(lo, hi, chunk);
    if (!nw) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((nw + kWalkWaves - 1) / kWalkWaves);
    if (gt_first_walk)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_af_walk<AfOp, true>), dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi,
                           chunk, nw, mode, span0, cap_w, le_b, alt_b, tot_b, nullptr, rowpre_b, status_b,
                           static_cast<LineMeta *>(meta_b), wcount, wgt, overflow, t);
    else if (dose && dose_head)
        hipLaunchKernelGGL(k_af_walk<DoseHeadOp>, dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, mode,
                           span0, cap_w, le_b, alt_b, tot_b, nullptr, rowpre_b, status_b, static_cast<LineMeta *>(meta_b),
                           wcount, wgt, overflow, t);
    else if (dose)
        hipLaunchKernelGGL(k_af_walk<DoseWalkOp>, dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, mode,
                           span0, cap_w, le_b, alt_b, tot_b, nullptr, rowpre_b, status_b, static_cast<LineMeta *>(meta_b),
                           wcount, wgt, overflow, t);
    else if (hwe_aux_b)
        hipLaunchKernelGGL(k_af_walk<HweOp>, dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, mode, span0,
                           cap_w, le_b, alt_b, tot_b, hwe_aux_b, rowpre_b, status_b, static_cast<LineMeta *>(meta_b),
                           wcount, wgt, overflow, t);
    else
        hipLaunchKernelGGL(k_af_walk<AfOp>, dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, mode, span0,
                           cap_w, le_b, alt_b, tot_b, nullptr, rowpre_b, status_b, static_cast<LineMeta *>(meta_b),
                           wcount, wgt, overflow, t);
    return hipGetLastError();
}

hipError_t launch_walk_compact(int64_t n_walkers, uint64_t cap_w, const uint64_t *offs, const uint32_t *wgt,
                               const uint64_t *le_b, const int32_t *alt_b, const int32_t *tot_b,
                               const uint32_t *rowpre_b, const uint8_t *status_b, const void *meta_b,
                               uint64_t *line_end, int32_t *alt, int32_t *tot, uint32_t *rowpre, uint8_t *status,
                               void *meta, uint64_t *n_lines, unsigned long long *counters, hipStream_t s,
                               const int32_t *aux_b, int32_t *aux, const uint64_t *bpre) {
    const int64_t blocks = std::min<int64_t>((n_walkers + 256 / kWave - 1) / (256 / kWave), 512);
    hipLaunchKernelGGL(k_walk_compact, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s, n_walkers, cap_w,
                       offs, wgt, le_b, alt_b, tot_b, aux_b, rowpre_b, status_b, static_cast<const LineMeta *>(meta_b),
                       line_end, alt, tot, aux, rowpre, status, static_cast<LineMeta *>(meta), n_lines, counters, bpre);
    return hipGetLastError();
}

}  // namespace vcfxg
