// vcfxg_gt.h -- the per-record sample sweep shared by the GT reducers (allele counts,
// genotype match, LD genotype codes).
//
// gt_fast: the fixed-stride path.  The sample region [S, E) of a record is tested for the
// layout of single-digit diploid GT-only records -- N 4-byte units "a s b \t" (the last
// without its tab), s the record's first separator ('/' or '|'), a, b in [0-9.] -- while
// the reducer consumes it.  Sample dwords d = bytes [p, p+4), p = S + 4k, come from the
// lane's 16 B block by v_alignbyte; per dword e = d ^ (0x09<<24 | '0'<<16 | s<<8 | '0'):
// bytes 1 and 3 must be 0, bytes 0 and 2 a digit (0..9) or '.' (0x1E).  A record that
// deviates anywhere returns false (wave-uniform) and the caller runs gt_general, which
// restates the reference's per-sample loop exactly.
#pragma once
#include <algorithm>
#include <type_traits>

#include "vcfxg_device.h"

// af_fixed's loads: a batch of kUnroll wave-steps per sweep step (default), or rolling
// (VCFXG_AF_ROLL=1: a step's loads re-issued as soon as it is consumed).  r04 A/B on one box,
// 2 alternations each (af_walk ms): batch 0.896-0.904, rolling 0.969-0.970, rolling at 5 steps
// 0.916-0.919 -- the rolling variant's extra VGPRs cost occupancy
#ifndef VCFXG_AF_ROLL
#define VCFXG_AF_ROLL 0
#endif
// gt_first_af's loads through a per-batch buffer resource (1) or clamped global addresses (0)
#ifndef VCFXG_GF_BUF
#define VCFXG_GF_BUF 1
#endif

#ifndef VCFXG_FQ_EXPT
#define VCFXG_FQ_EXPT 0
#endif

namespace vcfxg {

struct DwordView {
    uint32_t d;    // canonical sample dword: byte0 = allele a, byte1 = sep, byte2 = allele b
    uint32_t f;    // (d ^ exp) & 0x00FF00FF: allele digit values in 16-bit fields
    uint32_t dig;  // bit 8 / bit 24 set where the allele is a digit
    bool real;     // false: padding outside [S, E) (neutral ". ." bytes)
    int64_t p;     // offset of the sample's first byte
};

template <class Op>
__device__ __forceinline__ void fast_dword(uint32_t d, uint32_t exp_xor, uint32_t &err, Op &op, bool real,
                                           int64_t p) {
    uint32_t e = d ^ exp_xor;
    err |= e & 0xFF00FF00u;
    uint32_t f = e & 0x00FF00FFu;
    uint32_t notdig = (f + 0x00F600F6u) & 0x01000100u;  // field >= 10
    uint32_t notdot = ((f ^ 0x001E001Eu) + 0x00FF00FFu) & 0x01000100u;
    err |= notdig & notdot;
    DwordView v{d, f, notdig ^ 0x01000100u, real, p};
    op.dword(v);
}

// returns false (uniformly) if the record is not fixed-stride.  S and E must be
// wave-uniform.  Offsets inside the record are 32-bit, relative to b0 = S & ~15 (records
// are far below 2 GiB): no per-lane 64-bit bounds arithmetic, nothing for the compiler to
// hoist into dozens of loop-invariant 64-bit registers.
#ifndef VCFXG_UNROLL
#define VCFXG_UNROLL 4
#endif
#ifndef VCFXG_NT_SWEEP
#define VCFXG_NT_SWEEP 0
#endif
struct NoPre {
    __device__ void operator()() const {}
};
// reducers with a clean-step form: op.clean(e0..e3), four sample dwords whose alleles are all
// '0' / '1' (e = dword ^ the expected "0 s 0 \t": bit 0 = first allele '1', bit 16 = second)
template <class T, class = void>
struct HasClean : std::false_type {};
template <class T>
struct HasClean<T, std::void_t<decltype(&T::clean)>> : std::true_type {};
// ... or op.clean_at(e0..e3, p): the same with the offset p of the first of the four dwords
// (reducers that place per-sample results: the LD walk's genotype codes)
template <class T, class = void>
struct HasCleanAt : std::false_type {};
template <class T>
struct HasCleanAt<T, std::void_t<decltype(&T::clean_at)>> : std::true_type {};
// pre(): called once, right after the record's first batch of loads is issued.
// swept (optional): the end of the bytes the sweep examined -- E, or on an early exit
// (op.done()) the end of the last batch of loads
template <int kUnroll = VCFXG_UNROLL, class Op, class Pre = NoPre>
__device__ bool gt_fast(const char *__restrict__ buf, int64_t S, int64_t E, Op &op, uint32_t sep_hint = 0,
                        Pre pre = Pre(), int64_t *swept = nullptr) {
    S = uniform64(S);
    E = uniform64(E);
    int64_t L = E - S;
    if (L < 3 || ((L + 1) & 3)) return false;
    // sep_hint: the byte at S + 1 when the caller already has it (saves a dependent load)
    uint32_t sepc = sep_hint ? sep_hint : byte_at(buf, S + 1);
    sepc = __builtin_amdgcn_readfirstlane(sepc);
    if (sepc != '/' && sepc != '|') return false;
    const uint32_t exp_xor = 0x09000000u | (sepc << 8) | 0x00300030u;
    const uint32_t neutral = 0x092E002Eu | (sepc << 8);  // ". ." + tab: valid, reduces to nothing
    op.begin(sepc, neutral);
    const int s = (int)(S & 3);
    const int64_t b0 = S & ~(int64_t)15;
    const char *__restrict__ base = buf + b0;
    const int Sr = (int)(S - b0), Er = (int)(E - b0);  // record bounds relative to b0
#if VCFXG_NT_SWEEP
    const int lastblk = (Er - 1) & ~15;  // block holding the record's last byte
#endif
    uint32_t err = 0;
    if (swept) *swept = E;
    // kUnroll wave-steps per iteration: their loads are all issued before any is consumed
    const int lo16 = lane() * kBlockBytes;
#if !VCFXG_NT_SWEEP
    // the record's 16 B blocks as a buffer: a lane past the record reads zeros (its bytes are
    // masked below) with no clamped address, and the loads issue back to back in one basic
    // block (per-lane branches around them made the compiler wait for each before the next)
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(base, (uint32_t)((Er + 15) & ~15));
#endif
    for (int w0 = 0; w0 < Er; w0 += kUnroll * kWaveStep) {
        uint4 v[kUnroll];
        uint32_t x4[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            const int blk = w0 + u * kWaveStep + lo16;
#if VCFXG_NT_SWEEP  // streaming (non-temporal) loads for the read-once sample bytes
            const int bl = blk < Er ? blk : lastblk;  // (a lane past the record re-reads its last block)
            {
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(base + bl));
                v[u] = make_uint4(t.x, t.y, t.z, t.w);
            }
            x4[u] = load4(base, bl + 16);
#else
            v[u] = bload16(rs, blk);
            x4[u] = bload4(rs, blk + 16);
#endif
        }
        if (w0 == 0) pre();  // e.g. a prefetch that must not hold up these loads
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            const int w = w0 + u * kWaveStep;
            const int blk = w + lo16;
            // interior step: every sample dword of every lane lies in [S, E) and is not the last
            const bool interior = (w + s >= Sr) && (w + kWaveStep - 1 + s < Er);
            if (blk < Er) {
                uint32_t d[4] = {__builtin_amdgcn_alignbyte(v[u].y, v[u].x, s),
                                 __builtin_amdgcn_alignbyte(v[u].z, v[u].y, s),
                                 __builtin_amdgcn_alignbyte(v[u].w, v[u].z, s),
                                 __builtin_amdgcn_alignbyte(x4[u], v[u].w, s)};
                bool clean = false;
                if constexpr (HasClean<Op>::value || HasCleanAt<Op>::value) {
                    // an interior step whose every allele is '0' / '1' (e = d ^ exp has only
                    // bits 0 and 16): the reducer's SWAR form on the four e's at once
                    if (interior) {
                        const uint32_t e0 = d[0] ^ exp_xor, e1 = d[1] ^ exp_xor, e2 = d[2] ^ exp_xor,
                                       e3 = d[3] ^ exp_xor;
                        clean = !__any(((e0 | e1 | e2 | e3) & ~0x00010001u) != 0u);
                        if (clean) {
                            if constexpr (HasCleanAt<Op>::value) op.clean_at(e0, e1, e2, e3, b0 + blk + s);
                            else op.clean(e0, e1, e2, e3);
                        }
                    }
                }
                bool real[4] = {true, true, true, true};
                if (!interior) {
                    const int q0 = blk + s - Sr, last = Er - Sr - 3;  // dword i starts at S + q0 + 4i
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int q = q0 + 4 * i;
                        if (q < 0 || q > last) {
                            d[i] = neutral;
                            real[i] = false;
                        } else if (q == last) d[i] = (d[i] & 0x00FFFFFFu) | 0x09000000u;
                    }
                }
                if (!clean) {
#pragma unroll
                    for (int i = 0; i < 4; i++) fast_dword(d[i], exp_xor, err, op, real[i], b0 + blk + s + 4 * i);
                }
            }
        }
        if (op.done()) {  // wave-uniform early exit (e.g. a match was found)
            if (swept && b0 + w0 + kUnroll * kWaveStep < E) *swept = b0 + w0 + kUnroll * kWaveStep;
            break;
        }
        if (__any(err != 0u)) return false;  // not fixed-stride: stop reading the record
    }
    if (__any(err != 0u)) return false;
    op.finish();
    return true;
}

// general path: op.sample(st) for every sample start (S, and every tab+1 < E), one lane
// per start in its 16 B block; op.finish() reduces across the wave.
template <class Op>
__device__ void gt_general(const char *__restrict__ buf, int64_t S, int64_t E, Op &op) {
    for (int64_t w = S & ~(int64_t)15; w < E; w += kWaveStep) {
        int64_t blk = w + (int64_t)lane() * kBlockBytes;
        if (blk < E) {
            uint32_t tm = eq_mask16(load16(buf, blk), kRepTab);
            uint32_t starts = (tm << 1) & 0xFFFFu;
            if (blk > 0 && byte_at(buf, blk - 1) == '\t') starts |= 1u;
            starts &= range_mask16(blk, S + 1, E);
            if (S >= blk && S < blk + 16) starts |= 1u << (S - blk);
            while (starts) {
                int j = __builtin_ctz(starts);
                starts &= starts - 1u;
                op.sample(blk + j);
            }
        }
        if (op.done()) break;
    }
    op.finish();
}

// end of the sample starting at st: first '\t' at or after st, or E
__device__ __forceinline__ int64_t sample_end(const char *__restrict__ buf, int64_t st, int64_t E) {
    int64_t p = st;
    while (p < E && byte_at(buf, p) != '\t') p++;
    return p;
}

// ---------------------------------------------------------------------------------------
// gt_first: records whose FORMAT starts with GT and has more sub-fields ("GT:AD:DP", ...), so
// samples have any width.  One pass over [S, hi) finds the line end E (the first '\n', or hi;
// cr = its '\r' when strip_cr, ae = E - cr) and, for every sample start p in [S, ae) (S and
// each tab + 1), takes the bytes c0..c3 at p: a "quick" GT is c0 s c2 with s '/' or '|', c0
// and c2 not a separator, ':', tab, space or '\r', and c3 ':' or tab or p + 3 == ae -- the
// GT sub-field of exactly 3 bytes, whose tokens are c0 and c2 alone: op.gt3(c0, c2).  Any
// other sample makes the result false (wave-uniform): the caller runs gt_general with the
// end it now knows.  pre(E) is called once, as soon as E is known (the next line's prefetch).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool gt_special(uint32_t c) {
    return c == '/' || c == '|' || c == ':' || c == '\t' || c == ' ' || c == '\r';
}
template <int kU, class Op, class Pre>
__device__ bool gt_first(const char *__restrict__ buf, int64_t S, int64_t hi, int strip_cr, Op &op, Pre pre,
                         int64_t &E_out, uint8_t &cr_out) {
    S = uniform64(S);
    int64_t E = hi, ae = hi;
    bool found = false, bad = false;
    uint32_t carry = 0;  // byte 15 of the previous wave-step's last lane
    const int64_t b0 = S & ~(int64_t)15;
    const int lo16 = lane() * kBlockBytes;
    for (int64_t w0 = b0; w0 < hi && !found; w0 += kU * kWaveStep) {
        uint4 v[kU];
        uint32_t x4[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {  // branch-free: lanes past hi re-read the last block
            const int64_t blk = w0 + u * kWaveStep + lo16;
            const int64_t bl = blk < hi ? blk : ((hi - 1) & ~(int64_t)15);
            v[u] = load16(buf, bl);
            x4[u] = load4(buf, bl + 16);
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            if (found) break;
            const int64_t blk = w0 + u * kWaveStep + lo16;
            const uint32_t nlm = blk < hi ? eq_mask16(v[u], kRepNl) & range_mask16(blk, S, hi) : 0u;
            const uint64_t anyn = __ballot(nlm != 0u);
            if (anyn) {
                const int k = __builtin_ctzll(anyn);
                E = uniform64(w0 + u * kWaveStep + 16 * k + __builtin_ctz((uint32_t)__shfl((int)nlm, k)));
                found = true;
                const uint32_t cr = strip_cr && E > S ? __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r' : 0u;
                cr_out = (uint8_t)cr;
                ae = E - cr;
                pre(E);
            }
            // sample starts: S, and the byte after every tab, in [S, ae)
            const uint32_t tm = eq_mask16(v[u], kRepTab);
            const uint32_t last = lane_prev(v[u].w >> 24);
            const uint32_t prev = lane() ? last : carry;
            carry = lane_last(v[u].w >> 24);
            uint32_t starts = ((tm << 1) & 0xFFFFu) | (prev == '\t' ? 1u : 0u);
            if (S >= blk && S < blk + 16) starts |= 1u << (S - blk);
            starts &= range_mask16(blk, S, ae);
            const uint32_t wd[5] = {v[u].x, v[u].y, v[u].z, v[u].w, x4[u]};
            while (starts) {
                const int o = __builtin_ctz(starts);
                starts &= starts - 1u;
                const int q = o >> 2;
                const uint32_t lo = q == 0 ? wd[0] : q == 1 ? wd[1] : q == 2 ? wd[2] : wd[3];
                const uint32_t hw = q == 0 ? wd[1] : q == 1 ? wd[2] : q == 2 ? wd[3] : wd[4];
                const uint32_t d = __builtin_amdgcn_alignbyte(hw, lo, (uint32_t)(o & 3));
                const uint32_t c0 = d & 0xFFu, c1 = (d >> 8) & 0xFFu, c2 = (d >> 16) & 0xFFu, c3 = d >> 24;
                const int64_t p3 = blk + o + 3;
                const bool quick = (c1 == '/' || c1 == '|') && !gt_special(c0) && !gt_special(c2) &&
                                   (p3 == ae || (p3 < ae && (c3 == ':' || c3 == '\t')));
                if (quick) op.gt3(c0, c2);
                else bad = true;
            }
        }
    }
    if (!found) {
        E = hi;
        const uint32_t cr = strip_cr && E > S ? __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r' : 0u;
        cr_out = (uint8_t)cr;
        pre(E);
    }
    E_out = E;
    if (__any(bad)) return false;
    op.finish();
    return true;
}
struct NoPreE {
    __device__ void operator()(int64_t) const {}
};
// the GT-first sweep over a sample region [S, ae) of known end (no '\n' inside)
template <int kU = 8, class Op>
__device__ __forceinline__ bool gt_first_known(const char *__restrict__ buf, int64_t S, int64_t ae, Op &op) {
    int64_t e;
    uint8_t cr;
    return gt_first<kU>(buf, S, ae, 0, op, NoPreE(), e, cr);
}

// ---------------------------------------------------------------------------------------
// allele-count reducer: parseGenotypeAndCount (VCFX_allele_freq_calc.cpp:262-293) over
// extractGT (:321-337)
// ---------------------------------------------------------------------------------------
struct AfOp {
    const char *buf;
    int64_t E;
    int gi;
    uint32_t alt = 0, tot = 0;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {
        tot += __popc(v.dig);
        alt += __popc((v.f + 0x00FF00FFu) & v.dig);  // digit 1..9
    }
    // a 3-byte GT "c0 s c2" (gt_first): each single-byte token counts if it is a digit
    __device__ void gt3(uint32_t c0, uint32_t c2) {
        tot += (c0 - '0' < 10u) + (c2 - '0' < 10u);
        alt += (c0 - '1' < 9u) + (c2 - '1' < 9u);
    }
    __device__ void sample(int64_t st) {
        int64_t p = st;
        for (int k = 0; k < gi; k++) {  // skip gi colon fields
            while (p < E) {
                uint32_t c = byte_at(buf, p);
                if (c == '\t' || c == ':') break;
                p++;
            }
            if (p >= E || byte_at(buf, p) == '\t') return;
            p++;
        }
        bool in_tok = false, first_dot = false, numeric = true, nonzero = false;
        for (;; p++) {
            uint32_t c = p < E ? byte_at(buf, p) : (uint32_t)'\t';
            bool end = (c == '\t' || c == ':');
            if (end || c == '/' || c == '|') {
                if (in_tok && !first_dot && numeric) {
                    tot++;
                    if (nonzero) alt++;
                }
                in_tok = false;
                if (end) break;
                continue;
            }
            if (!in_tok) {
                in_tok = true;
                first_dot = (c == '.');
                numeric = true;
                nonzero = false;
            }
            if (c < '0' || c > '9') numeric = false;
            else if (c != '0') nonzero = true;
        }
    }
    __device__ void finish() {
        alt = wave_sum(alt);
        tot = wave_sum(tot);
    }
};

// the row's frequency text (VCFX_allele_freq_calc.cpp: writeDouble4 in file mode, printf "%.4f"
// on stdin) -- shared by the walk's staged rows and k_af_format_w
// writeDouble4 (VCFX_allele_freq_calc.cpp:119-143): (ull)(v*10000.0+0.5), no FMA contraction
__device__ __forceinline__ uint32_t fixed4_mmap(double v) {
    double sc = __dadd_rn(__dmul_rn(v, 10000.0), 0.5);
    return (uint32_t)(unsigned long long)sc;
}
// printf("%.4f") of v in [0, 1]: exact binary value, round half to even (glibc)
__device__ __forceinline__ uint32_t fixed4_printf(double v) {
    if (v == 0.0) return 0u;
    uint64_t bits = __double_as_longlong(v);
    int ex = (int)((bits >> 52) & 0x7FF);
    uint64_t m = bits & ((1ull << 52) - 1);
    int q;  // v = m * 2^-q
    if (ex == 0) q = 1074;
    else { m |= 1ull << 52; q = 1075 - ex; }
    if (q <= 0) return 10000u * (uint32_t)(m << -q);  // v >= 2^52: not reachable for freqs
    unsigned __int128 num = (unsigned __int128)m * 10000u;
    if (q >= 100) return 0u;
    unsigned __int128 k = num >> q;
    unsigned __int128 rem = num - (k << q);
    unsigned __int128 half = (unsigned __int128)1 << (q - 1);
    if (rem > half || (rem == half && (k & 1))) k += 1;
    return (uint32_t)k;
}

__device__ __forceinline__ void af_freq_text(int mode, int32_t a, int32_t t, uint32_t &lo, uint32_t &hi) {
    const double f = t > 0 ? __ddiv_rn((double)a, (double)t) : 0.0;
    const uint32_t k4 = mode == 0 ? fixed4_mmap(f) : fixed4_printf(f);
    const uint32_t ip = k4 / 10000u, fp = k4 % 10000u;
    // "i.dddd\n": bytes 0..3 in lo, 4..6 in hi
    lo = ('0' + ip) | ((uint32_t)'.' << 8) | (('0' + fp / 1000u) << 16) | (('0' + (fp / 100u) % 10u) << 24);
    hi = ('0' + (fp / 10u) % 10u) | (('0' + fp % 10u) << 8) | ((uint32_t)'\n' << 16);
}
// ---------------------------------------------------------------------------------------
// gt_first_af: gt_first for the allele counts, on per-byte flags instead of a loop over each
// lane's sample starts.  Bytes are classified SWAR on the lane's 16 B and the 4 B after them
// (bit 7 of each byte; every byte must be ASCII -- else the record goes to the exact path):
// for a byte b < 0x80, (b ^ c) + 0x7F has bit 7 set iff b != c, and b + (0x80 - c) iff b >= c.
// A sample start p (S, and the byte after a tab) is accepted when p+1 is '/' or '|', p+3 is
// ':', a tab or the line's '\n', and p, p+2 are digits or '.': the quick GT c0 s c2, whose
// tokens are c0 and c2 alone (letters and the like at p or p+2 go to the exact path, as do
// CRLF line ends).  The flags of p+1 and p+3 are lined up with p's by v_alignbyte over
// neighbouring dwords, and the start flags are moved to p+2 the same way, so the allele bytes
// (p and p+2) are one flag word: tot and alt are popcounts of its digit and nonzero-digit
// flags (r04: 8 fewer VALU per dword than aligning the digit flags of p+2 to p).  Same contract as gt_first: the record end E (first '\n'
// at or after S, else hi), pre(E) as soon as it is known, false (wave-uniform) -> the
// caller's exact path; on true op.alt / op.tot hold the record's counts.
// ---------------------------------------------------------------------------------------
template <int kU, class Pre>
__device__ bool gt_first_af(const char *__restrict__ buf, int64_t S, int64_t hi, int strip_cr, AfOp &op, Pre pre,
                            int64_t &E_out, uint8_t &cr_out) {
    S = uniform64(S);
    constexpr uint32_t M = 0x80808080u, K = 0x7F7F7F7Fu;
    int64_t E = hi, ae = hi;
    bool found = false;
    uint32_t bad = 0, asc = 0, tot = 0, alt = 0;
    uint32_t carry = 0;  // tab flags of the previous step's last lane (byte 3: the byte before this step)
    uint32_t scarry = 0;  // its last dword's starts
    const int64_t b0 = S & ~(int64_t)15;
    const int lo16 = lane() * kBlockBytes;
    const int64_t hend = (hi + 15) & ~(int64_t)15;  // (the block holding hi - 1 is read whole)
    for (int64_t w0 = b0; w0 < hi && !found; w0 += kU * kWaveStep) {
        uint4 v[kU];
        uint32_t x4[kU];
#if VCFXG_GF_BUF
        // the batch's bytes as a buffer based at w0: lanes past hi read zeros (masked below),
        // no per-lane 64-bit address or clamp
        const __amdgpu_buffer_rsrc_t rs =
            buf_rsrc(buf + w0, (uint32_t)std::min<int64_t>(hend - w0, (int64_t)kU * kWaveStep + 16));
#pragma unroll
        for (int u = 0; u < kU; u++) {
            v[u] = bload16(rs, u * kWaveStep + lo16);
            x4[u] = bload4(rs, u * kWaveStep + lo16 + 16);
        }
#else
#pragma unroll
        for (int u = 0; u < kU; u++) {  // branch-free: lanes past hi re-read the last block
            const int64_t blk = w0 + u * kWaveStep + lo16;
            const int64_t bl = blk < hi ? blk : hend - 16;
            v[u] = load16(buf, bl);
            x4[u] = load4(buf, bl + 16);
        }
#endif
#pragma unroll
        for (int u = 0; u < kU; u++) {
            if (found) break;
            const int64_t ws = w0 + u * kWaveStep, blk = ws + lo16;
            const uint32_t W[5] = {v[u].x, v[u].y, v[u].z, v[u].w, x4[u]};
            const uint32_t wor = W[0] | W[1] | W[2] | W[3];  // (bit 7: a byte >= 0x80)
            asc |= wor | W[4];
            // ---- the record end: the first '\n' at or after S (the first step may hold bytes
            // before S, the last lanes of the input's last step re-read its last block)
            const bool first = ws == b0, edge = first || ws + kWaveStep > hi;  // wave-uniform
            // interior steps: the ASCII shortcut (the same sums as the classes below), exact only
            // where it flags a byte.  A byte >= 0x80 can carry into the next byte's sum and hide
            // a '\n' there (and such a record goes to the exact path, which needs the true end):
            // the shortcut flags every such byte too, so its step takes the exact masks.
            uint32_t nlm = 0;
            if (edge) nlm = blk < hi ? eq_mask16(v[u], kRepNl) & range_mask16(blk, S, hi) : 0u;
            else
                nlm = (~(((W[0] ^ kRepNl) + K) & ((W[1] ^ kRepNl) + K) & ((W[2] ^ kRepNl) + K) &
                         ((W[3] ^ kRepNl) + K)) | wor) & M;
            uint64_t anyn = __ballot(nlm != 0u);
            if (anyn && !edge) {  // (rare: the step holding the record end) exact masks
                nlm = eq_mask16(v[u], kRepNl);
                anyn = __ballot(nlm != 0u);
            }
            if (anyn) {
                const int k = __builtin_ctzll(anyn);  // (lane k's mask is exact and nonzero)
                E = uniform64(ws + 16 * k + __builtin_ctz((uint32_t)__shfl((int)nlm, k)));
                found = true;
                const uint32_t cr = strip_cr && E > S ? __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r' : 0u;
                cr_out = (uint8_t)cr;
                ae = E - cr;
                pre(E);
            }
            // ---- sample starts: the byte after a tab (the byte before the lane's block: the
            // previous lane's, or the previous step's last), S, and only inside [S, ae)
            const uint32_t tab3 = ~((W[3] ^ kRepTab) + K);
            const uint32_t up = lane_prev(tab3);
            uint32_t tprev = lane() ? up : carry;
            carry = lane_last(tab3);
            uint32_t rm = 0xFFFFu;
            if (edge || found) {
                rm = blk < hi ? range_mask16(blk, S, ae) : 0u;
                rm |= ((S >= blk && S < blk + 16) ? 1u << (S - blk) : 0u) << 16;  // S: a start
            }
            // ---- the starts of the lane's 4 dwords (bit 7 of each byte), then the starts two
            // bytes back (s2: the c2 position of a start; dword 0's first two bytes are the
            // previous lane's, or the previous step's last lane's, last two starts).  A byte is
            // never both (a start two bytes after a start has a tab at the earlier start's
            // separator: that start is bad), so u = st | s2 marks every allele byte once.
            uint32_t st[4];
            {
                uint32_t tp = tprev;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t tb = i == 3 ? tab3 : ~((W[i] ^ kRepTab) + K);
                    uint32_t x = __builtin_amdgcn_alignbyte(tb, tp, 3) & M;
                    if (edge || found)
                        x = (x | nib_bytes((rm >> (16 + 4 * i)) & 0xFu)) & nib_bytes((rm >> (4 * i)) & 0xFu) & M;
                    st[i] = x;
                    tp = tb;
                }
            }
            const uint32_t sup = lane_prev(st[3]);
            const uint32_t sprev = lane() ? sup : scarry;
            scarry = lane_last(st[3]);
            // ---- dword by dword (classes of W[i] and W[i+1] live at a time): each start needs
            // c1 separator and c3 terminator, each allele byte (c0, c2) a digit or '.'; the counts
            // are the allele bytes' digit / nonzero-digit flags
            auto classes = [&](uint32_t x, uint32_t &sep, uint32_t &trm, uint32_t &vv, uint32_t &dg, uint32_t &nz) {
                const uint32_t nt = (x ^ kRepTab) + K, nn = (x ^ kRepNl) + K, nc = (x ^ kRepColon) + K;
                trm = ~(nt & nn & nc);
                const uint32_t ns = (x ^ 0x2F2F2F2Fu) + K;  // bit 7 clear: '/'
                sep = ~(ns & ((x ^ 0x7C7C7C7Cu) + K));
                const uint32_t g9 = x + 0x46464646u;  // >= ':'
                dg = (x + 0x50505050u) & ~g9;         // '0'..'9'
                nz = (x + 0x4F4F4F4Fu) & ~g9;         // '1'..'9'
                vv = (x + 0x52525252u) & ~g9 & ns;    // '.'..'9' but '/': '.' or a digit
            };
            uint32_t sep0, trm0, v0, dg0, nz0;
            classes(W[0], sep0, trm0, v0, dg0, nz0);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                uint32_t sep1, trm1, v1, dg1, nz1;
                classes(W[i + 1], sep1, trm1, v1, dg1, nz1);
                const uint32_t s1 = __builtin_amdgcn_alignbyte(sep1, sep0, 1);
                const uint32_t c3 = __builtin_amdgcn_alignbyte(trm1, trm0, 3);
                const uint32_t s2 = __builtin_amdgcn_alignbyte(st[i], i ? st[i - 1] : sprev, 2);
                const uint32_t u = st[i] | s2;
                bad |= (st[i] & ~(s1 & c3)) | (u & ~v0);
                tot = popc_acc(u & dg0, tot);  // (one v_bcnt each: the compiler split them into
                alt = popc_acc(u & nz0, alt);  // a bcnt and a share of an add3)
                sep0 = sep1, trm0 = trm1, v0 = v1, dg0 = dg1, nz0 = nz1;
            }
        }
    }
    if (!found) {
        E = hi;
        const uint32_t cr = strip_cr && E > S ? __builtin_amdgcn_readfirstlane(byte_at(buf, E - 1)) == '\r' : 0u;
        cr_out = (uint8_t)cr;
        pre(E);
    }
    E_out = E;
    if (__any((bad | (asc & M)) != 0u)) return false;
    op.alt = wave_sum32(alt);  // (every lane active: the walk's uniform per-record path)
    op.tot = wave_sum32(tot);
    return true;
}

// ---------------------------------------------------------------------------------------
// af_fixed: gt_fast + AfOp (the same record test and the same counts) on the raw 16 B
// blocks, without realigning them to the sample grid.  In a fixed-stride record every byte's
// role -- allele, separator or tab -- is (offset - S) mod 4, so a raw aligned dword holds the
// canonical unit "0 s 0 \t" rotated left by 8 (S mod 4) bits, whichever samples its bytes
// belong to (the allele counts do not care).  Per raw dword, against that rotated expectation:
//   e = d ^ exp:  a record whose alleles are all '0' / '1' has e = 0 except bit 0 of its
//   allele bytes, so  err |= e & rot(0xFFFEFFFE)  and  alt += popc(e)  are the whole test and
//   count (3 VALU per 4 bytes; tot = 2 x units), where gt_fast spends ~15 per sample and an
//   extra 4-byte load per lane for the realignment;
// a wave-step that fails that (some allele neither '0' nor '1') is counted again, from the
// same registers, with gt_fast's per-allele rules (digit: counts, 1..9: ALT, '.': not counted,
// anything else: not fixed-stride).  Bytes outside [S, E) read as the expected '0'-allele
// bytes (the last sample's byte at E -- its '\n' -- as its tab), so they neither count nor fail.
// Returns false (wave-uniform) where gt_fast returns false; op.alt / op.tot as gt_fast leaves
// them after op.finish().
// ---------------------------------------------------------------------------------------
// (first / vb: the walk's early loads -- the first kUnroll wave-steps from vb (16-aligned, <= S),
// issued before the record's head was analysed; vb < 0: none)
template <int kUnroll, class Pre>
__device__ bool af_fixed(const char *__restrict__ buf, int64_t S, int64_t E, AfOp &op, uint32_t sep_hint, Pre pre,
                         const uint4 *first = nullptr, int64_t vb = -1) {
    S = uniform64(S);
    E = uniform64(E);
    const int64_t L = E - S;
    if (L < 3 || ((L + 1) & 3)) return false;
    uint32_t sepc = sep_hint ? sep_hint : byte_at(buf, S + 1);
    sepc = __builtin_amdgcn_readfirstlane(sepc);
    if (sepc != '/' && sepc != '|') return false;
    const uint32_t sh = 8u * (uint32_t)(S & 3);
    auto rot = [&](uint32_t x) { return sh ? (x << sh) | (x >> (32u - sh)) : x; };
    const uint32_t exp = rot(0x09300030u | (sepc << 8));  // '0' s '0' \t
    const uint32_t mbin = rot(0xFFFEFFFEu);               // separator / tab bytes whole, allele bits 1..7
    const uint32_t msep = rot(0xFF00FF00u);               // separator / tab bytes
    const uint32_t fsh = (S & 1) ? 8u : 0u;               // allele bytes -> bytes 0 and 2
    const int64_t b0 = vb >= 0 ? uniform64(vb) : S & ~(int64_t)15;
    const char *__restrict__ base = buf + b0;
    const int Sr = (int)(S - b0), Er = (int)(E - b0);  // record bounds relative to b0
    // the record's 16 B blocks as a buffer: lanes past it read zeros (masked like the bytes
    // past E, below), with no clamped address per load
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(base, (uint32_t)((Er + 15) & ~15));
    const int lo16 = lane() * kBlockBytes;
    uint32_t alt = 0, dots = 0, err = 0, alt8 = 0;
    static_assert(4 * kUnroll <= 255, "af_fixed: bytewise allele sums");
#if VCFXG_AF_ROLL
    // rolling loads: as soon as a wave-step's registers are read, the same step of the next batch
    // is issued into them, so kUnroll steps stay in flight across batches (no bubble between a
    // record's batches) at no register cost
    uint4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; u++) v[u] = bload16(rs, u * kWaveStep + lo16);
    pre();
#endif
    for (int w0 = 0; w0 < Er; w0 += kUnroll * kWaveStep) {
#if !VCFXG_AF_ROLL
        uint4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) v[u] = first && w0 == 0 ? first[u] : bload16(rs, w0 + u * kWaveStep + lo16);
        if (w0 == 0) pre();
#endif
#if VCFXG_AF_ROLL
        const int wn = w0 + kUnroll * kWaveStep;  // the next batch (wave-uniform)
#endif
        // the step's dwords, bytes outside [S, E) replaced by the expected ones (edge steps only)
        auto dwords = [&](int u, const uint4 &x, uint32_t(&d)[4]) {
            d[0] = x.x, d[1] = x.y, d[2] = x.z, d[3] = x.w;
            const int w = w0 + u * kWaveStep;
            if (!(w >= Sr && w + kWaveStep <= Er)) {  // wave-uniform
                const int blk = w + lo16;
                const uint32_t rm = blk < Er ? range16(blk, Sr, Er) : 0u;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t bm = nib_bytes((rm >> (4 * i)) & 0xFu);
                    d[i] = (d[i] & bm) | (exp & ~bm);
                }
            }
        };
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            uint32_t d[4];
            dwords(u, v[u], d);
#if VCFXG_AF_ROLL
            if (wn < Er) v[u] = bload16(rs, wn + u * kWaveStep + lo16);
#endif
            // a clean step (berr = 0) has e = bit 0 of the '1' allele bytes alone: its count is
            // the byte sum of the e's, added bytewise (at most 4 kUnroll <= 255 per byte) and
            // folded into alt once per batch (v_sad_u8) -- two adds a step, not four popcounts
            const uint32_t e0 = d[0] ^ exp, e1 = d[1] ^ exp, e2 = d[2] ^ exp, e3 = d[3] ^ exp;
            const uint32_t berr = (e0 | e1 | e2 | e3) & mbin;
            if (!__any(berr != 0u)) {
                alt8 += e0 + e1 + e2 + e3;
                continue;
            }
            // some allele of the step is neither '0' nor '1': gt_fast's per-allele rules
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t e = d[i] ^ exp;
                err |= e & msep;
                const uint32_t f = (e >> fsh) & 0x00FF00FFu;
                const uint32_t notdig = (f + 0x00F600F6u) & 0x01000100u;  // field >= 10
                const uint32_t notdot = ((f ^ 0x001E001Eu) + 0x00FF00FFu) & 0x01000100u;
                err |= notdig & notdot;
                dots += __popc(notdig);  // (valid: not a digit = '.')
                alt += __popc((f + 0x00FF00FFu) & (notdig ^ 0x01000100u));  // digit 1..9
            }
        }
        if (__any(err != 0u)) return false;  // not fixed-stride: stop reading the record
        alt = __builtin_amdgcn_sad_u8(alt8, 0u, alt);
        alt8 = 0;
    }
    op.alt = wave_sum32(alt);  // (every lane active)
    op.tot = (uint32_t)(2 * ((L + 1) >> 2)) - wave_sum32(dots);
    return true;
}

// af_fixed on the walk's carried loads (VCFXG_AF_XREC): the same test and counts, with the
// sweep's grid based at vb (16-aligned, <= S; the bytes before S are masked like those past E)
// when v already holds the wave-steps [vb, vb + kUnroll KiB) (lane l: vb + 1 KiB u + 16 l),
// or at S & ~15 with its own first loads when vb < 0.  Its rolling loads continue past the
// record into the next line's first wave-steps, from nb (16-aligned) when nb >= 0: on a true
// return v holds [nb, nb + kUnroll KiB) and vb_out = nb, so the next record's sweep starts
// with its first KiBs already in flight -- issued before this record's last steps were read,
// not after the next head's analysis.  vb_out = -1 otherwise.
template <int kUnroll, class Pre>
__device__ bool af_fixed_x(const char *__restrict__ buf, int64_t S, int64_t E, int64_t hi, AfOp &op, uint32_t sep_hint,
                           Pre pre, uint4 (&v)[kUnroll], int64_t vb, int64_t nb, int64_t &vb_out) {
    S = uniform64(S);
    E = uniform64(E);
    vb_out = -1;
    const int64_t L = E - S;
    if (L < 3 || ((L + 1) & 3)) return false;
    uint32_t sepc = sep_hint ? sep_hint : byte_at(buf, S + 1);
    sepc = __builtin_amdgcn_readfirstlane(sepc);
    if (sepc != '/' && sepc != '|') return false;
    const uint32_t sh = 8u * (uint32_t)(S & 3);
    auto rot = [&](uint32_t x) { return sh ? (x << sh) | (x >> (32u - sh)) : x; };
    const uint32_t exp = rot(0x09300030u | (sepc << 8));  // '0' s '0' \t
    const uint32_t mbin = rot(0xFFFEFFFEu);
    const uint32_t msep = rot(0xFF00FF00u);
    const uint32_t fsh = (S & 1) ? 8u : 0u;
    const int64_t b0 = vb >= 0 ? uniform64(vb) : S & ~(int64_t)15;
    const char *__restrict__ base = buf + b0;
    const int Sr = (int)(S - b0), Er = (int)(E - b0);
    const int lastblk = (Er - 1) & ~15;
    const int lo16 = lane() * kBlockBytes;
    const int64_t hlast = (hi - 1) & ~(int64_t)15;
    uint32_t alt = 0, dots = 0, err = 0;
    if (vb < 0) {
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            const int blk = u * kWaveStep + lo16;
            v[u] = load16(base, blk < Er ? blk : lastblk);
        }
    }
    pre();
    for (int w0 = 0; w0 < Er; w0 += kUnroll * kWaveStep) {
        const int wn = w0 + kUnroll * kWaveStep;  // the next batch (wave-uniform)
        auto dwords = [&](int u, const uint4 &x, uint32_t(&d)[4]) {
            d[0] = x.x, d[1] = x.y, d[2] = x.z, d[3] = x.w;
            const int w = w0 + u * kWaveStep;
            if (!(w >= Sr && w + kWaveStep <= Er)) {  // wave-uniform
                const int blk = w + lo16;
                const uint32_t rm = blk < Er ? range16(blk, Sr, Er) : 0u;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t bm = nib_bytes((rm >> (4 * i)) & 0xFu);
                    d[i] = (d[i] & bm) | (exp & ~bm);
                }
            }
        };
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            uint32_t d[4];
            dwords(u, v[u], d);
            if (wn < Er) {
                const int blk = wn + u * kWaveStep + lo16;
                v[u] = load16(base, blk < Er ? blk : lastblk);
            } else if (nb >= 0) {  // the next line's first wave-steps
                const int64_t g = nb + u * kWaveStep + lo16;
                v[u] = load16(buf, g < hi ? g : hlast);
            }
            uint32_t berr = 0, balt = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t e = d[i] ^ exp;
                berr |= e & mbin;
                balt += __popc(e);
            }
            if (!__any(berr != 0u)) {
                alt += balt;
                continue;
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t e = d[i] ^ exp;
                err |= e & msep;
                const uint32_t f = (e >> fsh) & 0x00FF00FFu;
                const uint32_t notdig = (f + 0x00F600F6u) & 0x01000100u;
                const uint32_t notdot = ((f ^ 0x001E001Eu) + 0x00FF00FFu) & 0x01000100u;
                err |= notdig & notdot;
                dots += __popc(notdig);
                alt += __popc((f + 0x00FF00FFu) & (notdig ^ 0x01000100u));
            }
        }
        if (__any(err != 0u)) return false;
    }
    op.alt = wave_sum32(alt);  // (every lane active)
    op.tot = (uint32_t)(2 * ((L + 1) >> 2)) - wave_sum32(dots);
    vb_out = nb;
    return true;
}

// ---------------------------------------------------------------------------------------
// genotype-match reducer: genotypeMatchesFast (VCFX_genotype_query.cpp:275-316) over
// extractNthField (:199-218); "any sample matches" (checkAnySampleMatches :322-345)
// ---------------------------------------------------------------------------------------
struct GqQuery {
    const char *q;  // query bytes (device)
    int qlen;
    int strict;
    int qa, qb;     // parsed + sorted query alleles (host parse, partial-assignment semantics kept)
};

__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }

// parseDiploidAlleles (VCFX_genotype_query.cpp:246-272) on [g, g+n)
__device__ __forceinline__ bool parse_diploid(const char *__restrict__ buf, int64_t g, int64_t n, int &a1, int &a2) {
    int64_t sep = -1;
    for (int64_t i = 0; i < n; i++) {
        uint32_t c = byte_at(buf, g + i);
        if (c == '|' || c == '/') { sep = i; break; }
    }
    if (sep <= 0 || sep == n - 1) return false;
    if (sep == 1 && byte_at(buf, g) == '.') return false;
    uint32_t v = 0;
    for (int64_t i = 0; i < sep; i++) {
        uint32_t c = byte_at(buf, g + i);
        if (!is_digit(c)) return false;
        v = v * 10u + (c - '0');
    }
    a1 = (int)v;
    if (n - sep - 1 == 1 && byte_at(buf, g + sep + 1) == '.') return false;
    v = 0;
    for (int64_t i = sep + 1; i < n; i++) {
        uint32_t c = byte_at(buf, g + i);
        if (!is_digit(c)) return false;
        v = v * 10u + (c - '0');
    }
    a2 = (int)v;
    return true;
}

__device__ __forceinline__ bool gt_matches(const char *__restrict__ buf, int64_t g, int64_t n, const GqQuery &Q) {
    if (Q.strict) {
        if (n != Q.qlen) return false;
        for (int64_t i = 0; i < n; i++)
            if (byte_at(buf, g + i) != (uint32_t)(uint8_t)Q.q[i]) return false;
        return true;
    }
    if (n == 3 && Q.qlen == 3) {
        uint32_t s = byte_at(buf, g + 1);
        if (s != '|' && s != '/') return false;
        uint32_t g0 = byte_at(buf, g), g1 = byte_at(buf, g + 2);
        if (!is_digit(g0) || !is_digit(g1)) return false;
        int ga = (int)(g0 - '0'), gb = (int)(g1 - '0');
        if (ga > gb) { int t = ga; ga = gb; gb = t; }
        return ga == Q.qa && gb == Q.qb;
    }
    int a1 = 0, a2 = 0;
    if (!parse_diploid(buf, g, n, a1, a2)) return false;
    if (a1 > a2) { int t = a1; a1 = a2; a2 = t; }
    return a1 == Q.qa && a2 == Q.qb;
}

struct GqOp {
    const char *buf;
    int64_t E;
    int gi;
    GqQuery Q;
    uint32_t p1 = 0, p2 = 0, pmask = 0;  // fast-path dword pattern(s)
    // fast path: the least of (x ^ p1, x ^ p2) over this lane's dwords -- 0 iff one matched
    // (VALU min / xor: as lane booleans the match tests had cost three scalar mask ops each)
    uint32_t mn = ~0u;
    bool any = false;                    // this lane (general path)
    bool found = false;                  // wave
    __device__ void begin(uint32_t sepc, uint32_t) {
        begin_patterns();
        if (!pmask) p1 = p2 = ~0u;  // (no fast-path match: x never has bit 31)
        (void)sepc;
    }
    __device__ void begin_patterns() {
        // on the fixed-stride layout a GT is "a s b"; flexible: match <=> a, b digits with
        // sorted (a, b) == (qa, qb); strict: the 3 bytes equal the query
        if (Q.strict) {
            if (Q.qlen == 3) {
                p1 = p2 = (uint32_t)(uint8_t)Q.q[0] | ((uint32_t)(uint8_t)Q.q[1] << 8) | ((uint32_t)(uint8_t)Q.q[2] << 16);
                pmask = 0x00FFFFFFu;
            } else pmask = 0;
        } else if (Q.qa >= 0 && Q.qa <= 9 && Q.qb >= 0 && Q.qb <= 9) {
            p1 = (uint32_t)('0' + Q.qa) | ((uint32_t)('0' + Q.qb) << 16);
            p2 = (uint32_t)('0' + Q.qb) | ((uint32_t)('0' + Q.qa) << 16);
            pmask = 0x00FF00FFu;
        } else pmask = 0;
    }
    // (VCFXG_FQ_EXPT & 1, diagnostic builds: no early exit -- every record swept whole)
    __device__ bool done() {
        return (VCFXG_FQ_EXPT & 1) ? false : (found = found || __any(any || mn == 0u));
    }
    __device__ void dword(const DwordView &v) {
        const uint32_t x = (v.d & pmask) | (v.real ? 0u : 0x01000000u);  // (padding never matches)
        mn = std::min(mn, std::min(x ^ p1, x ^ p2));
    }
    __device__ void sample(int64_t st) {
        if (any) return;
        int64_t se = sample_end(buf, st, E);
        // extractNthField(sample, gi)
        int64_t p = st, fs = st;
        int fi = 0;
        for (;; p++) {
            bool end = (p == se) || byte_at(buf, p) == ':';
            if (end) {
                if (fi == gi) break;
                fi++;
                fs = p + 1;
                if (p == se) return;  // fewer fields: empty
            }
        }
        int64_t n = p - fs;
        if (n > 0 && gt_matches(buf, fs, n, Q)) any = true;
    }
    __device__ void finish() { found = __any(any || mn == 0u); }
};

// ---------------------------------------------------------------------------------------
// nonref reducer (VCFX_nonref_filter): "some sample is not hom-ref".
// Per sample the gi-th ':' subfield g (empty when absent) is hom-ref iff
//   mmap  (allSamplesHomRefDirect :286-300): |g| = 3 ? g = "0s0" (s '/' or '|')
//                                               : g non-empty of '0', '/', '|' only;
//   stdin (isDefinitelyHomRef :419-449): g = "0s0", or g non-empty of '0', '/', '|' only.
// An empty sample is not hom-ref in both modes.  On the fixed-stride layout (a, b digits or
// '.') both rules are "a = b = '0'": the dword's digit fields are both 0.
// ---------------------------------------------------------------------------------------
struct NrOp {
    const char *buf;
    int64_t E;
    int gi, mode;                // mode 0 mmap, 1 stdin
    bool any = false;            // this lane saw a sample that is not hom-ref
    bool found = false;          // wave
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() { return found = found || __any(any); }
    __device__ void dword(const DwordView &v) { any = any || (v.real && v.f != 0u); }
    __device__ void sample(int64_t st) {
        if (any) return;
        const int64_t se = sample_end(buf, st, E);
        int64_t p = st, fs = st;
        int fi = 0;
        for (;; p++) {  // extractNthField(sample, gi) / the gi-th getline token
            const bool end = (p == se) || byte_at(buf, p) == ':';
            if (end) {
                if (fi == gi) break;
                fi++;
                fs = p + 1;
                if (p == se) {  // fewer subfields: not hom-ref
                    any = true;
                    return;
                }
            }
        }
        const int64_t n = p - fs;
        bool hr = n > 0;
        bool only = n > 0;  // every byte '0', '/' or '|'
        for (int64_t k = fs; only && k < p; k++) {
            const uint32_t c = byte_at(buf, k);
            only = c == '0' || c == '/' || c == '|';
        }
        if (n == 3) {
            const uint32_t c1 = byte_at(buf, fs + 1);
            const bool pat = byte_at(buf, fs) == '0' && (c1 == '/' || c1 == '|') && byte_at(buf, fs + 2) == '0';
            hr = pat || (mode == 1 && only);
        } else hr = only;
        if (!hr) any = true;
    }
    __device__ void finish() { found = __any(any); }
};

// ---------------------------------------------------------------------------------------
// missing-genotype reducer (VCFX_missing_detector) on the fixed-stride
// layout: every sample is a 3-byte GT "a s b" between tabs, so a '.' allele is at its GT's
// start or end -- the sample is missing (hasMissingGenotypeInSamples,
// VCFX_missing_detector.cpp:290-336); early exit at the first one
// ---------------------------------------------------------------------------------------
struct MdOp {
    bool any = false;    // this lane saw a '.' allele
    bool found = false;  // wave
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() { return found = found || __any(any); }
    __device__ void dword(const DwordView &v) { any = any || (v.real && v.dig != 0x01000100u); }
    __device__ void finish() { found = __any(any); }
};

// ---------------------------------------------------------------------------------------
// HWE genotype-class reducer (VCFX_hwe_tester): per sample
// parseGenotypeForHWE (VCFX_hwe_tester.cpp:339-378) -> 0 hom-ref, 1 het, 2 hom-alt, or
// invalid (not counted).  The sample's first ':' sub-field, leading ' ' / '\r' skipped, two
// '/'- or '|'-separated integers (digits after the second are ignored), both <= 1.  On the
// fixed-stride layout a sample counts iff both fields are digits <= 1; the class is a + b.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int hwe_parse(const char *__restrict__ buf, int64_t p, int64_t end) {
    if (p >= end) return -1;
    for (int64_t k = p; k < end; k++)  // memchr(':')
        if (byte_at(buf, k) == ':') {
            end = k;
            break;
        }
    while (p < end && (byte_at(buf, p) == ' ' || byte_at(buf, p) == '\r')) p++;
    if (p >= end || !is_digit(byte_at(buf, p))) return -1;  // also '.'
    // int accumulation as the reference's (two's-complement wrap on absurdly long numbers)
    uint32_t a1 = 0, a2 = 0;
    while (p < end && is_digit(byte_at(buf, p))) {
        a1 = a1 * 10u + (byte_at(buf, p) - '0');
        p++;
    }
    if (p >= end || (byte_at(buf, p) != '/' && byte_at(buf, p) != '|')) return -1;
    p++;
    if (p >= end || !is_digit(byte_at(buf, p))) return -1;
    while (p < end && is_digit(byte_at(buf, p))) {
        a2 = a2 * 10u + (byte_at(buf, p) - '0');
        p++;
    }
    if ((int32_t)a1 > 1 || (int32_t)a2 > 1) return -1;
    if (a1 == 0u && a2 == 0u) return 0;
    if (a1 == 1u && a2 == 1u) return 2;
    return 1;
}

// VCFX_dosage_calculator's row-length pass on the walk (fixed-stride records): samples and the
// samples that print "NA" (not both alleles digits), as k_dose_len's DoseCountOp on gt_fast
struct DoseWalkOp {
    const char *buf;
    int64_t E;
    uint32_t ns = 0, na = 0;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {
        ns += v.real;
        na += v.real && v.dig != 0x01000100u;
    }
    __device__ void finish() {
        ns = wave_sum(ns);
        na = wave_sum(na);
    }
};

// the dosage HEAD walk (k_af_walk<DoseHeadOp>): a GT-only record whose end the walk predicts
// from the previous fixed-stride record (and whose predicted end byte is the '\n') is taken
// as fixed-stride without "NA" and without its samples being read; k_dose_fmt checks every
// sample byte of such a row while it writes it and flags the call when one fails (the call is
// then redone with DoseWalkOp).  Records the walk sweeps anyway count as DoseWalkOp does.
struct DoseHeadOp : DoseWalkOp {};

struct HweOp {
    const char *buf;
    int64_t E;
    uint32_t c0 = 0, c1 = 0, c2 = 0;  // hom-ref, het, hom-alt (after finish())
    // fixed-stride accumulators: (valid samples << 16) + ALT alleles of the valid ones, and
    // the hom-alt count (a lane sees < 65536 dwords of a record)
    uint32_t nv_alt = 0, two = 0;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {
        // both fields 0 or 1 (no other field value, '.' included, passes)
        const bool ok = (v.f & 0x00FE00FEu) == 0u;
        nv_alt += ok ? (uint32_t)__popc(v.f) + 0x10000u : 0u;
        two += v.f == 0x00010001u;
    }
    // four valid samples: their ALT alleles (popcounts) and hom-alt ones (both bits)
    __device__ void clean(uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3) {
        nv_alt = popc_acc(e3, popc_acc(e2, popc_acc(e1, popc_acc(e0, nv_alt + 0x40000u))));
        two += (e0 & (e0 >> 16)) + (e1 & (e1 >> 16)) + (e2 & (e2 >> 16)) + (e3 & (e3 >> 16));
    }
    __device__ void gt3(uint32_t c0, uint32_t c2) {  // both '0' or '1': the class a + b
        const bool ok = (c0 - '0' < 2u) && (c2 - '0' < 2u);
        const uint32_t s = (c0 - '0') + (c2 - '0');
        c0_ += ok && s == 0u;
        c1_ += ok && s == 1u;
        c2_ += ok && s == 2u;
    }
    uint32_t c0_ = 0, c1_ = 0, c2_ = 0;  // gt_first's counts (folded in finish())
    __device__ void sample(int64_t st) {
        const int g = hwe_parse(buf, st, sample_end(buf, st, E));
        c0 += g == 0;
        c1 += g == 1;
        c2 += g == 2;
    }
    __device__ void finish() {
        const uint32_t nv = nv_alt >> 16, alt = nv_alt & 0xFFFFu;
        c2 += two + c2_;
        c1 += alt - 2u * two + c1_;
        c0 += nv - (alt - two) + c0_;
        c0 = wave_sum(c0);
        c1 = wave_sum(c1);
        c2 = wave_sum(c2);
    }
};

}  // namespace vcfxg
