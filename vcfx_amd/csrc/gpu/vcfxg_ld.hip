// vcfxg_ld.hip -- VCFX_ld_calculator on the device.
//
// K_ld_parse  : one wave per line -> int8 genotype codes (0/1/2, -1 missing) of the first
//               numSamples samples (parseGenotypeRaw, VCFX_ld_calculator.cpp:145-174, on
//               extractGT :177-185), per-variant sums (computeStats :243-258), POS
//               (fastParseInt :188-197), region filter, chrom / ID spans.
// K_ld_block  : r^2 for a 64x64 block of variant pairs with int8 MFMA
//               (v_mfma_i32_32x32x32_i8, exact int32 sums), then the reference's fp64
//               epilogue (computeRsqSIMD x86 body :352-393 via computeRsqFast :397-401) with
//               correctly rounded __d*_rn ops.  Pass 1 counts pairs with r^2 >= threshold
//               per (row j, column block); pass 2 writes them in the reference's order
//               (j ascending, then i ascending = the window from oldest to newest).
// Missing genotypes: tiles whose variants are all complete need only X.X^T; otherwise the
// kernel accumulates X.X^T, X.V^T, V.X^T, V.V^T, X2.V^T, V.X2^T (V = valid mask, X2 = x^2).
#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_ld.h"
#include "vcfxg_walk.h"

namespace vcfxg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int int_len(int v) {
    unsigned u = v < 0 ? 0u - (unsigned)v : (unsigned)v;
    int n = v < 0 ? 1 : 0;
    do {
        n++;
        u /= 10u;
    } while (u);
    return n;
}
__device__ __forceinline__ char *put_int(char *o, int v) {  // formatInt :214-225 / to_string
    unsigned u = v < 0 ? 0u - (unsigned)v : (unsigned)v;
    if (v < 0) *o++ = '-';
    char t[12];
    int k = 0;
    do {
        t[k++] = (char)('0' + u % 10u);
        u /= 10u;
    } while (u);
    while (k) *o++ = t[--k];
    return o;
}


// ---------------------------------------------------------------------------------------
// parse
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int gt_code_raw(const char *__restrict__ buf, int64_t s, int64_t len) {
    // parseGenotypeRaw on [s, s+len)
    if (len == 0) return -1;
    uint32_t c0 = byte_at(buf, s);
    if (len == 1 && c0 == '.') return -1;
    if (len == 3 && c0 == '.' && (byte_at(buf, s + 1) == '/' || byte_at(buf, s + 1) == '|') &&
        byte_at(buf, s + 2) == '.')
        return -1;
    int64_t sep = 0;
    for (int64_t i = 0; i < len; i++) {
        uint32_t c = byte_at(buf, s + i);
        if (c == '/' || c == '|') {
            sep = i;
            break;
        }
    }
    if (sep == 0 || sep >= len - 1) return -1;
    uint32_t a1 = 0, a2 = 0;
    for (int64_t i = 0; i < sep; i++) {
        uint32_t c = byte_at(buf, s + i);
        if (c - '0' >= 10u) return -1;
        a1 = a1 * 10u + (c - '0');
    }
    for (int64_t i = sep + 1; i < len; i++) {
        uint32_t c = byte_at(buf, s + i);
        if (c - '0' >= 10u) return -1;
        a2 = a2 * 10u + (c - '0');
    }
    if ((int)a1 > 1 || (int)a2 > 1) return -1;
    return (int)(a1 + a2);
}

// std::stoi on [s, e): leading isspace, sign, >= 1 digit, int range; trailing text ignored
__device__ __forceinline__ bool cxx_stoi(const char *__restrict__ buf, int64_t s, int64_t e, int *out) {
    int64_t p = s;
    while (p < e) {
        uint32_t c = byte_at(buf, p);
        if (!(c == ' ' || (c >= 9 && c <= 13))) break;
        p++;
    }
    bool neg = false;
    if (p < e && (buf[p] == '+' || buf[p] == '-')) {
        neg = buf[p] == '-';
        p++;
    }
    int64_t v = 0;
    int nd = 0;
    while (p < e && byte_at(buf, p) - '0' < 10u) {
        v = v * 10 + (int64_t)(byte_at(buf, p) - '0');
        if (v > 2147483648ll) v = 2147483649ll;  // saturate: out of range either way
        p++;
        nd++;
    }
    if (!nd) return false;
    if (neg) v = -v;
    if (v < -2147483648ll || v > 2147483647ll) return false;
    *out = (int)v;
    return true;
}

// VCFXLDCalculator::parseGenotype (:468-482) on the whole sample field [s, s+len)
__device__ int gt_code_stoi(const char *__restrict__ buf, int64_t s, int64_t len) {
    if (len == 0) return -1;
    uint32_t c0 = byte_at(buf, s);
    if (len == 1 && c0 == '.') return -1;
    if (len == 3 && c0 == '.' && (byte_at(buf, s + 1) == '/' || byte_at(buf, s + 1) == '|') &&
        byte_at(buf, s + 2) == '.')
        return -1;
    int64_t sep = -1;
    for (int64_t i = 0; i < len; i++) {
        uint32_t c = byte_at(buf, s + i);
        if (c == '/' || c == '|') {
            sep = i;
            break;
        }
    }
    if (sep < 0) return -1;
    const int64_t n1 = sep, n2 = len - sep - 1;
    if (n1 == 0 || n2 == 0) return -1;
    if ((n1 == 1 && c0 == '.') || (n2 == 1 && byte_at(buf, s + sep + 1) == '.')) return -1;
    int i1, i2;
    // a '|' inside a2 reads as '/' after the replace; both stop stoi's digit run
    if (!cxx_stoi(buf, s, s + sep, &i1) || !cxx_stoi(buf, s + sep + 1, s + len, &i2)) return -1;
    if (i1 < 0 || i2 < 0 || i1 > 1 || i2 > 1) return -1;
    if (i1 == i2) return i1 == 0 ? 0 : 2;
    return 1;
}

struct LdStats {
    uint32_t cnt = 0, sx = 0, sx2 = 0;
    __device__ void add(int code) {
        if (code >= 0) {
            cnt++;
            sx += (uint32_t)code;
            sx2 += (uint32_t)(code * code);
        }
    }
};

// fixed-stride path: sample k = (p - S) / 4
struct LdOp {
    int8_t *row;
    int64_t S;
    int ns;
    LdStats st;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {
        if (!v.real) return;
        int64_t k = (v.p - S) >> 2;
        if (k >= ns) return;
        uint32_t a = v.d & 0xFF, b = (v.d >> 16) & 0xFF;
        int code = ((a - '0') < 2u && (b - '0') < 2u) ? (int)(a - '0' + b - '0') : -1;
        row[k] = (int8_t)code;
        st.add(code);
    }
    __device__ void sample(int64_t) {}
    __device__ void finish() {}
};

// the same codes into the wave's LDS row (an LDS-address-space pointer: ds_write_b8), written
// out afterwards as 16 B stores
struct LdOpL {
    __attribute__((address_space(3))) int8_t *row;
    int64_t S;
    int ns;
    LdStats st;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {
        if (!v.real) return;
        int64_t k = (v.p - S) >> 2;
        if (k >= ns) return;
        uint32_t a = v.d & 0xFF, b = (v.d >> 16) & 0xFF;
        int code = ((a - '0') < 2u && (b - '0') < 2u) ? (int)(a - '0' + b - '0') : -1;
        row[k] = (int8_t)code;
        st.add(code);
    }
    __device__ void sample(int64_t) {}
    __device__ void finish() {}
};
constexpr int kLdLdsRow = 4096;  // samples per record composed in LDS (more: byte stores to HBM)

// LdOpL with the clean-step form (vcfxg_gt.h HasCleanAt): four samples whose alleles are all
// '0' / '1' (e = dword ^ "0 s 0 \t", bits 0 and 16 only) -> their four codes as one dword
// into the LDS row (k is congruent mod 4 across the wave: one store shape per record)
struct LdOpW : LdOpL {
    __device__ void clean_at(uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3, int64_t p) {
        const int64_t k = (p - S) >> 2;
        const uint32_t c0 = (e0 + (e0 >> 16)) & 3u, c1 = (e1 + (e1 >> 16)) & 3u, c2 = (e2 + (e2 >> 16)) & 3u,
                       c3 = (e3 + (e3 >> 16)) & 3u;
        if (k + 3 < ns) {
            const uint32_t w = c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
            auto *r = row + k;
            if ((k & 3) == 0) {
                *reinterpret_cast<__attribute__((address_space(3))) uint32_t *>(r) = w;
            } else if ((k & 1) == 0) {
                reinterpret_cast<__attribute__((address_space(3))) uint16_t *>(r)[0] = (uint16_t)w;
                reinterpret_cast<__attribute__((address_space(3))) uint16_t *>(r)[1] = (uint16_t)(w >> 16);
            } else {
                r[0] = (int8_t)c0;
                r[1] = (int8_t)c1;
                r[2] = (int8_t)c2;
                r[3] = (int8_t)c3;
            }
            const uint32_t sum = c0 + c1 + c2 + c3;
            st.cnt += 4u;
            st.sx += sum;
            st.sx2 += sum + 2u * ((c0 >> 1) + (c1 >> 1) + (c2 >> 1) + (c3 >> 1));
        } else {
            const uint32_t c[4] = {c0, c1, c2, c3};
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (k + i < ns) {
                    row[k + i] = (int8_t)c[i];
                    st.add((int)c[i]);
                }
        }
    }
};

// general path: samples numbered by a running count of starts (sampleIdx, :598-611)
__device__ void ld_general(const char *__restrict__ buf, int64_t S, int64_t E, int ns, int8_t *row, LdStats &st,
                           int stoi_mode) {
    int64_t run = 0;
    for (int64_t w = S & ~(int64_t)15; w < E && run < ns; w += kWaveStep) {
        int64_t blk = w + (int64_t)lane() * kBlockBytes;
        uint32_t starts = 0;
        if (blk < E) {
            uint32_t tm = eq_mask16(load16(buf, blk), kRepTab);
            starts = (tm << 1) & 0xFFFFu;
            if (blk > 0 && byte_at(buf, blk - 1) == '\t') starts |= 1u;
            starts &= range_mask16(blk, S + 1, E);
            if (S >= blk && S < blk + 16) starts |= 1u << (S - blk);
        }
        int c = __popc(starts);
        int incl = wave_incl_scan(c);
        int64_t idx = run + incl - c;
        while (starts) {
            int j = __builtin_ctz(starts);
            starts &= starts - 1u;
            if (idx < ns) {
                int64_t st0 = blk + j, p = st0;
                while (p < E) {
                    uint32_t ch = byte_at(buf, p);
                    if (ch == '\t' || ch == ':') break;
                    p++;
                }
                int code;
                if (stoi_mode) {  // parseGenotype on the whole field (:468-482)
                    while (p < E && byte_at(buf, p) != '\t') p++;
                    code = gt_code_stoi(buf, st0, p - st0);
                } else code = gt_code_raw(buf, st0, p - st0);
                row[idx] = (int8_t)code;
                st.add(code);
            }
            idx++;
        }
        run += wave_bcast(incl, kWave - 1);
    }
}

// one line [ls, le) -> its LdLine; a valid line's codes into row (kpad bytes, global; composed
// in the wave's LDS row lrow when ns <= kLdLdsRow).  pad: also write -1 over the row's bytes
// past the codes (the walk's rows are not cleared beforehand; k_ld_parse's are, by a memset)
__device__ __forceinline__ LdLine ld_line(const char *__restrict__ buf, int64_t ls, int64_t le, const LdParseArgs &a,
                          int8_t *__restrict__ row, int8_t *lrow, int64_t *lds, bool pad) {
    LdLine out;
    out.valid = 0;
    if (le > ls && byte_at(buf, ls) != '#') {
        int64_t t[10];
        const int nt = head_tabs(buf, ls, le, 9, t, lds);
        bool ok = nt >= 9;
        int pos = 0;
        if (ok && !a.stoi_mode) {  // fastParseInt(field 1)
            const int64_t p0 = t[0] + 1, p1 = t[1];
            ok = p1 > p0;
            if (ok && p1 - p0 <= kWave) {
                // lane k holds digit k: one round of loads instead of a dependent byte
                // chain; sum of d_k * 10^(len-1-k) mod 2^32 = the wrapping Horner loop
                const int len = (int)(p1 - p0), k = lane();
                const uint32_t c = k < len ? byte_at(buf, p0 + k) : (uint32_t)'0';
                ok = !__any(c - '0' >= 10u);
                uint32_t pw = 1u;
                for (int e = k; e < len - 1; e++) pw *= 10u;
                pos = (int)wave_sum(k < len ? (c - '0') * pw : 0u);
            } else if (ok) {
                uint32_t v = 0;
                for (int64_t p = p0; ok && p < p1; p++) {
                    uint32_t c = byte_at(buf, p);
                    if (c - '0' >= 10u) ok = false;
                    else v = v * 10u + (c - '0');
                }
                pos = (int)v;
            }
        } else if (ok) {  // std::stoi(fields[1]) (computeLD :1026)
            ok = cxx_stoi(buf, t[0] + 1, t[1], &pos);
        }
        if (ok && a.has_region) {
            int64_t cl = t[0] - ls;
            ok = cl == a.rlen && pos >= a.rstart && pos <= a.rend;
            for (int64_t k = 0; ok && k < cl; k++) ok = buf[ls + k] == a.rchrom[k];
        }
        if (ok) {
            const int64_t S = t[8] + 1;
            LdStats st;
            bool fast;
            if (a.ns <= kLdLdsRow) {  // codes composed in LDS, then 16 B stores
                LdOpL op{(__attribute__((address_space(3))) int8_t *)lrow, S, a.ns};
                fast = gt_fast<6>(buf, S, le, op);  // (six 1 KiB steps in flight, as the walks)
                if (fast) {
                    st = op.st;
                    const int64_t nr = (le - S + 1) / 4;
                    const uint32_t nout = (uint32_t)(nr < a.ns ? nr : a.ns);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    for (uint32_t o = (uint32_t)lane() * 16; o < nout; o += kWave * 16) {
                        if (o + 16 <= nout)
                            *reinterpret_cast<uint4 *>(row + o) = *reinterpret_cast<const uint4 *>(lrow + o);
                        else
                            for (uint32_t q = o; q < nout; q++) row[q] = lrow[q];
                    }
                    if (pad)
                        for (uint32_t q = nout + (uint32_t)lane(); q < (uint32_t)a.kpad; q += kWave) row[q] = -1;
                    // the next line's byte writes must not pass these reads
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
            } else {
                if (pad)
                    for (int k = lane(); k < a.kpad; k += kWave) row[k] = -1;
                LdOp op{row, S, a.ns};
                fast = gt_fast<6>(buf, S, le, op);
                if (fast) st = op.st;
            }
            if (!fast) {
                // rewrite the row: the failed fast sweep may have stored codes
                for (int k = lane(); k < a.kpad; k += kWave) row[k] = -1;
                ld_general(buf, S, le, a.ns, row, st, a.stoi_mode);
            }
            out.valid = 1;
            out.pos = pos;
            out.cnt = wave_sum(st.cnt);
            out.sx = wave_sum(st.sx);
            out.sx2 = wave_sum(st.sx2);
            out.chrom = (uint64_t)ls;
            out.chrom_len = (uint32_t)(t[0] - ls);
            out.id = (uint64_t)(t[1] + 1);
            out.id_len = (uint32_t)(t[2] - t[1] - 1);
        }
    }
    return out;
}

__global__ __launch_bounds__(256) void k_ld_parse(const char *__restrict__ buf, int64_t data_start,
                                                  const uint64_t *__restrict__ line_end, const uint64_t *n_lines_p,
                                                  LdParseArgs a, int8_t *__restrict__ G, LdLine *__restrict__ lines) {
    __shared__ int64_t scratch[4][16];
    __shared__ __attribute__((aligned(16))) int8_t lrows[4][kLdLdsRow];
    int64_t *lds = scratch[threadIdx.x / kWave];
    int8_t *lrow = lrows[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
        const int64_t le = (int64_t)line_end[li];
        const LdLine out = ld_line(buf, ls, le, a, G + li * (uint64_t)a.kpad, lrow, lds, false);
        if (lane() == 0) lines[li] = out;
    }
}

// a valid line's variant record and fast-kernel terms: stats -> fp64 varX exactly as
// computeStats (:243-258); `line` = the line's index (its slot, for the walk)
__device__ __forceinline__ void ld_var_of(const LdLine &L, uint64_t line, int ns, LdVar &o, LdFast &f) {
    o.pos = L.pos;
    o.cnt = (int)L.cnt;
    o.sx = (int)L.sx;
    o.sx2 = (int)L.sx2;
    double varx = 0.0;
    if (L.cnt > 0) {
        double mean = __ddiv_rn((double)L.sx, (double)L.cnt);
        varx = __dsub_rn(__ddiv_rn((double)L.sx2, (double)L.cnt), __dmul_rn(mean, mean));
    }
    o.varx = varx;
    o.complete = L.cnt == (uint32_t)ns;
    o.chrom = L.chrom;
    o.chrom_len = L.chrom_len;
    o.id = L.id;
    o.id_len = L.id_len;
    o.line = line;
    f.mx = 0.0;
    f.vx = 0.0;
    f.sq = 0.0;
    f.vxp = __longlong_as_double(0x7FF0000000000000ll);  // +inf: never a prefilter candidate
    if (L.cnt > 0) {
        const double dn = (double)L.cnt;
        f.mx = __ddiv_rn((double)L.sx, dn);
        f.vx = __dsub_rn(__ddiv_rn((double)L.sx2, dn), __dmul_rn(f.mx, f.mx));
        f.sq = f.vx > 0.0 ? __dsqrt_rn(f.vx) : 0.0;
        const int64_t V = (int64_t)L.cnt * (int64_t)L.sx2 - (int64_t)L.sx * (int64_t)L.sx;
        if (V > 0) f.vxp = (double)V;
    }
    f.sx = (int)L.sx;
    f.pos = L.pos;
}

// gather valid variants into compact order
__global__ void k_ld_compact(const LdLine *__restrict__ lines, const uint64_t *__restrict__ vidx,
                             const uint64_t *n_lines_p, int kpad, int ns, const int8_t *__restrict__ G,
                             int8_t *__restrict__ Gc, LdVar *__restrict__ vars, LdFast *__restrict__ fv) {
    const uint64_t n = *n_lines_p;
    // one block per line-chunk; each valid line copies its row (kpad bytes) with the block
    for (uint64_t li = blockIdx.x; li < n; li += gridDim.x) {
        const LdLine L = lines[li];
        if (!L.valid) continue;
        const uint64_t v = vidx[li];
        const uint4 *src = reinterpret_cast<const uint4 *>(G + li * (uint64_t)kpad);
        uint4 *dst = reinterpret_cast<uint4 *>(Gc + v * (uint64_t)kpad);
        for (int k = threadIdx.x; k < kpad / 16; k += blockDim.x) dst[k] = src[k];
        if (threadIdx.x == 0) {
            LdVar o;
            LdFast f;
            ld_var_of(L, li, ns, o, f);
            vars[v] = o;
            fv[v] = f;
        }
    }
}

// ---------------------------------------------------------------------------------------
// the LD walk: the parse without a separate line index (vcfxg_af_walk.hip's scheme).  Walker
// wk's lines -- those starting in [b(chunk start), b(chunk end)), vcfxg_walk.h walker_lines --
// go to slots wk * cap_w + n: each one's LdLine and int8 code row (kpad bytes, every byte
// written: codes, then -1).  Per line: the kWin window (LDS-DMA'd during the previous line's
// sweep) gives the first '\n' if the line is short, the first 9 tabs and POS; the end is the
// window's '\n', or predicted from the previous fixed-stride record (S + span, accepted when
// the sweep validates [S, E) and the byte at E is the '\n'), or searched for; the fixed-stride
// sweep (gt_fast + LdOpW) composes the codes in LDS.  Every other line (a head past the
// window, a POS of more than 10 digits or not all digits, a record off the fixed stride, the
// region filter, the stoi parse mode: kGen) goes to the pending list, and k_ld_pending runs
// ld_line on its exact bounds (the k_ld_parse path).  k_ld_wcompact then gathers the valid
// lines in file order.
// ---------------------------------------------------------------------------------------
#ifndef VCFXG_LD_WALK_MINW
#define VCFXG_LD_WALK_MINW 5
#endif
template <bool kGen>
__global__ __launch_bounds__(kWalkThreads) __attribute__((amdgpu_waves_per_eu(VCFXG_LD_WALK_MINW))) void k_ld_walk(const char *__restrict__ buf, int64_t lo, int64_t hi,
                                                          int64_t chunk, int64_t n_walkers, int64_t span0,
                                                          uint64_t cap_w, LdParseArgs a, int8_t *__restrict__ G,
                                                          LdLine *__restrict__ lines, uint64_t *__restrict__ wcount,
                                                          uint64_t *__restrict__ wvalid, unsigned *overflow,
                                                          unsigned long long *pend_n, uint64_t *__restrict__ pend) {
    __shared__ uint4 win[kWalkWaves][2][kWave];  // two window slots per wave (double buffer)
    __shared__ __attribute__((aligned(16))) int8_t lrows[kWalkWaves][kLdLdsRow];
    const int wv = threadIdx.x / kWave;
    const int64_t wk = uniform64((int64_t)walk_block() * kWalkWaves + wv);
    if (wk >= n_walkers) return;
    int8_t *lrow = lrows[wv];
    const auto lrow3 = (__attribute__((address_space(3))) int8_t *)lrow;
    const int64_t cs = lo + wk * chunk;
    const int64_t ce = std::min<int64_t>(cs + chunk, hi);
    int64_t L, ce2;
    walker_lines(buf, lo, hi, cs, ce, L, ce2, chunk);
    int64_t span = span0;  // predicted '\n' distance from the sample start
    uint64_t n = 0, nv = 0;
    const uint64_t base = (uint64_t)wk * cap_w;
    int cur = 0;
    int64_t A = L & ~(int64_t)15;
    if (L < ce2) prefetch_window(buf, A, hi, win[wv][cur]);
    while (L < ce2) {
        if (n >= cap_w) {
            if (lane() == 0) atomicOr(overflow, 1u);
            break;
        }
        // ---- 1. the window: first '\n', 9 tabs, POS
        const int Lr = (int)(L - A);
        const uint4 *cw = win[wv][cur];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t w4 = reinterpret_cast<const uint32_t *>(cw)[lane()];
        const int hr = (int)std::min<int64_t>(hi - A, kWin);
        const uint32_t rg = range4(Lr, hr);
        const int N1r = first_match<4>(zero_bytes(w4 ^ kRepNl) & rg);
        int rt[9] = {};
        const uint32_t ntab = first_tabs<4>(zero_bytes(w4 ^ kRepTab) & rg, N1r >= 0 ? N1r : hr, rt);
        const uint32_t first = dword_byte(w4, Lr);
        const int64_t wend = A + hr;
        bool head = !kGen && ntab >= 9 && first != '#';
        int pos = 0;
        if (head) {  // fastParseInt (:188-197) on <= 10 digits (longer ones: ld_line's wrapping loop)
            const int p0 = rt[0] + 1, p1 = rt[1];
            head = p1 > p0 && p1 - p0 <= 10;
            uint32_t v = 0;
            for (int o = p0; head && o < p1; o++) {
                const uint32_t ch = dword_byte(w4, o);
                head = ch - '0' < 10u;
                v = v * 10u + (ch - '0');
            }
            pos = (int)v;
        }
        // ---- 2. the line end
        const int64_t S = head ? A + rt[8] + 1 : 0;
        int64_t E;
        bool predicted = false;
        if (N1r >= 0) E = A + N1r;
        else if (head && span > 0 && S + span <= hi) {
            E = S + span;
            predicted = true;
        } else E = scan_nl(buf, wend, hi);
        const uint32_t sep_w = head && rt[8] + 2 < hr ? dword_byte(w4, rt[8] + 2) : 0u;
        const int nxt = cur ^ 1;
        int64_t An = std::max<int64_t>(E - 1, 0) & ~(int64_t)15;
        bool pending = true;  // the next window's prefetch is still to be issued
        auto pre = [&]() {
            prefetch_window(buf, An, hi, win[wv][nxt]);
            pending = false;
        };
        // ---- 3. the fixed-stride sweep into the LDS row
        LdOpW op{{lrow3, S, a.ns}};
        bool ok = head && gt_fast<6>(buf, S, E, op, sep_w, pre);
        if (pending) pre();
        if (predicted) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t be = slot_byte(win[wv][nxt], (int)(E - An));
            const bool endok = E < hi ? be == '\n' : true;
            if (!(ok && endok)) {
                const int64_t Et = scan_nl(buf, wend, hi);
                ok = false;
                if (Et != E) {  // the line again with its true bounds
                    E = Et;
                    An = std::max<int64_t>(E - 1, 0) & ~(int64_t)15;
                    pending = true;
                    op = LdOpW{{lrow3, S, a.ns}};
                    ok = gt_fast<6>(buf, S, E, op, sep_w, pre);
                    if (pending) pre();
                }
            }
        }
        int8_t *row = G + (base + n) * (uint64_t)a.kpad;
        LdLine out;
        if (ok) {
            // ---- 4. the row: codes [0, nout) from LDS, -1 up to kpad (16 B stores)
            const int64_t nr = (E - S + 1) / 4;
            const uint32_t nout = (uint32_t)(nr < a.ns ? nr : a.ns);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t o = (uint32_t)lane() * 16; o < (uint32_t)a.kpad; o += kWave * 16) {
                uint4 val = make_uint4(~0u, ~0u, ~0u, ~0u);
                if (o < nout) {
                    val = *reinterpret_cast<const uint4 *>(lrow + o);
                    if (o + 16 > nout) {  // the codes' last block: -1 past them
                        const int j = (int)(nout - o);
                        auto fill = [&](uint32_t x, int q) {
                            const int kq = j - 4 * q;
                            const uint32_t keep = kq >= 4 ? ~0u : kq <= 0 ? 0u : ((1u << (8 * kq)) - 1u);
                            return (x & keep) | ~keep;
                        };
                        val = make_uint4(fill(val.x, 0), fill(val.y, 1), fill(val.z, 2), fill(val.w, 3));
                    }
                }
                *reinterpret_cast<uint4 *>(row + o) = val;
            }
            // the next record's LDS writes must not pass these reads
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            out.valid = 1;
            out.pos = pos;
            out.cnt = wave_sum32(op.st.cnt);
            out.sx = wave_sum32(op.st.sx);
            out.sx2 = wave_sum32(op.st.sx2);
            out.chrom = (uint64_t)L;
            out.chrom_len = (uint32_t)(rt[0] - Lr);
            out.id = (uint64_t)(A + rt[1] + 1);
            out.id_len = (uint32_t)(rt[2] - rt[1] - 1);
            span = E - S;
        } else {  // k_ld_pending parses the line on its exact bounds [L, E)
            out.valid = 0;
            out.chrom = (uint64_t)L;
            out.id = (uint64_t)E;
            if (lane() == 0) pend[atomicAdd(pend_n, 1ull)] = base + n;
        }
        if (lane() == 0) lines[base + n] = out;
        nv += out.valid;
        n++;
        L = E + 1;
        A = An;
        cur = nxt;
    }
    if (lane() == 0) {
        wcount[wk] = n;
        wvalid[wk] = nv;
    }
}

// the walk's pending lines (bounds [chrom, id) in their LdLine): one wave each, ld_line on the
// exact bounds into the slot's row; a valid one counts in its walker's wvalid (before the scan)
__global__ __launch_bounds__(256) void k_ld_pending(const char *__restrict__ buf, LdParseArgs a, uint64_t cap_w,
                                                    const unsigned long long *pend_n, const uint64_t *__restrict__ pend,
                                                    int8_t *__restrict__ G, LdLine *__restrict__ lines,
                                                    uint64_t *wvalid) {
    __shared__ int64_t scratch[4][16];
    __shared__ __attribute__((aligned(16))) int8_t lrows[4][kLdLdsRow];
    int64_t *lds = scratch[threadIdx.x / kWave];
    int8_t *lrow = lrows[threadIdx.x / kWave];
    const uint64_t np = *pend_n;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t k = wid; k < np; k += nw) {
        const uint64_t slot = uniform64((int64_t)pend[k]);
        const LdLine b = lines[slot];
        const LdLine out = ld_line(buf, (int64_t)b.chrom, (int64_t)b.id, a, G + slot * (uint64_t)a.kpad, lrow, lds, true);
        if (lane() == 0) {
            lines[slot] = out;
            if (out.valid) atomicAdd(reinterpret_cast<unsigned long long *>(wvalid + slot / cap_w), 1ull);
        }
    }
}

// walk slots -> variants in file order, one wave per walker (vbase: exclusive scan of the
// walkers' valid-line counts): each valid line's LdVar (line = its slot) / LdFast / prefix
// length (k_ld_prefix_len); flags bit 0: some variant misses a call (its rows are gathered into
// Gc, k_ld_gather); m_out = M.  The FP4 rows follow once M is known (k_ld_pack4, slots through
// vars[v].line: every row in parallel)
__global__ __launch_bounds__(256) void k_ld_wcompact(int64_t n_walkers, uint64_t cap_w,
                                                     const uint64_t *__restrict__ wcount,
                                                     const uint64_t *__restrict__ vbase,
                                                     const LdLine *__restrict__ lines, int ns,
                                                     const char *__restrict__ buf, int id_dot_to_pos,
                                                     LdVar *__restrict__ vars, LdFast *__restrict__ fv,
                                                     uint64_t *__restrict__ plen, unsigned *flags, uint64_t *m_out) {
    const int64_t nwaves = (int64_t)gridDim.x * (256 / kWave);
    const int l = lane();
    bool incomplete = false;
    for (int64_t w = (int64_t)blockIdx.x * (256 / kWave) + threadIdx.x / kWave; w < n_walkers; w += nwaves) {
        const uint64_t n = wcount[w], v0 = vbase[w], s0 = (uint64_t)w * cap_w;
        uint64_t run = 0;
        for (uint64_t i0 = 0; i0 < n; i0 += kWave) {
            const uint64_t i = i0 + l;
            LdLine x;
            x.valid = 0;
            if (i < n) x = lines[s0 + i];
            const uint64_t bal = __ballot(x.valid != 0);
            if (x.valid) {
                const uint64_t v = v0 + run + (uint64_t)__popcll(bal & ((1ull << l) - 1ull));
                LdVar o;
                LdFast f;
                ld_var_of(x, s0 + i, ns, o, f);
                vars[v] = o;
                fv[v] = f;
                uint64_t len = o.chrom_len + 1 + int_len(o.pos) + 1;
                if (id_dot_to_pos && o.id_len == 1 && buf[o.id] == '.') len += o.chrom_len + 1 + int_len(o.pos);
                else len += o.id_len;
                plen[v] = len;
                incomplete = incomplete || !o.complete;
            }
            run += (uint64_t)__popcll(bal);
        }
    }
    if (__any(incomplete) && lane() == 0) atomicOr(flags, 1u);
    if (blockIdx.x == 0 && threadIdx.x == 0) *m_out = vbase[n_walkers];
}

// the int8 rows of the walk's variants in compact order (when some variant misses a call: the
// sparse-missing and masked kernels' planes are built from Gc)
__global__ void k_ld_gather(const LdVar *__restrict__ vars, uint64_t m, const int8_t *__restrict__ G, int kpad,
                            int8_t *__restrict__ Gc) {
    for (uint64_t v = blockIdx.x; v < m; v += gridDim.x) {
        const uint4 *src = reinterpret_cast<const uint4 *>(G + vars[v].line * (uint64_t)kpad);
        uint4 *dst = reinterpret_cast<uint4 *>(Gc + v * (uint64_t)kpad);
        for (int k = threadIdx.x; k < kpad / 16; k += blockDim.x) dst[k] = src[k];
    }
}

// ---------------------------------------------------------------------------------------
// pairwise r^2 blocks
// ---------------------------------------------------------------------------------------
constexpr int kBM = 64;  // variants per block side (4 waves x one 32x32 tile each)

// epilogue: computeRsqFast(prev = i, v = j)
__device__ __forceinline__ double rsq_epilogue(const LdVar &vi, const LdVar &vj, int n, int sx, int sy, int sxy, int sx2,
                                               int sy2, bool gate = true) {
    if (gate && (vi.varx <= 0.0 || vj.varx <= 0.0)) return 0.0;
    if (n < 2) return 0.0;
    const double dn = (double)n;
    const double mx = __ddiv_rn((double)sx, dn), my = __ddiv_rn((double)sy, dn);
    const double cov = __dsub_rn(__ddiv_rn((double)sxy, dn), __dmul_rn(mx, my));
    const double vx = __dsub_rn(__ddiv_rn((double)sx2, dn), __dmul_rn(mx, mx));
    const double vy = __dsub_rn(__ddiv_rn((double)sy2, dn), __dmul_rn(my, my));
    if (vx <= 0.0 || vy <= 0.0) return 0.0;
    const double r = __ddiv_rn(cov, __dmul_rn(__dsqrt_rn(vx), __dsqrt_rn(vy)));
    return __dmul_rn(r, r);
}

// byte transforms of a 16-byte code vector (-1 = 0xFF missing): x' (missing -> 0), v, x'^2
__device__ __forceinline__ uint32_t xprime(uint32_t c) { return c & ~(((c & 0x80808080u) >> 7) * 0xFFu); }
__device__ __forceinline__ uint32_t vmask(uint32_t c) { return (~c & 0x80808080u) >> 7; }
__device__ __forceinline__ uint32_t xsq(uint32_t xp) { return xp + (xp & 0x02020202u); }

// sums of one 32x32 tile (rows i0.., columns j0..): lane holds column j0 + (l&31), rows
// i0 + (k&3) + 8*(k>>2) + 4*(l>>5) in accumulator element k
struct TileSums {
    bool comp;  // all variants complete: only xx is valid (n, sums from the per-variant stats)
    v16i xx, xv, vx, vv, x2v, vx2;
};

__device__ __forceinline__ void tile_sums(const int8_t *__restrict__ Gc, const LdVar *__restrict__ vars, int64_t M,
                                          int kpad, int ns, int64_t i0, int64_t j0, TileSums &T) {
    const int l = lane(), r = l & 31, h = l >> 5;
    // operand rows (clamped; out-of-range rows are masked in the epilogue)
    const int64_t ia = i0 + r < M ? i0 + r : M - 1, ja = j0 + r < M ? j0 + r : M - 1;
    const int8_t *A = Gc + ia * (int64_t)kpad + 16 * h;
    const int8_t *B = Gc + ja * (int64_t)kpad + 16 * h;
    // complete tiles need only X.X^T
    const bool comp = __all(vars[ia].complete && vars[ja].complete);
    v16i xx = {}, xv = {}, vx = {}, vv = {}, x2v = {}, vx2 = {};
    const int ksteps = kpad / 32;
    if (comp) {
        for (int ks = 0; ks < ksteps; ks++) {
            v4i av = *reinterpret_cast<const v4i *>(A + 32 * ks);
            v4i bv = *reinterpret_cast<const v4i *>(B + 32 * ks);
            xx = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, xx, 0, 0, 0);
        }
    } else {
        for (int ks = 0; ks < ksteps; ks++) {
            v4i ac = *reinterpret_cast<const v4i *>(A + 32 * ks);
            v4i bc = *reinterpret_cast<const v4i *>(B + 32 * ks);
            v4i ax, avm, ax2, bx, bvm, bx2;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t ca = (uint32_t)ac[q], cb = (uint32_t)bc[q];
                uint32_t xa = xprime(ca), xb = xprime(cb);
                ax[q] = (int)xa;
                avm[q] = (int)vmask(ca);
                ax2[q] = (int)xsq(xa);
                bx[q] = (int)xb;
                bvm[q] = (int)vmask(cb);
                bx2[q] = (int)xsq(xb);
            }
            xx = __builtin_amdgcn_mfma_i32_32x32x32_i8(ax, bx, xx, 0, 0, 0);
            xv = __builtin_amdgcn_mfma_i32_32x32x32_i8(ax, bvm, xv, 0, 0, 0);
            vx = __builtin_amdgcn_mfma_i32_32x32x32_i8(avm, bx, vx, 0, 0, 0);
            vv = __builtin_amdgcn_mfma_i32_32x32x32_i8(avm, bvm, vv, 0, 0, 0);
            x2v = __builtin_amdgcn_mfma_i32_32x32x32_i8(ax2, bvm, x2v, 0, 0, 0);
            vx2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(avm, bx2, vx2, 0, 0, 0);
        }
    }
    // complete rows hold -1 in the padding bytes [ns, kpad): (-1)(-1) per byte in X.X^T
    if (comp) xx -= (kpad - ns);
    T.comp = comp;
    T.xx = xx;
    T.xv = xv;
    T.vx = vx;
    T.vv = vv;
    T.x2v = x2v;
    T.vx2 = vx2;
}

template <int P>  // P = 1: count pass, 2: emit pass
__global__ __launch_bounds__(256) void k_ld_block(const int8_t *__restrict__ Gc, const LdVar *__restrict__ vars,
                                                  const uint32_t *__restrict__ chrom_id, LdWindowArgs a,
                                                  const uint32_t *__restrict__ blocks, uint16_t *__restrict__ cnt,
                                                  LdOffsets off, LdPair *__restrict__ pairs) {
    __shared__ uint32_t masks[kBM][kBM / 32];
    const int w = threadIdx.x / kWave;
    const int it = w >> 1, jt = w & 1;
    const uint32_t bI = blocks[2 * blockIdx.x], bJ = blocks[2 * blockIdx.x + 1];
    const int64_t i0 = (int64_t)bI * kBM + it * 32, j0 = (int64_t)bJ * kBM + jt * 32;
    const int l = lane(), r = l & 31, h = l >> 5;
    const int64_t M = (int64_t)a.m;
    TileSums T;
    tile_sums(Gc, vars, M, a.kpad, a.ns, i0, j0, T);
    const bool comp = T.comp;
    const v16i &xx = T.xx, &xv = T.xv, &vx = T.vx, &vv = T.vv, &x2v = T.x2v, &vx2 = T.vx2;
    // epilogue: lane holds column j = j0 + r, rows i = i0 + (k&3) + 8*(k>>2) + 4*h
    const int64_t j = j0 + r;
    const bool jok = j < M && j >= (int64_t)a.j_lo && j < (int64_t)a.j_hi;
    LdVar vj;
    if (jok) vj = vars[j];
    uint32_t bits = 0;  // bit k: pair (row(k), j) passes
    double r2v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int64_t i = i0 + (k & 3) + 8 * (k >> 2) + 4 * h;
        r2v[k] = 0.0;
        if (!jok || i >= j || i >= M || i + (int64_t)a.window < j) continue;
        const LdVar vi = vars[i];
        if (a.max_dist > 0 && chrom_id[i] == chrom_id[j]) {
            int d = vj.pos - vi.pos;
            if (d < 0) d = -d;
            if (d > a.max_dist) continue;
        }
        double rr;
        if (comp) rr = rsq_epilogue(vi, vj, a.ns, vi.sx, vj.sx, xx[k], vi.sx2, vj.sx2);
        else rr = rsq_epilogue(vi, vj, vv[k], xv[k], vx[k], xx[k], x2v[k], vx2[k]);
        if (rr >= a.threshold) {
            bits |= 1u << k;
            r2v[k] = rr;
        }
    }
    // 32-row pass mask of column j in this tile: lanes l and l^32 hold rows 4h + ...
    uint32_t m32 = 0;
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (bits & (1u << k)) m32 |= 1u << ((k & 3) + 8 * (k >> 2) + 4 * h);
    m32 |= __shfl_xor(m32, 32);
    if (h == 0) masks[jt * 32 + r][it] = m32;
    __syncthreads();
    // first column block of row block bJ: rows j >= bJ*kBM pair with i >= j - window
    const uint64_t jrow0 = (uint64_t)bJ * kBM;
    const uint32_t ifirst = (uint32_t)(jrow0 > a.window ? (jrow0 - a.window) / kBM : 0);
    const uint64_t slot_col = (uint64_t)(bI - ifirst);
    if (P == 1) {
        if (threadIdx.x < kBM) {
            const int64_t jj = (int64_t)bJ * kBM + threadIdx.x;
            if (jj < M && jj >= (int64_t)a.j_lo && jj < (int64_t)a.j_hi)
                cnt[(uint64_t)(jj - (int64_t)a.j_lo) * a.nb + slot_col] =
                    (uint16_t)(__popc(masks[threadIdx.x][0]) + __popc(masks[threadIdx.x][1]));
        }
        return;
    }
    if (!jok || !bits) return;
    const uint64_t base = off.at((uint64_t)(j - (int64_t)a.j_lo), a.nb, slot_col);
    const uint32_t above = it ? __popc(masks[jt * 32 + r][0]) : 0u;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if (!(bits & (1u << k))) continue;
        const int row = (k & 3) + 8 * (k >> 2) + 4 * h;
        const uint32_t rank = above + __popc(m32 & ((1u << row) - 1u));
        LdPair pr;
        pr.i = (uint32_t)(i0 + row);
        pr.j = (uint32_t)j;
        pr.r2 = r2v[k];
        pairs[base + rank] = pr;
    }
}

// ---------------------------------------------------------------------------------------
// matrix mode: cells (i, j) of an M x M grid, 7 bytes each ("\t" + r^2 text), row-major
// ---------------------------------------------------------------------------------------
__device__ void fmt_r2(char *o, double r2);
__device__ __forceinline__ void fmt_printf4(char *o, double v) {  // "%.4f" of v in [0, 1]
    uint32_t k = 0;
    if (v != 0.0) {
        uint64_t bits = __double_as_longlong(v);
        int ex = (int)((bits >> 52) & 0x7FF);
        uint64_t m = bits & ((1ull << 52) - 1);
        int q;
        if (ex == 0) q = 1074;
        else {
            m |= 1ull << 52;
            q = 1075 - ex;
        }
        if (q < 100) {
            unsigned __int128 num = (unsigned __int128)m * 10000u;
            unsigned __int128 kk = num >> q;
            unsigned __int128 rem = num - (kk << q);
            unsigned __int128 half = (unsigned __int128)1 << (q - 1);
            if (rem > half || (rem == half && (kk & 1))) kk += 1;
            k = (uint32_t)kk;
        }
    }
    o[0] = (char)('0' + k / 10000u);
    o[1] = '.';
    const uint32_t f = k % 10000u;
    o[2] = (char)('0' + f / 1000u);
    o[3] = (char)('0' + (f / 100u) % 10u);
    o[4] = (char)('0' + (f / 10u) % 10u);
    o[5] = (char)('0' + f % 10u);
}

// gate = computeRsqFast (mmap) vs computeRsq (stdin); printf4 = setprecision(4) vs formatR2
__global__ __launch_bounds__(256) void k_ld_matrix(const int8_t *__restrict__ Gc, const LdVar *__restrict__ vars,
                                                   uint64_t m, int kpad, int ns, int gate, int printf4,
                                                   const uint32_t *__restrict__ blocks, char *__restrict__ cells) {
    const int w = threadIdx.x / kWave;
    const int it = w >> 1, jt = w & 1;
    const uint32_t bI = blocks[2 * blockIdx.x], bJ = blocks[2 * blockIdx.x + 1];
    const int64_t i0 = (int64_t)bI * kBM + it * 32, j0 = (int64_t)bJ * kBM + jt * 32;
    const int l = lane(), r = l & 31, h = l >> 5;
    const int64_t M = (int64_t)m;
    TileSums T;
    tile_sums(Gc, vars, M, kpad, ns, i0, j0, T);
    const int64_t j = j0 + r;
    if (j >= M) return;
    const LdVar vj = vars[j];
    const uint64_t stride = 7ull * (uint64_t)M;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int64_t i = i0 + (k & 3) + 8 * (k >> 2) + 4 * h;
        if (i >= j) continue;
        const LdVar vi = vars[i];
        double rr;
        if (T.comp) rr = rsq_epilogue(vi, vj, ns, vi.sx, vj.sx, T.xx[k], vi.sx2, vj.sx2, gate);
        else rr = rsq_epilogue(vi, vj, T.vv[k], T.xv[k], T.vx[k], T.xx[k], T.x2v[k], T.vx2[k], gate);
        char c6[6];
        if (printf4) fmt_printf4(c6, rr);
        else fmt_r2(c6, rr);
        char *a = cells + (uint64_t)i * stride + 7ull * (uint64_t)j;
        char *b = cells + (uint64_t)j * stride + 7ull * (uint64_t)i;
        a[0] = b[0] = '\t';
#pragma unroll
        for (int q = 0; q < 6; q++) a[q + 1] = b[q + 1] = c6[q];
    }
}

__global__ void k_ld_matrix_diag(uint64_t m, char *__restrict__ cells) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += gridDim.x * (uint64_t)blockDim.x) {
        char *a = cells + i * 7ull * m + 7ull * i;
        a[0] = '\t'; a[1] = '1'; a[2] = '.'; a[3] = '0'; a[4] = '0'; a[5] = '0'; a[6] = '0';
    }
}

// ---------------------------------------------------------------------------------------
// text: per-variant "chrom\tpos\tid" prefixes, then pair lines
// ---------------------------------------------------------------------------------------
__global__ void k_ld_prefix_len(const LdVar *__restrict__ vars, uint64_t m, const char *__restrict__ buf,
                                int id_dot_to_pos, uint64_t *__restrict__ len) {
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < m; v += gridDim.x * (uint64_t)blockDim.x) {
        const LdVar x = vars[v];
        uint64_t L = x.chrom_len + 1 + int_len(x.pos) + 1;
        if (id_dot_to_pos && x.id_len == 1 && buf[x.id] == '.') L += x.chrom_len + 1 + int_len(x.pos);
        else L += x.id_len;
        len[v] = L;
    }
}
__global__ void k_ld_prefix_write(const LdVar *__restrict__ vars, uint64_t m, const char *__restrict__ buf,
                                  int id_dot_to_pos, const uint64_t *__restrict__ off, char *__restrict__ out) {
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < m; v += gridDim.x * (uint64_t)blockDim.x) {
        const LdVar x = vars[v];
        char *o = out + off[v];
        for (uint32_t k = 0; k < x.chrom_len; k++) *o++ = buf[x.chrom + k];
        *o++ = '\t';
        o = put_int(o, x.pos);
        *o++ = '\t';
        if (id_dot_to_pos && x.id_len == 1 && buf[x.id] == '.') {
            for (uint32_t k = 0; k < x.chrom_len; k++) *o++ = buf[x.chrom + k];
            *o++ = ':';
            o = put_int(o, x.pos);
        } else
            for (uint32_t k = 0; k < x.id_len; k++) *o++ = buf[x.id + k];
    }
}

__global__ void k_ld_pairlen(const LdPair *__restrict__ pairs, uint64_t np, const uint64_t *__restrict__ poff,
                             uint64_t *__restrict__ len) {
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < np; p += gridDim.x * (uint64_t)blockDim.x) {
        const LdPair x = pairs[p];
        len[p] = (poff[x.i + 1] - poff[x.i]) + (poff[x.j + 1] - poff[x.j]) + 9;
    }
}

// formatR2 (:200-211)
__device__ void fmt_r2(char *o, double r2) {
    if (r2 <= 0.0) {
        o[0] = '0'; o[1] = '.'; o[2] = '0'; o[3] = '0'; o[4] = '0'; o[5] = '0';
        return;
    }
    if (r2 >= 1.0) {
        o[0] = '1'; o[1] = '.'; o[2] = '0'; o[3] = '0'; o[4] = '0'; o[5] = '0';
        return;
    }
    int v = (int)__dadd_rn(__dmul_rn(r2, 10000.0), 0.5);
    if (v > 9999) v = 9999;
    o[0] = '0';
    o[1] = '.';
    o[5] = (char)('0' + v % 10); v /= 10;
    o[4] = (char)('0' + v % 10); v /= 10;
    o[3] = (char)('0' + v % 10); v /= 10;
    o[2] = (char)('0' + v % 10);
}

// pair lines, 64 per wave: the wave's lines are contiguous in the text, so they are composed
// in the wave's LDS tile (at their text position mod 16) and leave as aligned 16 B stores (the
// tile's partial first and last blocks byte by byte: their other bytes belong to the
// neighbouring waves); a wave whose lines exceed the tile writes each line straight out
constexpr int kPwTile = 8192;
__global__ __launch_bounds__(256) void k_ld_pairwrite(const LdPair *__restrict__ pairs, uint64_t np,
                                                      const uint64_t *__restrict__ poff,
                                                      const char *__restrict__ prefix,
                                                      const uint64_t *__restrict__ toff, char *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) char tile_all[4][kPwTile + 16];
    char *tile = tile_all[threadIdx.x / kWave];
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
    for (uint64_t p0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave * kWave; p0 < np;
         p0 += nw * kWave) {
        const uint64_t p = p0 + lane();
        const bool ok = p < np;
        LdPair x{};
        uint64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0, t = 0;
        if (ok) {
            x = pairs[p];
            a0 = poff[x.i], a1 = poff[x.i + 1], b0 = poff[x.j], b1 = poff[x.j + 1];
            t = toff[p];
        }
        const uint64_t len = ok ? (a1 - a0) + 1 + (b1 - b0) + 1 + 7 : 0;
        const uint64_t g0 = wave_bcast(t, 0);
        const int last = (int)(np - 1 - p0 < (uint64_t)kWave - 1 ? np - 1 - p0 : (uint64_t)kWave - 1);
        const uint64_t B = wave_bcast(t + len, last) - g0;  // (the lines are contiguous)
        auto line = [&](char *o) {
            for (uint64_t k = a0; k < a1; k++) *o++ = prefix[k];
            *o++ = '\t';
            for (uint64_t k = b0; k < b1; k++) *o++ = prefix[k];
            *o++ = '\t';
            fmt_r2(o, x.r2);
            o[6] = '\n';
        };
        if (B + 16 > (uint64_t)kPwTile) {  // (wave-uniform) long lines: straight out
            if (ok) line(out + t);
            continue;
        }
        const uint32_t sh = (uint32_t)(g0 & 15);  // tile byte sh + q = text byte g0 + q
        if (ok) line(tile + sh + (t - g0));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // text bytes [g0, g0 + B): aligned blocks [A0, A1) whole, the rest byte by byte
        const uint64_t ge = g0 + B, A0 = (g0 + 15) & ~(uint64_t)15, A1 = ge & ~(uint64_t)15;
        if (A0 >= A1) {
            for (uint64_t q = g0 + lane(); q < ge; q += kWave) out[q] = tile[sh + (q - g0)];
        } else {
            for (uint64_t q = g0 + lane(); q < A0; q += kWave) out[q] = tile[sh + (q - g0)];
            for (uint64_t q = A0 + 16u * lane(); q < A1; q += 16u * kWave)
                *reinterpret_cast<uint4 *>(out + q) = *reinterpret_cast<const uint4 *>(tile + sh + (q - g0));
            for (uint64_t q = A1 + lane(); q < ge; q += kWave) out[q] = tile[sh + (q - g0)];
        }
        // the next group's composition must not pass these reads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------------------
// self-test of the i8 MFMA operand layout: C = A (32x32) . B^T (32x32) over K = 32
// ---------------------------------------------------------------------------------------
__global__ void k_mfma_i8_selftest(const int8_t *A, const int8_t *B, int *C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    v4i a = *reinterpret_cast<const v4i *>(A + r * 32 + 16 * h);
    v4i b = *reinterpret_cast<const v4i *>(B + r * 32 + 16 * h);
    v16i c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int k = 0; k < 16; k++) C[((k & 3) + 8 * (k >> 2) + 4 * h) * 32 + r] = c[k];
}

// =======================================================================================
static unsigned gridfor(uint64_t n, uint64_t per, unsigned cap) {
    uint64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

hipError_t launch_ld_parse(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, const LdParseArgs &a, int8_t *G, LdLine *lines, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_ld_parse, dim3(gridfor(n_lines_host, 4, 8192)), dim3(256), 0, s, buf, data_start, line_end,
                       n_lines_dev, a, G, lines);
    return hipGetLastError();
}
hipError_t launch_ld_walk(const char *buf, int64_t lo, int64_t hi, int64_t chunk, int64_t span0, uint64_t cap_w,
                          const LdParseArgs &a, int8_t *G, LdLine *lines, uint64_t *wcount, uint64_t *wvalid,
                          unsigned *overflow, unsigned long long *pend_n, uint64_t *pend, hipStream_t s) {
    if (hi <= lo || chunk <= 0 || a.ns > kLdLdsRow) return hipErrorInvalidValue;
    const int64_t nw = (hi - lo + chunk - 1) / chunk;
    const unsigned grid = (unsigned)((nw + kWalkWaves - 1) / kWalkWaves);
    if (a.has_region || a.stoi_mode)
        hipLaunchKernelGGL(k_ld_walk<true>, dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, span0, cap_w,
                           a, G, lines, wcount, wvalid, overflow, pend_n, pend);
    else
        hipLaunchKernelGGL(k_ld_walk<false>, dim3(grid), dim3(kWalkThreads), 0, s, buf, lo, hi, chunk, nw, span0, cap_w,
                           a, G, lines, wcount, wvalid, overflow, pend_n, pend);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the pending lines: a grid-stride loop over the device count (none: every wave exits)
    hipLaunchKernelGGL(k_ld_pending, dim3(256), dim3(256), 0, s, buf, a, cap_w, pend_n, pend, G, lines, wvalid);
    return hipGetLastError();
}
hipError_t launch_ld_wcompact(int64_t nw, uint64_t cap_w, const uint64_t *wcount, const uint64_t *vbase,
                              const LdLine *lines, int ns, const char *buf, int id_dot_to_pos, LdVar *vars, LdFast *fv,
                              uint64_t *plen, unsigned *flags, uint64_t *m_out, hipStream_t s) {
    if (nw <= 0) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<int64_t>((nw + 3) / 4, 4096);
    hipLaunchKernelGGL(k_ld_wcompact, dim3(grid), dim3(256), 0, s, nw, cap_w, wcount, vbase, lines, ns, buf,
                       id_dot_to_pos, vars, fv, plen, flags, m_out);
    return hipGetLastError();
}
hipError_t launch_ld_gather(const LdVar *vars, uint64_t m, const int8_t *G, int kpad, int8_t *Gc, hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_ld_gather, dim3(gridfor(m, 1, 65536)), dim3(256), 0, s, vars, m, G, kpad, Gc);
    return hipGetLastError();
}
hipError_t launch_ld_compact(const LdLine *lines, const uint64_t *vidx, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int kpad, int ns, const int8_t *G, int8_t *Gc, LdVar *vars,
                             LdFast *fv, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_ld_compact, dim3(gridfor(n_lines_host, 1, 65536)), dim3(256), 0, s, lines, vidx, n_lines_dev,
                       kpad, ns, G, Gc, vars, fv);
    return hipGetLastError();
}
hipError_t launch_ld_block(int pass, const int8_t *Gc, const LdVar *vars, const uint32_t *chrom_id,
                           const LdWindowArgs &a, const uint32_t *blocks, uint32_t nblocks, uint16_t *cnt,
                           LdOffsets off, LdPair *pairs, hipStream_t s) {
    if (!nblocks) return hipSuccess;
    if (pass == 1)
        hipLaunchKernelGGL(k_ld_block<1>, dim3(nblocks), dim3(256), 0, s, Gc, vars, chrom_id, a, blocks, cnt, off,
                           pairs);
    else
        hipLaunchKernelGGL(k_ld_block<2>, dim3(nblocks), dim3(256), 0, s, Gc, vars, chrom_id, a, blocks, cnt, off,
                           pairs);
    return hipGetLastError();
}
hipError_t launch_ld_prefix(int which, const LdVar *vars, uint64_t m, const char *buf, int id_dot_to_pos,
                            uint64_t *len_or_off, char *out, hipStream_t s) {
    if (!m) return hipSuccess;
    if (which == 0)
        hipLaunchKernelGGL(k_ld_prefix_len, dim3(gridfor(m, 256, 4096)), dim3(256), 0, s, vars, m, buf, id_dot_to_pos,
                           len_or_off);
    else
        hipLaunchKernelGGL(k_ld_prefix_write, dim3(gridfor(m, 256, 4096)), dim3(256), 0, s, vars, m, buf,
                           id_dot_to_pos, len_or_off, out);
    return hipGetLastError();
}
hipError_t launch_ld_pairtext(int which, const LdPair *pairs, uint64_t np, const uint64_t *poff, const char *prefix,
                              uint64_t *len_or_off, char *out, hipStream_t s) {
    if (!np) return hipSuccess;
    if (which == 0)
        hipLaunchKernelGGL(k_ld_pairlen, dim3(gridfor(np, 256, 8192)), dim3(256), 0, s, pairs, np, poff, len_or_off);
    else
        hipLaunchKernelGGL(k_ld_pairwrite, dim3(gridfor(np, 256, 16384)), dim3(256), 0, s, pairs, np, poff, prefix,
                           len_or_off, out);
    return hipGetLastError();
}
hipError_t launch_ld_matrix(const int8_t *Gc, const LdVar *vars, uint64_t m, int kpad, int ns, int gate, int printf4,
                            const uint32_t *blocks, uint32_t nblocks, char *cells, hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_ld_matrix_diag, dim3(gridfor(m, 256, 4096)), dim3(256), 0, s, m, cells);
    if (nblocks)
        hipLaunchKernelGGL(k_ld_matrix, dim3(nblocks), dim3(256), 0, s, Gc, vars, m, kpad, ns, gate, printf4, blocks,
                           cells);
    return hipGetLastError();
}
hipError_t launch_mfma_i8_selftest(const int8_t *A, const int8_t *B, int *C, hipStream_t s) {
    hipLaunchKernelGGL(k_mfma_i8_selftest, dim3(1), dim3(64), 0, s, A, B, C);
    return hipGetLastError();
}

}  // namespace vcfxg
