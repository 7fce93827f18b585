// vcfxg_kernels.hip -- record kernels of the MI355X VCF engine (gfx950).
//
// K1 line index  : two HBM sweeps (count, emit) -> line end offsets.
// K2 AF records  : one wave per record; fixed-stride "a|b\t" fast path (SWAR on 16 B per
//                  lane, validated per record) with an exact general per-sample fallback.
// K5 AF rows     : row length -> exclusive scan -> device-formatted text rows.
//
// Reference behaviour restated: VCFX_allele_freq_calc.cpp (citations per function).
#include "vcfxg_device.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

// =======================================================================================
// K1: line index
// =======================================================================================
constexpr int kIdxThreads = 256;
constexpr int64_t kIdxChunk = 64 * 1024;  // bytes per block
constexpr int kIdxTile = kIdxThreads * kBlockBytes;

__global__ __launch_bounds__(kIdxThreads) void k_nl_count(const char *__restrict__ buf, int64_t lo, int64_t hi,
                                                           int64_t nchunks, uint32_t *__restrict__ counts) {
    int64_t a0 = lo & ~(int64_t)15;
    for (int64_t b = blockIdx.x; b < nchunks; b += gridDim.x) {
        int64_t base = a0 + b * kIdxChunk;
        uint32_t c = 0;
#pragma unroll 4
        for (int t = 0; t < kIdxChunk / kIdxTile; t++) {
            int64_t blk = base + (int64_t)t * kIdxTile + (int64_t)threadIdx.x * kBlockBytes;
            if (blk < hi) c += __popc(eq_mask16(load16(buf, blk), kRepNl) & range_mask16(blk, lo, hi));
        }
        c = wave_sum(c);
        __shared__ uint32_t part[kIdxThreads / kWave];
        if (lane() == 0) part[threadIdx.x / kWave] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t s = 0;
            for (int w = 0; w < kIdxThreads / kWave; w++) s += part[w];
            counts[b] = s;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kIdxThreads) void k_nl_emit(const char *__restrict__ buf, int64_t lo, int64_t hi,
                                                          int64_t nchunks, const uint64_t *__restrict__ offs,
                                                          uint64_t *__restrict__ line_end, uint64_t cap) {
    __shared__ uint32_t wtot[kIdxThreads / kWave];
    int64_t a0 = lo & ~(int64_t)15;
    for (int64_t b = blockIdx.x; b < nchunks; b += gridDim.x) {
        int64_t base = a0 + b * kIdxChunk;
        uint64_t run = offs[b];
        for (int t = 0; t < kIdxChunk / kIdxTile; t++) {
            int64_t blk = base + (int64_t)t * kIdxTile + (int64_t)threadIdx.x * kBlockBytes;
            uint32_t m = 0;
            if (blk < hi) m = eq_mask16(load16(buf, blk), kRepNl) & range_mask16(blk, lo, hi);
            uint32_t c = __popc(m);
            uint32_t incl = wave_incl_scan(c);
            if (lane() == kWave - 1) wtot[threadIdx.x / kWave] = incl;
            __syncthreads();
            uint32_t wbase = 0, btot = 0;
            for (int w = 0; w < kIdxThreads / kWave; w++) {
                uint32_t x = wtot[w];
                if (w < (int)(threadIdx.x / kWave)) wbase += x;
                btot += x;
            }
            uint64_t idx = run + wbase + (incl - c);
            while (m) {
                int j = __builtin_ctz(m);
                m &= m - 1u;
                if (idx < cap) line_end[idx] = (uint64_t)(blk + j);
                idx++;
            }
            run += btot;
            __syncthreads();
        }
    }
}

// =======================================================================================
// K2: allele frequency per record
// =======================================================================================
// Fast path: the sample region [S, E) is N fixed 4-byte units "a s b \t" (last one without
// the tab), s == the record's first separator ('/' or '|'), a/b in [0-9.] -- the layout of
// phased/unphased single-digit diploid GT-only records (1000 Genomes).  Any deviation makes
// the record take af_general, which restates the reference loop per sample exactly.
// Sample dwords d = bytes [p, p+4) for p = S + 4k, built with v_alignbyte from the lane's
// 16 B block; per dword: e = d ^ (0x09 << 24 | sep << 8 | '0' << 16 | '0'):
//   bytes 1 and 3 must be 0 (sep, tab); bytes 0 and 2 in 0..9 (digit) or 0x1E ('.').
struct FastAcc {
    uint32_t alt, tot, err;
};

__device__ __forceinline__ void fast_dword(uint32_t d, uint32_t exp_xor, FastAcc &a) {
    uint32_t e = d ^ exp_xor;
    a.err |= e & 0xFF00FF00u;
    uint32_t f = e & 0x00FF00FFu;
    uint32_t notdig = (f + 0x00F600F6u) & 0x01000100u;          // field >= 10
    uint32_t dig = notdig ^ 0x01000100u;
    uint32_t nz = (f + 0x00FF00FFu) & dig;                        // 1..9
    uint32_t notdot = ((f ^ 0x001E001Eu) + 0x00FF00FFu) & 0x01000100u;
    a.err |= notdig & notdot;
    a.tot += __popc(dig);
    a.alt += __popc(nz);
}

// returns false (uniformly) if the record is not fixed-stride; otherwise alt/tot (uniform)
__device__ bool af_fast(const char *__restrict__ buf, int64_t S, int64_t E, int &alt_o, int &tot_o) {
    int64_t L = E - S;
    if (L < 3 || ((L + 1) & 3)) return false;
    uint32_t sepc = byte_at(buf, S + 1);
    if (sepc != '/' && sepc != '|') return false;
    const uint32_t exp_xor = 0x09000000u | (sepc << 8) | 0x00300030u;
    const uint32_t neutral = 0x092E002Eu | (sepc << 8);  // ". ." with tab: counts 0, valid
    const int s = (int)(S & 3);
    const int64_t b0 = S & ~(int64_t)15;
    FastAcc a = {0, 0, 0};
    for (int64_t w = b0; w < E; w += kWaveStep) {
        const int64_t blk = w + (int64_t)lane() * kBlockBytes;
        // interior step: every sample dword of every lane lies in [S, E) and is not last
        const bool interior = (w + s >= S) && (w + kWaveStep - 4 + s + 3 < E);
        if (blk < E + 4) {
            uint4 v = load16(buf, blk);
            uint32_t x4 = load4(buf, blk + 16);
            uint32_t d0 = __builtin_amdgcn_alignbyte(v.y, v.x, s);
            uint32_t d1 = __builtin_amdgcn_alignbyte(v.z, v.y, s);
            uint32_t d2 = __builtin_amdgcn_alignbyte(v.w, v.z, s);
            uint32_t d3 = __builtin_amdgcn_alignbyte(x4, v.w, s);
            if (!interior) {
                uint32_t dd[4] = {d0, d1, d2, d3};
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    int64_t p = blk + s + 4 * i;
                    if (p < S || p + 3 > E) dd[i] = neutral;
                    else if (p + 3 == E) dd[i] = (dd[i] & 0x00FFFFFFu) | 0x09000000u;
                }
                d0 = dd[0]; d1 = dd[1]; d2 = dd[2]; d3 = dd[3];
            }
            fast_dword(d0, exp_xor, a);
            fast_dword(d1, exp_xor, a);
            fast_dword(d2, exp_xor, a);
            fast_dword(d3, exp_xor, a);
        }
    }
    if (__any(a.err != 0u)) return false;
    alt_o = wave_sum((int)a.alt);
    tot_o = wave_sum((int)a.tot);
    return true;
}

// parseGenotypeAndCount (VCFX_allele_freq_calc.cpp:262-293) over the GT sub-field
// (extractGT :321-337) of the sample starting at st; the sample ends at '\t' or E.
__device__ void af_sample(const char *__restrict__ buf, int64_t st, int64_t E, int gi, int &alt, int &tot) {
    int64_t p = st;
    // skip gi colon fields
    for (int k = 0; k < gi; k++) {
        while (p < E) {
            uint32_t c = byte_at(buf, p);
            if (c == '\t' || c == ':') break;
            p++;
        }
        if (p >= E || byte_at(buf, p) == '\t') return;  // fewer sub-fields: empty GT
        p++;                                            // skip ':'
    }
    // GT = [p, first of ':' '\t' E)
    bool in_tok = false, first_dot = false, numeric = true, nonzero = false;
    for (;; p++) {
        uint32_t c = p < E ? byte_at(buf, p) : (uint32_t)'\t';
        bool end = (c == '\t' || c == ':');
        bool sep = end || c == '/' || c == '|';
        if (sep) {
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

// general path: one lane per sample start (S, and every tab+1 < E) in its 16 B block
__device__ void af_general(const char *__restrict__ buf, int64_t S, int64_t E, int gi, int &alt_o, int &tot_o) {
    int alt = 0, tot = 0;
    for (int64_t w = S & ~(int64_t)15; w < E; w += kWaveStep) {
        int64_t blk = w + (int64_t)lane() * kBlockBytes;
        if (blk < E) {
            uint32_t tm = eq_mask16(load16(buf, blk), kRepTab);
            uint32_t starts = (tm << 1) & 0xFFFFu;
            if (blk > 0 && byte_at(buf, blk - 1) == '\t') starts |= 1u;
            starts &= range_mask16(blk, S + 1, E);  // starts after tabs: S < st < E
            if (S >= blk && S < blk + 16) starts |= 1u << (S - blk);
            while (starts) {
                int j = __builtin_ctz(starts);
                starts &= starts - 1u;
                af_sample(buf, blk + j, E, gi, alt, tot);
            }
        }
    }
    alt_o = wave_sum(alt);
    tot_o = wave_sum(tot);
}

// one wave per line of the indexed region; writes per-line status/alt/tot/row prefix len
__global__ __launch_bounds__(256) void k_af_records(const char *__restrict__ buf, int64_t data_start,
                                                    const uint64_t *__restrict__ line_end, const uint64_t *n_lines_p,
                                                    int mode, int32_t *__restrict__ alt_o, int32_t *__restrict__ tot_o,
                                                    uint32_t *__restrict__ rowpre_o, uint8_t *__restrict__ status_o,
                                                    unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[256 / kWave][16];
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave;
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    uint32_t c_rows = 0, c_data = 0, c_warn = 0, c_gen = 0;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
        const int64_t le = (int64_t)line_end[li];
        int64_t ae = le;
        if (mode == 0 && ae > ls && byte_at(buf, ae - 1) == '\r') ae--;  // processMmap :362-364
        uint8_t st = 0;
        int alt = 0, tot = 0;
        uint32_t rowpre = 0;
        if (ae > ls && byte_at(buf, ls) != '#') {
            c_data++;
            int64_t t[10];
            int nt = head_tabs(buf, ls, ae, 10, t, lds);
            bool ok = true;
            int64_t fs = 0, fe = 0;
            if (mode == 0) {
                // getField(8) non-empty (processMmap :391-401)
                if (nt < 8) ok = false;
                else {
                    fs = t[7] + 1;
                    fe = nt >= 9 ? t[8] : ae;
                    if (fe <= fs) ok = false;
                }
            } else {
                // processStdin :509-523: fields = tabs + (last char != '\t')
                int nf = nt + ((byte_at(buf, ae - 1) != '\t') ? 1 : 0);
                if (nt >= 9) nf = 10;
                if (nf < 9) { st = 3; ok = false; }
                else { fs = t[7] + 1; fe = nt >= 9 ? t[8] : ae; }
            }
            if (ok) {
                int gi = gt_index(buf, fs, fe);
                if (gi >= 0) {
                    if (nt >= 9) {
                        int64_t S = t[8] + 1;
                        bool fast = gi == 0 && af_fast(buf, S, ae, alt, tot);
                        if (!fast) {
                            af_general(buf, S, ae, gi, alt, tot);
                            c_gen++;
                        }
                    }
                    st = 1;
                    rowpre = (uint32_t)(t[4] - ls + 1);
                }
            }
        }
        if (lane() == 0) {
            status_o[li] = st;
            alt_o[li] = alt;
            tot_o[li] = tot;
            rowpre_o[li] = rowpre;
        }
        c_rows += st == 1;
        c_warn += st == 3;
    }
    if (lane() == 0 && (c_rows | c_data | c_warn | c_gen)) {
        atomicAdd(&counters[0], (unsigned long long)c_rows);
        atomicAdd(&counters[1], (unsigned long long)c_data);
        atomicAdd(&counters[2], (unsigned long long)c_warn);
        atomicAdd(&counters[3], (unsigned long long)c_gen);
    }
}

// =======================================================================================
// K5: AF rows
// =======================================================================================
__global__ void k_af_rowlen(const uint32_t *__restrict__ rowpre, const uint8_t *__restrict__ status,
                            const uint64_t *n_lines_p, uint64_t *__restrict__ len) {
    const uint64_t n = *n_lines_p;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gridDim.x * (uint64_t)blockDim.x)
        len[i] = status[i] == 1 ? (uint64_t)rowpre[i] + 7u : 0u;
}

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

__global__ void k_af_format(const char *__restrict__ buf, int64_t data_start, const uint64_t *__restrict__ line_end,
                            const uint64_t *n_lines_p, int mode, const int32_t *__restrict__ alt,
                            const int32_t *__restrict__ tot, const uint32_t *__restrict__ rowpre,
                            const uint8_t *__restrict__ status, const uint64_t *__restrict__ off,
                            char *__restrict__ out) {
    const uint64_t n = *n_lines_p;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gridDim.x * (uint64_t)blockDim.x) {
        if (status[i] != 1) continue;
        const int64_t ls = i ? (int64_t)line_end[i - 1] + 1 : data_start;
        char *o = out + off[i];
        const uint32_t pl = rowpre[i];
        for (uint32_t k = 0; k < pl; k++) o[k] = buf[ls + k];
        const int a = alt[i], t = tot[i];
        const double f = t > 0 ? __ddiv_rn((double)a, (double)t) : 0.0;
        const uint32_t k4 = mode == 0 ? fixed4_mmap(f) : fixed4_printf(f);
        const uint32_t ip = k4 / 10000u, fp = k4 % 10000u;
        o += pl;
        o[0] = (char)('0' + ip);  // freq <= 1
        o[1] = '.';
        o[2] = (char)('0' + fp / 1000u);
        o[3] = (char)('0' + (fp / 100u) % 10u);
        o[4] = (char)('0' + (fp / 10u) % 10u);
        o[5] = (char)('0' + fp % 10u);
        o[6] = '\n';
    }
}

// =======================================================================================
// launchers
// =======================================================================================
int64_t idx_nchunks(int64_t lo, int64_t hi) {
    int64_t a0 = lo & ~(int64_t)15;
    return hi > lo ? (hi - a0 + kIdxChunk - 1) / kIdxChunk : 0;
}
static unsigned grid_for(int64_t n, int64_t per, unsigned cap) {
    int64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

hipError_t launch_nl_count(const char *buf, int64_t lo, int64_t hi, uint32_t *counts, hipStream_t s) {
    int64_t nc = idx_nchunks(lo, hi);
    if (!nc) return hipSuccess;
    hipLaunchKernelGGL(k_nl_count, dim3(grid_for(nc, 1, 1u << 20)), dim3(kIdxThreads), 0, s, buf, lo, hi, nc, counts);
    return hipGetLastError();
}
hipError_t launch_nl_emit(const char *buf, int64_t lo, int64_t hi, const uint64_t *offs, uint64_t *line_end,
                          uint64_t cap, hipStream_t s) {
    int64_t nc = idx_nchunks(lo, hi);
    if (!nc) return hipSuccess;
    hipLaunchKernelGGL(k_nl_emit, dim3(grid_for(nc, 1, 1u << 20)), dim3(kIdxThreads), 0, s, buf, lo, hi, nc, offs,
                       line_end, cap);
    return hipGetLastError();
}
hipError_t launch_af_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int mode, int32_t *alt, int32_t *tot, uint32_t *rowpre,
                             uint8_t *status, unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    unsigned grid = grid_for((int64_t)n_lines_host, 4, 65536);
    hipLaunchKernelGGL(k_af_records, dim3(grid), dim3(256), 0, s, buf, data_start, line_end, n_lines_dev, mode, alt,
                       tot, rowpre, status, counters);
    return hipGetLastError();
}
hipError_t launch_af_rowlen(const uint32_t *rowpre, const uint8_t *status, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, uint64_t *len, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_af_rowlen, dim3(grid_for((int64_t)n_lines_host, 256, 4096)), dim3(256), 0, s, rowpre, status,
                       n_lines_dev, len);
    return hipGetLastError();
}
hipError_t launch_af_format(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, int mode, const int32_t *alt, const int32_t *tot,
                            const uint32_t *rowpre, const uint8_t *status, const uint64_t *off, char *out,
                            hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_af_format, dim3(grid_for((int64_t)n_lines_host, 256, 4096)), dim3(256), 0, s, buf, data_start,
                       line_end, n_lines_dev, mode, alt, tot, rowpre, status, off, out);
    return hipGetLastError();
}

}  // namespace vcfxg
