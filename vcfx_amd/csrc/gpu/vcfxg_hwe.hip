// vcfxg_hwe.hip -- VCFX_hwe_tester's per-record pass (another per-sample
// GT reducer on the record path).
//
// Counting: the AF walk (vcfxg_af_walk.hip) with the HweOp reducer gives each fixed-stride
// GT record its (hom-ref, het, hom-alt) counts in the same single HBM pass; k_hwe_lines runs
// hwe_line, the exact per-line restatement, on everything else (and on every line of the
// two-sweep schedule for short records).  The row rules on CHROM..ALT come from the walk's head
// window (or hwe_line), k_hwe_rowlen + a scan give row offsets, and k_hwe_format writes the rows
// "CHROM\tPOS\tID\tREF\tALT\t<p>\n" with <p> in the mode's 6-digit format.
//
// Exactness: the p-value (calculateHWE_chisq / chi2_pvalue_1df, VCFX_hwe_tester.cpp:278-315)
// is the reference's fp64 operation sequence in correctly rounded ops, except exp(), whose
// device implementation may differ from the host libm's in the last bits.  The printed
// digits are a monotone function of the value, so a row is certain when the values kUlps
// units in the last place below and above the device value print the same; the (very rare)
// rows that do not are listed for the host, which recomputes them with its libm exp
// (vcfxg_hwe_rechecks) and overwrites their 8 digit bytes in place.
#include <algorithm>

#include "vcfx_gpu.h"
#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

constexpr int kHweThreads = 256;
constexpr int kHweWaves = kHweThreads / kWave;

// One line [ls, le) in mode 0 (performHWE_Mmap :475-558) or 1 (performHWE_Stdin :572-607):
// status 1 = row, 0 = skipped.
// Both modes drop one trailing '\r' and skip empty and '#' lines.  Both need >= 9 tabs
// (mmap: getField(8) + skipToField(9); stdin: >= 10 split_tabs fields) and a FORMAT that
// starts with "GT"; mmap also a non-empty sample region.  Every tab-separated sample of
// [S, ae) is parsed (stdin's trailing empty field parses as invalid, as in split_tabs).
__device__ __forceinline__ void hwe_line(const char *__restrict__ buf, int64_t ls, int64_t le, int mode, int64_t *lds,
                                         uint8_t &st, uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &rowpre,
                                         bool &general) {
    st = 0;
    c0 = c1 = c2 = rowpre = 0;
    general = false;
    int64_t ae = le;
    if (ae > ls && byte_at(buf, ae - 1) == '\r') ae--;
    if (ae <= ls || byte_at(buf, ls) == '#') return;
    int64_t t[10];
    const int nt = head_tabs(buf, ls, ae, 10, t, lds);
    if (nt < 9) return;
    if (t[8] - t[7] - 1 < 2 || byte_at(buf, t[7] + 1) != 'G' || byte_at(buf, t[7] + 2) != 'T') return;
    const int64_t S = t[8] + 1;
    if (mode == 0 && S >= ae) return;
    // CHROM..ALT: ALT without ',' (both modes); CHROM, POS, ALT non-empty (mmap :497)
    if (mode == 0 && (t[0] == ls || t[1] == t[0] + 1 || t[4] == t[3] + 1)) return;
    for (int64_t w = t[3] + 1; w < t[4]; w += kWave) {
        const int64_t p = w + lane();
        if (__ballot(p < t[4] && byte_at(buf, p) == ',')) return;
    }
    HweOp op{buf, ae};
    if (!gt_fast(buf, S, ae, op)) {
        op = HweOp{buf, ae};
        if (!gt_first_known(buf, S, ae, op)) {  // (every sample's first sub-field is its GT)
            op = HweOp{buf, ae};
            gt_general(buf, S, ae, op);
        }
        general = true;
    }
    st = 1;
    c0 = op.c0;
    c1 = op.c1;
    c2 = op.c2;
    rowpre = (uint32_t)(t[4] - ls + 1);
}

// meta == nullptr: every line [0, n) (two-sweep schedule); else the lines the walk left:
// kind kMetaFull and status kAfPending.  counters[3] += lines off the fixed-stride sweep.
__global__ __launch_bounds__(kHweThreads) void k_hwe_lines(const char *__restrict__ buf, int64_t data_start,
                                                           const uint64_t *__restrict__ line_end,
                                                           const uint64_t *n_lines_p, int mode,
                                                           const LineMeta *__restrict__ meta,
                                                           int32_t *__restrict__ c0_o, int32_t *__restrict__ c1_o,
                                                           int32_t *__restrict__ c2_o, uint32_t *__restrict__ rowpre_o,
                                                           uint8_t *__restrict__ status_o,
                                                           unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kHweWaves][16];
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    uint32_t ngen = 0;
    for (uint64_t l0 = wid * kWave; l0 < n_lines; l0 += nw * kWave) {
        const uint64_t mine = l0 + lane();
        bool todo_me = mine < n_lines;
        if (meta && todo_me) todo_me = meta[mine].kind == kMetaFull || status_o[mine] == kAfPending;
        uint64_t todo = __ballot(todo_me);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1ull;
            const uint64_t li = l0 + k;
            const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start, le = (int64_t)line_end[li];
            uint8_t st;
            uint32_t a, b, c, rp;
            bool gen;
            hwe_line(buf, ls, le, mode, lds, st, a, b, c, rp, gen);
            ngen += gen ? 1u : 0u;
            if (lane() == 0) {
                status_o[li] = st;
                c0_o[li] = (int32_t)a;
                c1_o[li] = (int32_t)b;
                c2_o[li] = (int32_t)c;
                rowpre_o[li] = rp;
            }
        }
    }
    if (lane() == 0 && ngen) atomicAdd(&counters[3], (unsigned long long)ngen);
}

// Row lengths (prefix + 8 digits + '\n', or 0).  The rules on CHROM..ALT were applied by
// hwe_line, or for the walk's kMetaGt lines (meta != nullptr) come as the flags the walk took
// from its head window: ALT holds a ',' (isBiallelic :380-382, both modes) or CHROM, POS or ALT
// is empty (mmap :497).  A rejected line's status becomes 0; counters[0] += rows.
__global__ void k_hwe_rowlen(const uint64_t *n_lines_p, int mode, const LineMeta *__restrict__ meta,
                             const uint32_t *__restrict__ rowpre, uint8_t *__restrict__ status,
                             uint64_t *__restrict__ len, unsigned long long *__restrict__ counters) {
    const uint64_t n = *n_lines_p;
    uint32_t rows = 0;
    const uint8_t reject = mode == 0 ? (kHweAltComma | kHweEmptyField) : kHweAltComma;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gridDim.x * (uint64_t)blockDim.x) {
        uint64_t l = 0;
        if (status[i] == 1) {
            bool ok = true;
            if (meta) {
                const LineMeta m = meta[i];
                ok = m.kind != kMetaGt || (m.pad & reject) == 0;
            }
            if (ok) {
                l = (uint64_t)rowpre[i] + 9u;
                rows++;
            } else status[i] = 0;
        }
        len[i] = l;
    }
    // one atomic per block (same-address atomics serialise in L2: one per wave cost ~80 us)
    __shared__ uint32_t red[256 / kWave];
    rows = wave_sum(rows);
    if (lane() == 0) red[threadIdx.x / kWave] = rows;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < 256 / kWave; k++) t += red[k];
        if (t) atomicAdd(&counters[0], (unsigned long long)t);
    }
}

// calculateHWE_chisq (:290-315) + chi2_pvalue_1df (:278-287): the reference's operation
// order in correctly rounded fp64 ops; exact = false when the value went through exp()
__device__ double hwe_pvalue(int32_t h0, int32_t h1, int32_t h2, bool &exact) {
    exact = true;
    const int32_t N = h0 + h1 + h2;
    if (N < 1) return 1.0;
    const double dN = (double)N;
    const double p = __ddiv_rn(__dadd_rn(__dmul_rn(2.0, (double)h0), (double)h1), __dmul_rn(2.0, dN));
    const double q = __dsub_rn(1.0, p);
    if (p <= 0.0 || p >= 1.0) return 1.0;
    const double ex[3] = {__dmul_rn(__dmul_rn(dN, p), p), __dmul_rn(__dmul_rn(__dmul_rn(dN, 2.0), p), q),
                          __dmul_rn(__dmul_rn(dN, q), q)};
    const double ob[3] = {(double)h0, (double)h1, (double)h2};
    double chi2 = 0.0;
    for (int k = 0; k < 3; k++) {
        double y = 0.0;
        if (ex[k] > 0.0) {
            double diff = __dsub_rn(fabs(__dsub_rn(ob[k], ex[k])), 0.5);
            if (diff < 0.0) diff = 0.0;
            y = __ddiv_rn(__dmul_rn(diff, diff), ex[k]);
        }
        chi2 = k == 0 ? y : __dadd_rn(chi2, y);
    }
    if (chi2 <= 0.0) return 1.0;
    if (chi2 > 700.0) return 0.0;
    const double x = __dsqrt_rn(__dmul_rn(chi2, 0.5));
    const double t = __ddiv_rn(1.0, __dadd_rn(1.0, __dmul_rn(0.3275911, x)));
    double y = __dadd_rn(-1.453152027, __dmul_rn(t, 1.061405429));
    y = __dadd_rn(1.421413741, __dmul_rn(t, y));
    y = __dadd_rn(-0.284496736, __dmul_rn(t, y));
    y = __dadd_rn(0.254829592, __dmul_rn(t, y));
    y = __dmul_rn(t, y);
    exact = false;
    return __dmul_rn(y, exp(-__dmul_rn(x, x)));
}

// OutputBuffer::appendDouble (:236-268) for 0 <= v < 10: integer digit, '.', 6 digits by
// repeated *10 and truncation
__device__ __forceinline__ void fmt6_trunc(double v, char *o) {
    const long long ip = (long long)v;
    double fr = __dsub_rn(v, (double)ip);
    o[0] = (char)('0' + ip);
    o[1] = '.';
    for (int k = 0; k < 6; k++) {
        fr = __dmul_rn(fr, 10.0);
        const int d = (int)fr;
        o[2 + k] = (char)('0' + d);
        fr = __dsub_rn(fr, (double)d);
    }
}

// std::fixed << setprecision(6) (glibc printf "%.6f": the exact binary value rounded half to
// even) for 0 <= v < 10
__device__ __forceinline__ void fmt6_printf(double v, char *o) {
    uint64_t k = 0;
    if (v != 0.0) {
        const uint64_t bits = (uint64_t)__double_as_longlong(v);
        const int ex = (int)((bits >> 52) & 0x7FF);
        uint64_t m = bits & ((1ull << 52) - 1);
        int q;  // v = m * 2^-q
        if (ex == 0) q = 1074;
        else {
            m |= 1ull << 52;
            q = 1075 - ex;
        }
        if (q <= 0) k = ~0ull;  // v >= 2^52 (only a far recheck neighbour): any mismatch will do
        else if (q < 100) {     // else v < 2^-46: rounds to 0
            const unsigned __int128 num = (unsigned __int128)m * 1000000u;
            unsigned __int128 kk = num >> q;
            const unsigned __int128 rem = num - (kk << q);
            const unsigned __int128 half = (unsigned __int128)1 << (q - 1);
            if (rem > half || (rem == half && (kk & 1))) kk += 1;
            k = (uint64_t)kk;
        }
    }
    const uint32_t ip = (uint32_t)(k / 1000000u), fp = (uint32_t)(k % 1000000u);
    o[0] = (char)('0' + ip);
    o[1] = '.';
    uint32_t d = 100000u;
    for (int j = 0; j < 6; j++, d /= 10u) o[2 + j] = (char)('0' + (fp / d) % 10u);
}

__device__ __forceinline__ void fmt6(int mode, double v, char *o) {
    if (mode == 0) fmt6_trunc(v, o);
    else fmt6_printf(v, o);
}

// one thread per line: the row of every status-1 line whose end fits the text capacity
__global__ void k_hwe_format(const char *__restrict__ buf, int64_t data_start, const uint64_t *__restrict__ line_end,
                             const uint64_t *n_lines_p, int mode, const int32_t *__restrict__ c0,
                             const int32_t *__restrict__ c1, const int32_t *__restrict__ c2,
                             const uint32_t *__restrict__ rowpre, const uint8_t *__restrict__ status,
                             const uint64_t *__restrict__ off, char *__restrict__ out, uint64_t cap, int64_t ulps,
                             vcfxg_hwe_recheck *__restrict__ rc, unsigned long long *rc_n, uint64_t rc_cap) {
    const uint64_t n = *n_lines_p;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gridDim.x * (uint64_t)blockDim.x) {
        if (status[i] != 1 || off[i + 1] > cap) continue;
        const int64_t ls = i ? (int64_t)line_end[i - 1] + 1 : data_start;
        char *o = out + off[i];
        const uint32_t pl = rowpre[i];
        for (uint32_t k = 0; k < pl; k++) o[k] = buf[ls + k];
        bool exact;
        const double v = hwe_pvalue(c0[i], c1[i], c2[i], exact);
        char d[8];
        fmt6(mode, v, d);
        if (!exact) {
            // v > 0 here: the neighbours kUlps representable values away, by bit pattern
            const int64_t b = __double_as_longlong(v);
            char lo[8], hi[8];
            fmt6(mode, __longlong_as_double(b - ulps > 0 ? b - ulps : 0), lo);
            fmt6(mode, __longlong_as_double(b + ulps), hi);
            bool same = true;
            for (int k = 0; k < 8; k++) same = same && lo[k] == hi[k];
            if (!same) {
                const unsigned long long r = atomicAdd(rc_n, 1ull);
                if (r < rc_cap) {
                    vcfxg_hwe_recheck e;
                    e.text_offset = off[i] + pl;
                    e.hom_ref = c0[i];
                    e.het = c1[i];
                    e.hom_alt = c2[i];
                    e.reserved = 0;
                    rc[r] = e;
                }
            }
        }
        for (int k = 0; k < 8; k++) o[pl + k] = d[k];
        o[pl + 8] = '\n';
    }
}

static unsigned grid_of(int64_t n, int64_t per, unsigned cap) {
    int64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

hipError_t launch_hwe_lines(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, int mode, const void *meta, int32_t *c0, int32_t *c1, int32_t *c2,
                            uint32_t *rowpre, uint8_t *status, unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    // a wave takes 64 lines per step; the walk's leftovers are few, every line otherwise
    const unsigned grid = grid_of((int64_t)((n_lines_host + kWave - 1) / kWave), kHweWaves, meta ? 1024 : 8192);
    hipLaunchKernelGGL(k_hwe_lines, dim3(grid), dim3(kHweThreads), 0, s, buf, data_start, line_end, n_lines_dev, mode,
                       static_cast<const LineMeta *>(meta), c0, c1, c2, rowpre, status, counters);
    return hipGetLastError();
}

hipError_t launch_hwe_rowlen(const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, const void *meta,
                             const uint32_t *rowpre, uint8_t *status, uint64_t *len, unsigned long long *counters,
                             hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_hwe_rowlen, dim3(grid_of((int64_t)n_lines_host, 256, 1024)), dim3(256), 0, s, n_lines_dev,
                       mode, static_cast<const LineMeta *>(meta), rowpre, status, len, counters);
    return hipGetLastError();
}

hipError_t launch_hwe_format(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int mode, const int32_t *c0, const int32_t *c1, const int32_t *c2,
                             const uint32_t *rowpre, const uint8_t *status, const uint64_t *off, char *out,
                             uint64_t text_cap, int64_t ulps, void *rc, unsigned long long *rc_n, uint64_t rc_cap,
                             hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_hwe_format, dim3(grid_of((int64_t)n_lines_host, 256, 4096)), dim3(256), 0, s, buf, data_start,
                       line_end, n_lines_dev, mode, c0, c1, c2, rowpre, status, off, out, text_cap, ulps,
                       static_cast<vcfxg_hwe_recheck *>(rc), rc_n, rc_cap);
    return hipGetLastError();
}

}  // namespace vcfxg
