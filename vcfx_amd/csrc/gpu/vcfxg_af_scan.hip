// vcfxg_af_scan.hip -- VCFX_allele_freq_calc in ONE sweep of the input.
//
// The fixed-stride fast path needs, per record, only byte-class statistics of its sample
// region [S, E): with s = S mod 4 the units "a sep b \t" put alleles in the absolute
// position classes s and s+2 (mod 4), the separator in s+1 and the tab in s+3.  So the
// sweep never needs S: one wave per 16 KiB chunk classifies every byte once (digit,
// non-zero digit, '.', '/', '|', tab) and accumulates per-class counts for each line
// segment of the chunk (segments end at newlines), while recording the chunk's newline
// offsets for the line index (the same chunk geometry as k_idx_sweep).  After the scan of
// the per-chunk newline counts, k_af_combine (one lane per line) parses the line head
// (tabs, FORMAT = GT..., row prefix, S), adds up the line's segments, subtracts the head
// bytes and decides exactly as gt_fast would: every unit valid <=> the class counts equal
// the unit counts; then alt = non-zero digit alleles, total = digit alleles
// (parseGenotypeAndCount, VCFX_allele_freq_calc.cpp:262-293, on the fixed layout).  Lines
// that are not GT-first / not fixed-stride go to k_af_complex (the exact general path).
#include "vcfxg_device.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

constexpr int kScanCap = 16;              // newline slots per chunk (as kPosCap)
constexpr int kSegSlots = kScanCap + 1;   // line segments per chunk
constexpr int64_t kScanChunk = 16 * 1024;
constexpr int kCats = 6;                  // tab, digit, non-zero digit, '.', '/', '|'

struct SegCounts {  // per line segment: count[category][class], class = position mod 4
    uint16_t c[kCats][4];
};

// 0x01 in every byte of x that belongs to each category
struct ByteCats {
    uint32_t v[kCats];
};
__device__ __forceinline__ uint32_t eq01(uint32_t x, uint32_t rep) { return zero_bytes(x ^ rep) >> 7; }
__device__ __forceinline__ ByteCats classify(uint32_t x) {
    ByteCats b;
    const uint32_t t = x ^ 0x30303030u;
    const uint32_t dig = (~(((t & 0x7F7F7F7Fu) + 0x76767676u) | t) & 0x80808080u) >> 7;  // t < 10
    b.v[0] = eq01(x, 0x09090909u);
    b.v[1] = dig;
    b.v[2] = dig & ~(zero_bytes(t) >> 7);  // digit other than '0'
    b.v[3] = eq01(x, 0x2E2E2E2Eu);
    b.v[4] = eq01(x, 0x2F2F2F2Fu);
    b.v[5] = eq01(x, 0x7C7C7C7Cu);
    return b;
}
// 0x01 per byte j of the dword at `base` (4-aligned) with lo <= base + j < hi
__device__ __forceinline__ uint32_t range01(int64_t base, int64_t lo, int64_t hi) {
    const uint32_t m4 = range_mask16(base, lo, hi) & 0xFu;
    return (m4 * 0x00204081u) & 0x01010101u;
}

struct SegAcc {  // per-lane byte counters (one byte per class) for the open segment
    uint32_t a[kCats];
    __device__ void clear() {
#pragma unroll
        for (int k = 0; k < kCats; k++) a[k] = 0;
    }
    __device__ void add(uint32_t x, uint32_t keep01) {
        const ByteCats b = classify(x);
#pragma unroll
        for (int k = 0; k < kCats; k++) a[k] += b.v[k] & keep01;
    }
    __device__ void add_all(uint32_t x) {
        const ByteCats b = classify(x);
#pragma unroll
        for (int k = 0; k < kCats; k++) a[k] += b.v[k];
    }
    // wave-reduce into the segment slot (lane 0 writes); counters are <= 64 per byte lane
    // (16 steps x 4 dwords) so two 16-bit fields per word never carry
    __device__ void flush(SegCounts *out) {
#pragma unroll
        for (int k = 0; k < kCats; k++) {
            const uint32_t lo = wave_sum(a[k] & 0x00FF00FFu), hi = wave_sum((a[k] >> 8) & 0x00FF00FFu);
            if (lane() == 0) {
                out->c[k][0] = (uint16_t)(lo & 0xFFFFu);
                out->c[k][2] = (uint16_t)(lo >> 16);
                out->c[k][1] = (uint16_t)(hi & 0xFFFFu);
                out->c[k][3] = (uint16_t)(hi >> 16);
            }
        }
        clear();
    }
};

// a 1 KiB step holding newlines: offsets into the slot table, then the step's bytes split
// at each newline into the open segment (flushed) and the next one.  Out of line: it runs
// for ~1 step in 10 and would otherwise be unrolled into every step of the sweep.
__device__ __forceinline__ void seg_step(const uint4 v, int64_t w, int64_t blk, bool in, uint32_t m,
                                                   uint64_t lanes, int64_t lo, int64_t hi, uint32_t &run,
                                                   uint64_t *slot, SegCounts *sg, SegAcc &acc) {
    const uint32_t c1 = __popc(m);
    const uint32_t incl = wave_incl_scan(c1);
    uint32_t idx = run + incl - c1;
    for (uint32_t mm = m; mm; mm &= mm - 1u) {
        if (idx < (uint32_t)kScanCap) slot[idx] = (uint64_t)(blk + __builtin_ctz(mm));
        idx++;
    }
    const uint32_t total = wave_bcast(incl, kWave - 1);
    int64_t from = w > lo ? w : lo;
    uint32_t lm = m;
    for (uint32_t k = 0; k < total; k++) {
        const int src = __builtin_ctzll(lanes);
        const uint32_t bits = (uint32_t)__shfl((int)lm, src);
        const int64_t p = w + (int64_t)src * kBlockBytes + __builtin_ctz(bits);
        if (in) {
            acc.add(v.x, range01(blk, from, p));
            acc.add(v.y, range01(blk + 4, from, p));
            acc.add(v.z, range01(blk + 8, from, p));
            acc.add(v.w, range01(blk + 12, from, p));
        }
        if (run < (uint32_t)kSegSlots) acc.flush(&sg[run]);
        else acc.clear();
        run++;
        from = p + 1;
        if (lane() == src) lm &= lm - 1u;
        lanes = __ballot(lm != 0);
    }
    if (in) {
        const int64_t to = w + kWaveStep < hi ? w + kWaveStep : hi;
        acc.add(v.x, range01(blk, from, to));
        acc.add(v.y, range01(blk + 4, from, to));
        acc.add(v.z, range01(blk + 8, from, to));
        acc.add(v.w, range01(blk + 12, from, to));
    }
}

__global__ __launch_bounds__(256) void k_af_scan(const char *__restrict__ buf, int64_t lo, int64_t hi, int64_t nchunks,
                                                 uint32_t *__restrict__ counts, uint64_t *__restrict__ pos,
                                                 SegCounts *__restrict__ seg, unsigned *__restrict__ overflow) {
    const int64_t a0 = lo & ~(int64_t)15;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x / kWave; c < nchunks; c += nw) {
        const int64_t base = a0 + c * kScanChunk;
        uint64_t *slot = pos + (uint64_t)c * kScanCap;
        SegCounts *sg = seg + (uint64_t)c * kSegSlots;
        uint32_t run = 0;  // newlines so far = index of the open segment
        SegAcc acc;
        acc.clear();
        constexpr int kSteps = (int)(kScanChunk / kWaveStep), kU = 8;
        for (int t0 = 0; t0 < kSteps; t0 += kU) {
            uint4 v[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int64_t blk = base + (int64_t)(t0 + u) * kWaveStep + (int64_t)lane() * kBlockBytes;
                if (blk < hi) v[u] = load16(buf, blk);
            }
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int64_t w = base + (int64_t)(t0 + u) * kWaveStep;
                if (w >= hi) break;  // wave-uniform
                const int64_t blk = w + (int64_t)lane() * kBlockBytes;
                const bool in = blk < hi;
                uint32_t m = in ? eq_mask16(v[u], kRepNl) & range_mask16(blk, lo, hi) : 0u;
                const uint64_t any = __ballot(m != 0);
                const bool edge = w < lo || w + kWaveStep > hi;  // wave-uniform
                if (!any) {
                    if (!edge) {
                        acc.add_all(v[u].x);
                        acc.add_all(v[u].y);
                        acc.add_all(v[u].z);
                        acc.add_all(v[u].w);
                    } else if (in) {
                        acc.add(v[u].x, range01(blk, lo, hi));
                        acc.add(v[u].y, range01(blk + 4, lo, hi));
                        acc.add(v[u].z, range01(blk + 8, lo, hi));
                        acc.add(v[u].w, range01(blk + 12, lo, hi));
                    }
                    continue;
                }
                seg_step(v[u], w, blk, in, m, any, lo, hi, run, slot, sg, acc);
            }
        }
        // the open segment continues into the next chunk (or is the file's tail)
        if (run < (uint32_t)kSegSlots) acc.flush(&sg[run]);
        if (lane() == 0) {
            counts[c] = run;
            if (run > (uint32_t)kScanCap) atomicOr(overflow, 1u);
        }
    }
}

// newline offsets -> line_end; each newline's chunk -> nl_chunk (for the segment walk)
__global__ void k_af_compact(int64_t nchunks, const uint32_t *__restrict__ counts, const uint64_t *__restrict__ offs,
                             const uint64_t *__restrict__ pos, uint64_t *__restrict__ line_end,
                             uint32_t *__restrict__ nl_chunk) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t b = i / kScanCap, k = i % kScanCap;
    if ((int64_t)b >= nchunks || k >= counts[b]) return;
    line_end[offs[b] + k] = pos[i];
    nl_chunk[offs[b] + k] = (uint32_t)b;
}

// class counts (per category) of the bytes of [ls, S) held in the head window
struct HeadCounts {
    uint32_t c[kCats][4];
};

__global__ __launch_bounds__(256) void k_af_combine(const char *__restrict__ buf, int64_t data_start, int64_t hi,
                                                    const uint64_t *__restrict__ line_end, uint64_t n_lines,
                                                    uint64_t n_newlines, int64_t nchunks, int mode,
                                                    const uint64_t *__restrict__ offs,
                                                    const uint32_t *__restrict__ nl_chunk,
                                                    const SegCounts *__restrict__ seg, LineMeta *__restrict__ meta,
                                                    int32_t *__restrict__ alt_o, int32_t *__restrict__ tot_o,
                                                    uint32_t *__restrict__ rowpre_o, uint8_t *__restrict__ status_o,
                                                    unsigned long long *__restrict__ counters) {
    __shared__ uint32_t cnt[2];
    if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t is_row = 0;
    if (li < n_lines) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
        const int64_t le = (int64_t)line_end[li];
        LineMeta m{};
        m.kind = kMetaFull;
        uint8_t st = 0;
        uint32_t alt = 0, tot = 0, rowpre = 0;
        if (le <= ls) m.kind = kMetaEmpty;
        else {
            const int64_t a = ls & ~(int64_t)15;
            constexpr int kB = 10;  // 160-byte head window
            uint4 v[kB];
#pragma unroll
            for (int b = 0; b < kB; b++) v[b] = load16(buf, a + 16 * b);
            int64_t ae = le;
            if (mode == 0 && byte_at(buf, le - 1) == '\r') {
                ae--;
                m.cr = 1;
            }
            const uint32_t first = byte_at(buf, ls);
            if (ae <= ls || first == '#') m.kind = ae <= ls ? kMetaEmpty : kMetaHeader;
            else {
                int nt = 0;
                int64_t t4 = 0, t7 = 0, t8 = 0;
#pragma unroll
                for (int b = 0; b < kB; b++) {
                    uint32_t mk = eq_mask16(v[b], kRepTab) & range_mask16(a + 16 * b, ls, ae);
                    while (mk && nt < 9) {
                        const int j = __builtin_ctz(mk);
                        mk &= mk - 1u;
                        const int64_t p = a + 16 * b + j;
                        nt++;
                        if (nt == 5) t4 = p;
                        if (nt == 8) t7 = p;
                        if (nt == 9) t8 = p;
                    }
                }
                if (nt == 9 && t8 - t7 >= 3 && byte_at(buf, t7 + 1) == 'G' && byte_at(buf, t7 + 2) == 'T' &&
                    (t8 - t7 == 3 || byte_at(buf, t7 + 3) == ':')) {
                    const int64_t S = t8 + 1;
                    m.kind = kMetaGt;
                    m.S = (uint64_t)S;
                    m.rowpre = (uint32_t)(t4 - ls + 1);
                    m.sep = S + 1 < ae ? (uint8_t)byte_at(buf, S + 1) : 0;
                    // class counts of the whole line = its segments; minus the head [ls, S)
                    uint32_t cc[kCats][4];
#pragma unroll
                    for (int k = 0; k < kCats; k++)
#pragma unroll
                        for (int q = 0; q < 4; q++) cc[k][q] = 0;
                    // first segment: after newline li-1 (slot rank+1 of its chunk), or
                    // chunk 0 slot 0 for line 0; then slot 0 of every following chunk up
                    // to the one holding the line's own newline (the last chunk for a tail)
                    uint64_t c0, k0;
                    if (li == 0) {
                        c0 = 0;
                        k0 = 0;
                    } else {
                        c0 = nl_chunk[li - 1];
                        k0 = (li - 1) - offs[c0] + 1;
                    }
                    const uint64_t ce = li < n_newlines ? nl_chunk[li] : (uint64_t)(nchunks - 1);
                    for (uint64_t c = c0; c <= ce; c++) {
                        const SegCounts &sgc = seg[c * kSegSlots + (c == c0 ? k0 : 0)];
#pragma unroll
                        for (int k = 0; k < kCats; k++)
#pragma unroll
                            for (int q = 0; q < 4; q++) cc[k][q] += sgc.c[k][q];
                    }
#pragma unroll
                    for (int b = 0; b < kB; b++) {
                        const int64_t blk = a + 16 * b;
                        const uint32_t d[4] = {v[b].x, v[b].y, v[b].z, v[b].w};
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const uint32_t keep = range01(blk + 4 * q, ls, S);
                            if (!keep) continue;
                            const ByteCats bc = classify(d[q]);
#pragma unroll
                            for (int k = 0; k < kCats; k++) {
                                const uint32_t x = bc.v[k] & keep;
                                cc[k][0] -= x & 0xFFu;
                                cc[k][1] -= (x >> 8) & 0xFFu;
                                cc[k][2] -= (x >> 16) & 0xFFu;
                                cc[k][3] -= x >> 24;
                            }
                        }
                    }
                    // gt_fast's acceptance, from the counts of [S, ae)
                    const int64_t L = ae - S;
                    bool ok = L >= 3 && ((L + 1) & 3) == 0 && (m.sep == '/' || m.sep == '|');
                    if (ok) {
                        const uint32_t units = (uint32_t)((L + 1) >> 2);
                        const int s0 = (int)(S & 3);
                        // class (s0 + k) & 3 by selects (no dynamically indexed register array)
                        auto cls = [&](int k, int q) {
                            const int c = (s0 + q) & 3;
                            return c == 0 ? cc[k][0] : c == 1 ? cc[k][1] : c == 2 ? cc[k][2] : cc[k][3];
                        };
                        const uint32_t sep1 = m.sep == '/' ? cls(4, 1) : cls(5, 1);
                        ok = cls(1, 0) + cls(3, 0) == units && cls(1, 2) + cls(3, 2) == units && sep1 == units &&
                             cls(0, 3) == units - 1;
                        tot = cls(1, 0) + cls(1, 2);
                        alt = cls(2, 0) + cls(2, 2);
                    }
                    st = ok ? 1 : kAfPending;  // pending: k_af_complex runs the general sweep
                    rowpre = m.rowpre;
                    is_row = 1;
                }
            }
        }
        meta[li] = m;
        if (m.kind != kMetaFull) {
            status_o[li] = st;
            alt_o[li] = (int32_t)alt;
            tot_o[li] = (int32_t)tot;
            rowpre_o[li] = rowpre;
        }
    }
    // counters 0 rows / 1 data lines: each kMetaGt line is one of both (block-reduced)
    const uint64_t b = __ballot(is_row != 0);
    if (lane() == 0 && b) atomicAdd(&cnt[0], (uint32_t)__popcll(b));
    __syncthreads();
    if (threadIdx.x == 0 && cnt[0]) {
        atomicAdd(&counters[0], (unsigned long long)cnt[0]);
        atomicAdd(&counters[1], (unsigned long long)cnt[0]);
    }
}

size_t af_scan_seg_bytes() { return sizeof(SegCounts) * kSegSlots; }
int af_scan_cap() { return kScanCap; }

hipError_t launch_af_scan(const char *buf, int64_t lo, int64_t hi, uint32_t *counts, uint64_t *pos, void *seg,
                          unsigned *overflow, hipStream_t s) {
    const int64_t nc = idx_wchunks(lo, hi);
    if (!nc) return hipSuccess;
    const int64_t g = (nc + 3) / 4;
    hipLaunchKernelGGL(k_af_scan, dim3((unsigned)(g < (1 << 20) ? g : (1 << 20))), dim3(256), 0, s, buf, lo, hi, nc,
                       counts, pos, static_cast<SegCounts *>(seg), overflow);
    return hipGetLastError();
}

hipError_t launch_af_combine(const char *buf, int64_t lo, int64_t hi, const uint32_t *counts, const uint64_t *offs,
                             const uint64_t *pos, const void *seg, uint64_t n_lines, uint64_t n_newlines, int mode,
                             uint64_t *line_end, uint32_t *nl_chunk, void *meta, int32_t *alt, int32_t *tot,
                             uint32_t *rowpre, uint8_t *status, unsigned long long *counters, hipStream_t s) {
    const int64_t nc = idx_wchunks(lo, hi);
    if (!nc || !n_lines) return hipSuccess;
    const uint64_t n = (uint64_t)nc * kScanCap;
    hipLaunchKernelGGL(k_af_compact, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nc, counts, offs, pos,
                       line_end, nl_chunk);
    hipLaunchKernelGGL(k_af_combine, dim3((unsigned)((n_lines + 255) / 256)), dim3(256), 0, s, buf, lo, hi, line_end,
                       n_lines, n_newlines, nc, mode, offs, nl_chunk, static_cast<const SegCounts *>(seg),
                       static_cast<LineMeta *>(meta), alt, tot, rowpre, status, counters);
    return hipGetLastError();
}

}  // namespace vcfxg
