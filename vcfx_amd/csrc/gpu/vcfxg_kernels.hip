// vcfxg_kernels.hip -- record kernels of the MI355X VCF engine (gfx950).
//
// K1 line index  : one HBM sweep (per 16 KiB wave-chunk newline counts + offsets) -> scan ->
//                  compaction into line end offsets (emit sweep only for very short lines).
// K2 AF records  : one wave per record; fixed-stride "a|b\t" fast path (SWAR on 16 B per
//                  lane, validated per record) with an exact general per-sample fallback.
// K5 AF rows     : row length -> exclusive scan -> device-formatted text rows.
//
// Reference behaviour restated: VCFX_allele_freq_calc.cpp (citations per function).
#include <algorithm>

#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_meta.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

// =======================================================================================
// K1: line index
// =======================================================================================
constexpr int kIdxThreads = 256;

// Single-sweep index over 16 KiB wave-chunks: the count pass also keeps the first kPosCap
// newline offsets of every chunk in a scratch table (wave-level ranks, no block barriers);
// after the scan a small compaction copies them to line_end, so the emit sweep runs only
// when some chunk holds more than kPosCap newlines (lines shorter than ~1 KiB on average).
constexpr int kPosCap = 16;
constexpr int64_t kWChunk = 16 * 1024;

template <bool kEmit>
__global__ __launch_bounds__(kIdxThreads) void k_idx_sweep(const char *__restrict__ buf, int64_t lo, int64_t hi,
                                                            int64_t nchunks, uint32_t *__restrict__ counts,
                                                            uint64_t *__restrict__ pos,
                                                            unsigned *__restrict__ overflow,
                                                            const uint64_t *__restrict__ offs,
                                                            uint64_t *__restrict__ line_end) {
    const int64_t a0 = lo & ~(int64_t)15;
    const int64_t nw = (int64_t)gridDim.x * (kIdxThreads / kWave);
    for (int64_t c = (int64_t)blockIdx.x * (kIdxThreads / kWave) + threadIdx.x / kWave; c < nchunks; c += nw) {
        const int64_t base = a0 + c * kWChunk;
        uint32_t run = 0;
        uint64_t *slot = kEmit ? line_end + offs[c] : pos + (uint64_t)c * kPosCap;
        constexpr int kSteps = (int)(kWChunk / kWaveStep), kU = 8;
        for (int t0 = 0; t0 < kSteps; t0 += kU) {
            uint4 v[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int64_t blk = base + (int64_t)(t0 + u) * kWaveStep + (int64_t)lane() * kBlockBytes;
                if (blk < hi) v[u] = load16(buf, blk);
            }
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int64_t blk = base + (int64_t)(t0 + u) * kWaveStep + (int64_t)lane() * kBlockBytes;
                uint32_t m = blk < hi ? eq_mask16(v[u], kRepNl) & range_mask16(blk, lo, hi) : 0u;
                const uint64_t any = __ballot(m != 0);
                if (!any) continue;  // wave-uniform: no newline in this 1 KiB
                const uint32_t c1 = __popc(m);
                const uint32_t incl = wave_incl_scan(c1);
                uint32_t idx = run + incl - c1;
                while (m) {
                    const int j = __builtin_ctz(m);
                    m &= m - 1u;
                    if (kEmit || idx < (uint32_t)kPosCap) slot[idx] = (uint64_t)(blk + j);
                    idx++;
                }
                run += wave_bcast(incl, kWave - 1);
            }
        }
        if (!kEmit && lane() == 0) {
            counts[c] = run;
            if (run > (uint32_t)kPosCap) atomicOr(overflow, 1u);
        }
    }
}

__global__ void k_nl_compact(int64_t nchunks, const uint32_t *__restrict__ counts, const uint64_t *__restrict__ offs,
                             const uint64_t *__restrict__ pos, uint64_t *__restrict__ line_end, uint64_t cap) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t b = i / kPosCap, k = i % kPosCap;
    if ((int64_t)b >= nchunks || k >= counts[b] || offs[b] + k >= cap) return;
    line_end[offs[b] + k] = pos[i];
}

// asynchronous index tail: line count (+ the unterminated last line) published on the
// device; a chunk over kPosCap newlines or a count over `cap` publishes 0 lines and raises
// *fail (the caller then reruns the synchronous index)
__global__ void k_idx_finish(const uint64_t *__restrict__ offs, int64_t nchunks, const unsigned *idx_overflow,
                             int tail, int64_t hi, uint64_t cap, uint64_t *__restrict__ line_end,
                             uint64_t *n_lines, unsigned *fail) {
    const uint64_t total = offs[nchunks];
    const uint64_t n = total + (tail ? 1 : 0);
    if (*idx_overflow || n > cap) {
        *fail = 1u;
        *n_lines = 0;
        return;
    }
    if (tail) line_end[total] = (uint64_t)hi;
    *n_lines = n;
}

// one small record for the host's single synchronisation of an AF call: line count, text
// bytes (row offsets scanned over a capacity, read at the device count), counters, failure
__global__ void k_af_summary(const uint64_t *n_lines, const uint64_t *__restrict__ rowoff,
                             const unsigned long long *__restrict__ counters, const unsigned *fail,
                             uint64_t *__restrict__ out) {
    const uint64_t n = *n_lines;
    out[0] = n;
    out[1] = rowoff[n];
    for (int k = 0; k < 4; k++) out[2 + k] = counters[k];
    out[6] = *fail;
}


// =======================================================================================
// K2: per-record GT reducers (allele counts, genotype match); one wave per line
// =======================================================================================
constexpr int kRecThreads = 256;
constexpr int kRecWaves = kRecThreads / kWave;

// block-reduced counters: one global atomic per block and counter
struct BlockCounters {
    uint32_t *lds;  // kNC entries
    static constexpr int kNC = 4;
    __device__ void add(int k, uint32_t v) {
        if (lane() == 0 && v) atomicAdd(&lds[k], v);
    }
};
__device__ __forceinline__ void flush_counters(uint32_t *lds, unsigned long long *g) {
    __syncthreads();
    if (threadIdx.x < BlockCounters::kNC && lds[threadIdx.x])
        atomicAdd(&g[threadIdx.x], (unsigned long long)lds[threadIdx.x]);
}

__device__ __forceinline__ void line_bounds(const uint64_t *__restrict__ line_end, int64_t data_start, uint64_t li,
                                            int64_t &ls, int64_t &le) {
    ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
    le = (int64_t)line_end[li];
}

// One AF data line [ls, le): processMmap :355-470 (mode 0) / processStdin :490-556 (mode 1).
// Status 1 = output row, 3 = "<9 fields" warning (stdin), 0 = nothing.  Counters: 0 rows,
// 1 data lines, 2 warn lines, 3 general-path records.
__device__ __forceinline__ void af_line(const char *__restrict__ buf, int64_t ls, int64_t le, int mode, int64_t *lds,
                                        BlockCounters &bc, uint8_t &st, uint32_t &alt, uint32_t &tot,
                                        uint32_t &rowpre) {
    int64_t ae = le;
    if (mode == 0 && ae > ls && byte_at(buf, ae - 1) == '\r') ae--;  // processMmap :362-364
    st = 0;
    alt = tot = rowpre = 0;
    if (ae > ls && byte_at(buf, ls) != '#') {
        bc.add(1, 1);
        int64_t t[10];
        const int nt = head_tabs(buf, ls, ae, 10, t, lds);
        bool ok = true;
        int64_t fs = 0, fe = 0;
        if (mode == 0) {
            // getField(8) must be non-empty (processMmap :391-401)
            if (nt < 8) ok = false;
            else {
                fs = t[7] + 1;
                fe = nt >= 9 ? t[8] : ae;
                ok = fe > fs;
            }
        } else {
            // processStdin :509-523: #fields = tabs + (last char != '\t')
            int nf = nt >= 9 ? 10 : nt + ((byte_at(buf, ae - 1) != '\t') ? 1 : 0);
            if (nf < 9) {
                st = 3;
                ok = false;
            } else {
                fs = t[7] + 1;
                fe = nt >= 9 ? t[8] : ae;
            }
        }
        if (ok) {
            const int gi = gt_index(buf, fs, fe);
            if (gi >= 0) {
                if (nt >= 9) {
                    const int64_t S = t[8] + 1;
                    AfOp op{buf, ae, gi};
                    bool fast = gi == 0 && af_fixed<VCFXG_UNROLL>(buf, S, ae, op, 0u, NoPre());
                    if (!fast && gi == 0) {  // GT-first, variable-width samples
                        op = AfOp{buf, ae, gi};
                        fast = gt_first_known(buf, S, ae, op);
                    }
                    if (fast) {
                        alt = op.alt;
                        tot = op.tot;
                    } else {
                        AfOp g{buf, ae, gi};
                        gt_general(buf, S, ae, g);
                        alt = g.alt;
                        tot = g.tot;
                        bc.add(3, 1);
                    }
                }
                st = 1;
                rowpre = (uint32_t)(t[4] - ls + 1);
            }
        }
    }
    bc.add(0, st == 1);
    bc.add(2, st == 3);
}

// one wave per indexed line
#ifdef VCFXG_AF_WAVES
__attribute__((amdgpu_waves_per_eu(VCFXG_AF_WAVES, 8)))
#endif
__global__ __launch_bounds__(kRecThreads) void k_af_records(const char *__restrict__ buf, int64_t data_start,
                                                            const uint64_t *__restrict__ line_end,
                                                            const uint64_t *n_lines_p, int mode,
                                                            int32_t *__restrict__ alt_o, int32_t *__restrict__ tot_o,
                                                            uint32_t *__restrict__ rowpre_o,
                                                            uint8_t *__restrict__ status_o,
                                                            unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kRecWaves][16];
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        int64_t ls, le;
        line_bounds(line_end, data_start, li, ls, le);
        uint8_t st;
        uint32_t alt, tot, rowpre;
        af_line(buf, ls, le, mode, lds, bc, st, alt, tot, rowpre);
        if (lane() == 0) {
            status_o[li] = st;
            alt_o[li] = (int32_t)alt;
            tot_o[li] = (int32_t)tot;
            rowpre_o[li] = rowpre;
        }
    }
    flush_counters(cnt, counters);
}

// =======================================================================================
// K2a/K2b: AF as a head pass + a sweep pass.  k_af_meta (one lane per line) parses each
// line's head out of its first 160 bytes: blank / '#' lines are settled, lines whose FORMAT
// starts with the GT sub-field (gi == 0, the reference's findGTIndex) get their sample
// region start S, the separator byte and the row prefix; anything else is left to the full
// per-line path.  k_af_sweep (one wave per line) then runs only the sample sweep for those
// lines, so a record's serial chain is one small metadata load + the sweep itself.
// =======================================================================================

typedef LineMeta AfMeta;

__device__ __forceinline__ void line_meta_one(const char *__restrict__ buf, int64_t data_start,
                                              const uint64_t *__restrict__ line_end, uint64_t li, int strip_cr,
                                              const uint8_t *__restrict__ gate, LineMeta *__restrict__ meta);

// lines [0, n_lines), one thread each; with `range` (device [first, end), the pipelined AF
// pieces) a grid-stride loop over [range[0], range[1]) instead
__global__ __launch_bounds__(256) void k_line_meta(const char *__restrict__ buf, int64_t data_start,
                                                   const uint64_t *__restrict__ line_end, uint64_t n_lines,
                                                   int strip_cr, const uint8_t *__restrict__ gate,
                                                   LineMeta *__restrict__ meta, const uint64_t *range) {
    const uint64_t gt = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (!range) {
        if (gt < n_lines) line_meta_one(buf, data_start, line_end, gt, strip_cr, gate, meta);
        return;
    }
    const uint64_t end = range[1], stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t li = range[0] + gt; li < end; li += stride) line_meta_one(buf, data_start, line_end, li, strip_cr, gate, meta);
}

__device__ __forceinline__ void line_meta_one(const char *__restrict__ buf, int64_t data_start,
                                              const uint64_t *__restrict__ line_end, uint64_t li, int strip_cr,
                                              const uint8_t *__restrict__ gate, LineMeta *__restrict__ meta) {
    if (gate && gate[li] != 1) {
        LineMeta m{};
        m.kind = kMetaGated;
        meta[li] = m;
        return;
    }
    const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
    const int64_t le = (int64_t)line_end[li];
    meta[li] = head_meta(GlobalSrc{buf}, ls, le, strip_cr);
}

__global__ __launch_bounds__(kRecThreads)
#ifdef VCFXG_SWEEP_MAXW
__attribute__((amdgpu_waves_per_eu(1, VCFXG_SWEEP_MAXW)))
#endif
void k_af_sweep(const char *__restrict__ buf, int64_t data_start,
                                                          const uint64_t *__restrict__ line_end,
                                                          const uint64_t *n_lines_p, int mode,
                                                          const AfMeta *__restrict__ meta,
                                                          int32_t *__restrict__ alt_o, int32_t *__restrict__ tot_o,
                                                          uint32_t *__restrict__ rowpre_o,
                                                          uint8_t *__restrict__ status_o,
                                                          unsigned long long *__restrict__ counters,
                                                          const uint64_t *first_p) {
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    const uint64_t n_lines = *n_lines_p;
    const uint64_t first = first_p ? *first_p : 0;  // lines [first, n_lines)
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    // the next line's head record and end are loaded before this line's sweep (their
    // latency hides behind it instead of opening every line)
    uint64_t li = first + wid;
    AfMeta mnext{};
    uint64_t lenext = 0;
    if (li < n_lines) {
        mnext = meta[li];
        lenext = line_end[li];
    }
    for (; li < n_lines; li += nw) {
        const AfMeta m = mnext;
        const uint64_t lecur = lenext;
        if (li + nw < n_lines) {
            mnext = meta[li + nw];
            lenext = line_end[li + nw];
        }
        uint8_t st = 0;
        uint32_t alt = 0, tot = 0, rowpre = 0;
        if (m.kind == kMetaGt) {
            const int64_t le = (int64_t)lecur, ae = le - m.cr;
            bc.add(1, 1);
            bc.add(0, 1);
            AfOp op{buf, ae, 0};
            if (af_fixed<VCFXG_UNROLL>(buf, (int64_t)m.S, ae, op, m.sep, NoPre())) {
                alt = op.alt;
                tot = op.tot;
                st = 1;
            } else {
                st = kAfPending;  // not fixed-stride: k_af_complex runs the general sweep
            }
            rowpre = m.rowpre;
        } else if (m.kind == kMetaFull) {
            continue;  // k_af_complex
        }
        if (lane() == 0) {
            status_o[li] = st;
            alt_o[li] = (int32_t)alt;
            tot_o[li] = (int32_t)tot;
            rowpre_o[li] = rowpre;
        }
    }
    flush_counters(cnt, counters);
}

// the lines k_af_meta left to the full per-line path (kind 2: FORMAT without a leading GT,
// heads longer than 160 bytes, fewer than 9 tabs, ...) and the kind-1 lines whose
// fixed-stride sweep failed (status kAfPending): the exact general per-sample sweep
__global__ __launch_bounds__(kRecThreads) void k_af_complex(const char *__restrict__ buf, int64_t data_start,
                                                            const uint64_t *__restrict__ line_end,
                                                            const uint64_t *n_lines_p, int mode,
                                                            const AfMeta *__restrict__ meta,
                                                            int32_t *__restrict__ alt_o, int32_t *__restrict__ tot_o,
                                                            uint32_t *__restrict__ rowpre_o,
                                                            uint8_t *__restrict__ status_o,
                                                            unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kRecWaves][16];
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    // a wave scans 64 lines' kinds per step and works only on the kind-2 ones
    for (uint64_t l0 = wid * kWave; l0 < n_lines; l0 += nw * kWave) {
        const uint64_t mine = l0 + lane();
        const bool full = mine < n_lines && meta[mine].kind == kMetaFull;
        const bool pend = mine < n_lines && !full && status_o[mine] == kAfPending;
        uint64_t todo = __ballot(full || pend);
        const uint64_t pendm = __ballot(pend);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1ull;
            const uint64_t li = l0 + k;
            if ((pendm >> k) & 1ull) {
                const AfMeta m = meta[li];
                const int64_t ae = (int64_t)line_end[li] - m.cr;
                AfOp g{buf, ae, 0};
                if (!gt_first_known(buf, (int64_t)m.S, ae, g)) {
                    g = AfOp{buf, ae, 0};
                    gt_general(buf, (int64_t)m.S, ae, g);
                }
                bc.add(3, 1);
                if (lane() == 0) {
                    status_o[li] = 1;
                    alt_o[li] = (int32_t)g.alt;
                    tot_o[li] = (int32_t)g.tot;
                }
                continue;
            }
            int64_t ls, le;
            line_bounds(line_end, data_start, li, ls, le);
            uint8_t st;
            uint32_t alt, tot, rowpre;
            af_line(buf, ls, le, mode, lds, bc, st, alt, tot, rowpre);
            if (lane() == 0) {
                status_o[li] = st;
                alt_o[li] = (int32_t)alt;
                tot_o[li] = (int32_t)tot;
                rowpre_o[li] = rowpre;
            }
        }
    }
    flush_counters(cnt, counters);
}

// one genotype_query data line [ls, le) -> status (1 keep, 2 drop, 3 warn, 4 header, 0 empty)
__device__ __forceinline__ uint8_t gq_line(const char *__restrict__ buf, int64_t ls, int64_t le, int strip_cr,
                                           const GqQuery &Q, int64_t *lds, BlockCounters &bc) {
    int64_t ae = le;
    if (strip_cr && ae > ls && byte_at(buf, ae - 1) == '\r') ae--;
    uint8_t st = 0;
    if (ae > ls) {
        if (byte_at(buf, ls) == '#') st = 4;
        else {
            bc.add(1, 1);
            int64_t t[10];
            const int nt = head_tabs(buf, ls, ae, 10, t, lds);
            // skipToField(8) (:223-230): NULL iff fewer than 8 tabs and the walk ends
            // before the line end
            const int64_t pn = nt ? t[(nt < 8 ? nt : 8) - 1] + 1 : ls;
            st = 2;
            if (nt < 8 && pn < ae) st = 3;
            else if (nt >= 9) {
                const int gi = gt_index(buf, t[7] + 1, t[8]);
                if (gi >= 0) {
                    const int64_t S = t[8] + 1;
                    GqOp op{buf, ae, gi, Q};
                    bool fast = gi == 0 && gt_fast(buf, S, ae, op);
                    bool hit;
                    if (fast) hit = op.found;
                    else {
                        GqOp g{buf, ae, gi, Q};
                        gt_general(buf, S, ae, g);
                        hit = g.found;
                        bc.add(3, 1);
                    }
                    if (hit) st = 1;
                }
            }
            // nt == 8: FORMAT runs to the line end and there is no sample field -> drop
        }
    }
    bc.add(0, st == 1);
    bc.add(2, st == 3);
    return st;
}
__device__ __forceinline__ uint8_t gq_gated(uint8_t st, const uint8_t *gate) {
    return gate ? (st == 1 ? 1 : (st == 3 ? 7 : 6)) : st;  // kept-by-filter: match / warn / no match
}

// genotype_query per line: status 1 keep, 2 drop, 3 "<9 fields" warning, 4 header, 0 empty.
// genotypeQueryMmap :450-516 / genotypeQueryStream :546-607 per data line; strip_cr = the
// line as VCFX_record_filter emitted it (fused RF|GQ pipeline).
__global__ __launch_bounds__(kRecThreads) void k_gq_records(const char *__restrict__ buf, int64_t data_start,
                                                            const uint64_t *__restrict__ line_end,
                                                            const uint64_t *n_lines_p, int strip_cr, GqQuery Q,
                                                            uint8_t *__restrict__ status_o,
                                                            unsigned long long *__restrict__ counters,
                                                            const uint8_t *gate) {
    __shared__ int64_t scratch[kRecWaves][16];
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        // gated (fused record_filter | genotype_query): only lines record_filter kept
        if (gate && uniform32(gate[li]) != 1) continue;
        int64_t ls, le;
        line_bounds(line_end, data_start, li, ls, le);
        const uint8_t st = gq_gated(gq_line(buf, ls, le, strip_cr, Q, lds, bc), gate);
        if (lane() == 0) status_o[li] = st;
    }
    flush_counters(cnt, counters);
}

// nonref_filter per line: status 1 keep, 2 drop, 4 '#' line, 0 empty.
// filterNonRefMmap :458-551 (mode 0: '\r' stripped; FORMAT = field 8; keep when there is
// no FORMAT, no GT in it or no 9th tab) / filterNonRef :553-636 (mode 1: keep under 10
// fields or without GT; a trailing tab is an empty last sample, which keeps the line).
// Data lines before '#CHROM' are the host's (warning + pass-through).
__device__ uint8_t nr_line(const char *__restrict__ buf, int64_t ls, int64_t le, int mode, int64_t *lds,
                           BlockCounters &bc) {
    int64_t ae = le;
    if (mode == 0 && ae > ls && byte_at(buf, ae - 1) == '\r') ae--;
    if (ae <= ls) return 0;
    if (byte_at(buf, ls) == '#') return 4;
    int64_t t[9];
    const int nt = head_tabs(buf, ls, ae, 9, t, lds);
    bool keep = true;
    if (nt >= 8 && (mode == 0 || nt >= 9)) {
        const int64_t fs = t[7] + 1, fe = nt >= 9 ? t[8] : ae;
        const int gi = gt_index(buf, fs, fe);  // findGTIndex :317-335 (first "GT" getline token)
        if (gi >= 0 && nt >= 9) {
            const int64_t S = t[8] + 1;
            if (S >= ae) keep = mode == 1;  // "...\tGT\t": mmap sees no sample, stdin an empty one
            else if (mode == 1 && byte_at(buf, ae - 1) == '\t') keep = true;  // empty last sample
            else {
                NrOp op{buf, ae, gi, mode};
                bool fast = gi == 0 && gt_fast<6>(buf, S, ae, op);
                if (!fast) {
                    bc.add(3, 1);
                    NrOp g{buf, ae, gi, mode};
                    gt_general(buf, S, ae, g);
                    keep = g.found;
                } else keep = op.found;
            }
        }
    }
    bc.add(0, keep);
    bc.add(1, 1);
    return keep ? 1 : 2;
}
__global__ __launch_bounds__(kRecThreads) void k_nr_records(const char *__restrict__ buf, int64_t data_start,
                                                            const uint64_t *__restrict__ line_end,
                                                            const uint64_t *n_lines_p, int mode,
                                                            uint8_t *__restrict__ status_o,
                                                            unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kRecWaves][16];
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        int64_t ls, le;
        line_bounds(line_end, data_start, li, ls, le);
        const uint8_t st = nr_line(buf, ls, le, mode, lds, bc);
        if (lane() == 0) status_o[li] = st;
    }
    flush_counters(cnt, counters);
}

// after the nonref walk: the lines it left (kGqPending: a GT-first record off the fixed-stride
// sweep; kGqFull: everything else) through nr_line, one wave each, and the tool's counters
// over all lines (lane per line, 64 lines per wave step)
__global__ __launch_bounds__(kRecThreads) void k_nr_complex(const char *__restrict__ buf, int64_t data_start,
                                                            const uint64_t *__restrict__ line_end,
                                                            const uint64_t *n_lines_p, int mode,
                                                            uint8_t *__restrict__ status,
                                                            unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kRecWaves][16];
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    uint32_t kept = 0, data = 0;  // this lane's walk-decided lines (nr_line counts its own)
    for (uint64_t g0 = wid * kWave; g0 < n_lines; g0 += nw * kWave) {
        const uint64_t li = g0 + lane();
        const uint8_t st = li < n_lines ? status[li] : 0;
        const bool pend = st == kGqPending || st == kGqFull;
        kept += !pend && st == 1;
        data += !pend && (st == 1 || st == 2);
        uint64_t todo = __ballot(pend);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t lk = g0 + k;
            int64_t ls, le;
            line_bounds(line_end, data_start, lk, ls, le);
            const uint8_t r = nr_line(buf, ls, le, mode, lds, bc);
            if (lane() == 0) status[lk] = r;
        }
    }
    bc.add(0, wave_sum(kept));
    bc.add(1, wave_sum(data));
    flush_counters(cnt, counters);
}

// genotype_query as head pass (k_line_meta) + sweep: GT-first lines run only the sample
// sweep (gt_fast with the GqOp early exit); full-path lines and fast-sweep failures go to
// k_gq_complex (status kGqPending marks the latter)

__global__ __launch_bounds__(kRecThreads) void k_gq_sweep(const char *__restrict__ buf,
                                                          const uint64_t *__restrict__ line_end,
                                                          const uint64_t *n_lines_p, GqQuery Q,
                                                          const LineMeta *__restrict__ meta,
                                                          uint8_t *__restrict__ status_o,
                                                          unsigned long long *__restrict__ counters,
                                                          const uint8_t *gate) {
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        const LineMeta m = meta[li];
        uint8_t st;
        if (m.kind == kMetaGated || m.kind == kMetaFull) continue;
        if (m.kind == kMetaEmpty) st = 0;
        else if (m.kind == kMetaHeader) st = 4;
        else {
            const int64_t ae = (int64_t)line_end[li] - m.cr;
            bc.add(1, 1);
            GqOp op{buf, ae, 0, Q};
            if (gt_fast(buf, (int64_t)m.S, ae, op, m.sep)) {
                st = op.found ? 1 : 2;
                bc.add(0, st == 1);
            } else {
                if (lane() == 0) status_o[li] = kGqPending;
                continue;
            }
        }
        if (lane() == 0) status_o[li] = gq_gated(st, gate);
    }
    flush_counters(cnt, counters);
}

__global__ __launch_bounds__(kRecThreads) void k_gq_complex(const char *__restrict__ buf, int64_t data_start,
                                                            const uint64_t *__restrict__ line_end,
                                                            const uint64_t *n_lines_p, int strip_cr, GqQuery Q,
                                                            const LineMeta *__restrict__ meta,
                                                            uint8_t *__restrict__ status_o,
                                                            unsigned long long *__restrict__ counters,
                                                            const uint8_t *gate) {
    __shared__ int64_t scratch[kRecWaves][16];
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t l0 = wid * kWave; l0 < n_lines; l0 += nw * kWave) {
        const uint64_t mine = l0 + lane();
        const bool full = mine < n_lines && meta[mine].kind == kMetaFull;
        const bool pend = mine < n_lines && !full && meta[mine].kind == kMetaGt && status_o[mine] == kGqPending;
        uint64_t todo = __ballot(full || pend);
        const uint64_t pendm = __ballot(pend);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1ull;
            const uint64_t li = l0 + k;
            uint8_t st;
            if ((pendm >> k) & 1ull) {
                const LineMeta m = meta[li];
                const int64_t ae = (int64_t)line_end[li] - m.cr;
                GqOp g{buf, ae, 0, Q};
                gt_general(buf, (int64_t)m.S, ae, g);
                bc.add(3, 1);
                st = g.found ? 1 : 2;
                bc.add(0, st == 1);
            } else {
                int64_t ls, le;
                line_bounds(line_end, data_start, li, ls, le);
                st = gq_line(buf, ls, le, strip_cr, Q, lds, bc);
            }
            if (lane() == 0) status_o[li] = gq_gated(st, gate);
        }
    }
    flush_counters(cnt, counters);
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

__global__ void k_af_format(const char *__restrict__ buf, int64_t data_start, const uint64_t *__restrict__ line_end,
                            const uint64_t *n_lines_p, int mode, const int32_t *__restrict__ alt,
                            const int32_t *__restrict__ tot, const uint32_t *__restrict__ rowpre,
                            const uint8_t *__restrict__ status, const uint64_t *__restrict__ off,
                            char *__restrict__ out, uint64_t cap) {
    const uint64_t n = *n_lines_p;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gridDim.x * (uint64_t)blockDim.x) {
        if (status[i] != 1 || off[i + 1] > cap) continue;
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
// AF region tail straight from the walk's regions (no dense per-line arrays)
// =======================================================================================
// the walk's leftover slots: kMetaFull lines run af_line (the exact per-line path), GT lines
// whose fixed-stride sweep failed the general sweep (their row bytes are already counted);
// a kMetaFull line that becomes a row adds its bytes to its walker's total
__global__ __launch_bounds__(kRecThreads) void k_af_cx(const char *__restrict__ buf, int mode, uint64_t cap_w,
                                                       const uint64_t *__restrict__ list,
                                                       const unsigned long long *list_n, uint64_t list_cap,
                                                       const uint64_t *__restrict__ wstart,
                                                       const uint64_t *__restrict__ le_b,
                                                       const LineMeta *__restrict__ meta_b, int32_t *__restrict__ alt_b,
                                                       int32_t *__restrict__ tot_b, uint32_t *__restrict__ rowpre_b,
                                                       uint8_t *__restrict__ status_b, uint64_t *__restrict__ wtext,
                                                       unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kRecWaves][16];
    __shared__ uint32_t cnt[BlockCounters::kNC];
    if (threadIdx.x < BlockCounters::kNC) cnt[threadIdx.x] = 0;
    __syncthreads();
    BlockCounters bc{cnt};
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n = std::min<uint64_t>(*list_n, list_cap);
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t e = wid; e < n; e += nw) {
        const uint64_t sl = (uint64_t)uniform64((int64_t)list[e]);
        const uint64_t w = sl / cap_w, i = sl - w * cap_w;
        const int64_t le = (int64_t)le_b[sl];
        const LineMeta m = meta_b[sl];
        if (m.kind == kMetaGt) {
            const int64_t ae = le - m.cr;
            AfOp g{buf, ae, 0};
            if (!gt_first_known(buf, (int64_t)m.S, ae, g)) {
                g = AfOp{buf, ae, 0};
                gt_general(buf, (int64_t)m.S, ae, g);
            }
            bc.add(3, 1);
            if (lane() == 0) {
                status_b[sl] = 1;
                alt_b[sl] = (int32_t)g.alt;
                tot_b[sl] = (int32_t)g.tot;
            }
            continue;
        }
        const int64_t ls = i ? (int64_t)le_b[sl - 1] + 1 : (int64_t)wstart[w];
        uint8_t st;
        uint32_t alt, tot, rowpre;
        af_line(buf, ls, le, mode, lds, bc, st, alt, tot, rowpre);
        if (lane() == 0) {
            status_b[sl] = st;
            alt_b[sl] = (int32_t)alt;
            tot_b[sl] = (int32_t)tot;
            rowpre_b[sl] = rowpre;
            if (st == 1) atomicAdd(reinterpret_cast<unsigned long long *>(&wtext[w]), (unsigned long long)rowpre + 7ull);
        }
    }
    flush_counters(cnt, counters);
}

// exclusive scans of the walkers' line counts and row bytes, 1024 walkers per block: each
// block writes block-local offsets and its totals; the last block to finish scans the block
// totals into bpre_* (entry k = the offsets before block k; bpre[nb] = the grand totals), so a
// walker's offset is woff[w] + bpre[w >> 10] with no second pass.  The last block also adds
// the GT-line total to counters[0..1] (rows, data lines) and writes the line count to *n_lines
// and the call summary (lines, text bytes, counters[0..3], *fail).
constexpr int kWScan = kWalkerScanBlock;
__device__ __forceinline__ void block_scan2(uint64_t &a, uint64_t &b, uint64_t *sa, uint64_t *sb) {
    // inclusive: wave scans, then the 16 wave totals by one wave
    const int t = threadIdx.x, wv = t / kWave;
    a = wave_incl_scan(a);
    b = wave_incl_scan(b);
    if (lane() == kWave - 1) {
        sa[wv] = a;
        sb[wv] = b;
    }
    __syncthreads();
    if (wv == 0) {
        uint64_t x = lane() < kWScan / kWave ? sa[lane()] : 0, y = lane() < kWScan / kWave ? sb[lane()] : 0;
        x = wave_incl_scan(x);
        y = wave_incl_scan(y);
        if (lane() < kWScan / kWave) {
            sa[lane()] = x;
            sb[lane()] = y;
        }
    }
    __syncthreads();
    if (wv) {
        a += sa[wv - 1];
        b += sb[wv - 1];
    }
}
__global__ __launch_bounds__(kWScan) void k_walker_scan(int64_t nw, const uint64_t *__restrict__ wcount,
                                                        const uint64_t *__restrict__ wtext,
                                                        const uint32_t *__restrict__ wgt, uint64_t *__restrict__ woff,
                                                        uint64_t *__restrict__ wtoff, uint64_t *bpre_a, uint64_t *bpre_b,
                                                        uint64_t *bsum, unsigned *done,
                                                        unsigned long long *counters, const unsigned *fail,
                                                        uint64_t *n_lines, uint64_t *__restrict__ summary,
                                                        uint64_t *reset) {
    __shared__ uint64_t sa[kWScan / kWave], sb[kWScan / kWave];
    __shared__ bool last;
    const int t = threadIdx.x;
    const int64_t nb = (nw + kWScan - 1) / kWScan;
    const int64_t w = (int64_t)blockIdx.x * kWScan + t;
    const uint64_t a0 = w < nw ? wcount[w] : 0, b0 = w < nw ? wtext[w] : 0;
    // wgt: GT-first lines (low 16 bits) | the GT-first walk's lines swept by gt_first (high 16)
    const uint32_t gw = w < nw ? wgt[w] : 0u;
    uint64_t g = (uint64_t)(gw & 0xFFFFu) | ((uint64_t)(gw >> 16) << 32);
    uint64_t a = a0, b = b0;
    block_scan2(a, b, sa, sb);
    if (w <= nw) {  // (w == nw: the block total, the end offset within this block)
        woff[w] = a - a0;
        wtoff[w] = b - b0;
    }
    g = wave_sum(g);
    __syncthreads();
    __shared__ uint64_t sg[kWScan / kWave];
    if (lane() == 0) sg[t / kWave] = g;
    __syncthreads();
    if (t == kWScan - 1) {
        uint64_t G = 0;
        for (int k = 0; k < kWScan / kWave; k++) G += sg[k];
        // block totals -> bsum[3 * blk], published before the arrival count (device scope)
        __hip_atomic_store(&bsum[3 * blockIdx.x], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&bsum[3 * blockIdx.x + 1], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&bsum[3 * blockIdx.x + 2], G, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (unsigned)nb - 1;
    }
    __syncthreads();
    if (!last) return;
    // the last block: prefix of the block totals (atomic loads: other CUs' stores), 64 blocks
    // per step by wave 0 (a serial loop paid one L2 round trip per block)
    if (t >= kWave) return;
    uint64_t ra = 0, rb = 0, G = 0;
    for (int64_t k0 = 0; k0 < nb; k0 += kWave) {
        const int64_t k = k0 + lane();
        const bool in = k < nb;
        const uint64_t x = in ? __hip_atomic_load(&bsum[3 * k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0,
                       y = in ? __hip_atomic_load(&bsum[3 * k + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0,
                       z = in ? __hip_atomic_load(&bsum[3 * k + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        const uint64_t xi = wave_incl_scan(x), yi = wave_incl_scan(y);
        if (in) {
            bpre_a[k] = ra + xi - x;
            bpre_b[k] = rb + yi - y;
        }
        ra += wave_bcast(xi, kWave - 1);
        rb += wave_bcast(yi, kWave - 1);
        G += wave_sum(z);
    }
    if (lane() == 0) {
        bpre_a[nb] = ra;
        bpre_b[nb] = rb;
        if (nw % kWScan == 0) {  // no thread stood at w == nw
            woff[nw] = 0;
            wtoff[nw] = 0;
        }
        *done = 0;  // ready for the next launch
        counters[0] += G & 0xFFFFFFFFull;
        counters[1] += G & 0xFFFFFFFFull;
        counters[3] += G >> 32;  // records of the general (gt_first) sweep
        *n_lines = ra;
        summary[0] = ra;
        summary[1] = rb;
        for (int k = 0; k < 4; k++) summary[2 + k] = counters[k];
        summary[6] = *fail;
        if (reset) {  // the call's flags and counters, zeroed once read: no memset before the next call
            summary[7] = reset[1];
            for (int k = 0; k < 6; k++) reset[k] = 0;
        }
    }
}

// k_af_format_w.  A clean walker (the walk composed every row of it into its stage:
// wdirty[w] == 0) is copied out whole by a 16-lane group, four walkers per wave: lane l of the
// group writes the aligned 16 B blocks l, l + 16, ... of the walker's text span, each the byte
// rotation (uniform per walker: the span's offset mod 16) of two aligned stage blocks; the
// span's first and last blocks, shared with the neighbouring walkers, by byte stores.  One
// round trip for the offsets, one for the stage, and a quarter of the waves a wave per walker
// took.  The other walkers (a line left to k_af_cx, a stage too small) take the whole wave one
// at a time: row offsets = the walker's text offset + a wave scan of its rows' lengths, each
// lane writes its line's row.  Rows / walkers ending past cap are skipped (the host writes all
// again once the text has grown).
constexpr int kFmtWaves = 4, kFmtGroup = 16, kFmtPerWave = kWave / kFmtGroup;
__device__ __forceinline__ uint32_t sel4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t i) {
    return i == 0 ? a : i == 1 ? b : i == 2 ? c : d;
}
__global__ __launch_bounds__(kFmtWaves *kWave) void k_af_format_w(const char *__restrict__ buf, int mode, int64_t nw,
                                                                   uint64_t cap_w, const uint64_t *__restrict__ wcount,
                                                                   const uint64_t *__restrict__ wtoff,
                                                                   const uint64_t *__restrict__ bpre_b,
                                                                   const uint64_t *__restrict__ wstart,
                                                                   const uint64_t *__restrict__ le_b,
                                                                   const int32_t *__restrict__ alt_b,
                                                                   const int32_t *__restrict__ tot_b,
                                                                   const uint32_t *__restrict__ rowpre_b,
                                                                   const uint8_t *__restrict__ status_b,
                                                                   char *__restrict__ out, uint64_t cap,
                                                                   const char *__restrict__ stage, uint32_t stage_cap,
                                                                   const uint8_t *__restrict__ wdirty,
                                                                   const uint64_t *__restrict__ wtext) {
    const int64_t step = (int64_t)gridDim.x * kFmtWaves * kFmtPerWave;
    const int g = lane() / kFmtGroup, gl = lane() % kFmtGroup;
    const int64_t qmax = (int64_t)(stage_cap / 16) - 1;
    for (int64_t w0 = ((int64_t)blockIdx.x * kFmtWaves + threadIdx.x / kWave) * kFmtPerWave; w0 < nw; w0 += step) {
        const int64_t w = w0 + g;
        const bool have = w < nw;
        const bool clean = have && stage && !wdirty[w];
        const uint64_t run = have ? wtoff[w] + bpre_b[w / kWScan] : 0, len = clean ? wtext[w] : 0;
        if (clean && len && run + len <= cap) {
            const uint4 *__restrict__ src = reinterpret_cast<const uint4 *>(stage + (uint64_t)w * stage_cap);
            const uint64_t d0 = run & ~15ull, dend = run + len;
            const int nblk = (int)(((dend + 15) >> 4) - (d0 >> 4));
            const int s = (int)(run & 15);
            const uint32_t r = (uint32_t)(16 - s) & 15u, rq = r >> 2, rb = r & 3u;
            for (int j0 = 0; j0 < nblk; j0 += 2 * kFmtGroup) {
                uint4 a[2], b[2];
#pragma unroll
                for (int u = 0; u < 2; u++) {  // dst block j <- stage blocks q, q + 1 (q = j - 1 when s > 0)
                    const int64_t q = (int64_t)(j0 + u * kFmtGroup + gl) - (s ? 1 : 0);
                    a[u] = src[q < 0 ? 0 : (q > qmax ? qmax : q)];
                    b[u] = src[q + 1 > qmax ? qmax : q + 1];
                }
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const int j = j0 + u * kFmtGroup + gl;
                    if (j >= nblk) continue;
                    const uint32_t W[8] = {a[u].x, a[u].y, a[u].z, a[u].w, b[u].x, b[u].y, b[u].z, b[u].w};
                    uint32_t o[4];
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        o[i] = __builtin_amdgcn_alignbyte(sel4(W[i + 1], W[i + 2], W[i + 3], W[i + 4], rq),
                                                          sel4(W[i], W[i + 1], W[i + 2], W[i + 3], rq), rb);
                    const uint64_t D = d0 + 16u * (uint64_t)j;
                    if (D >= run && D + 16 <= dend) {
                        *reinterpret_cast<uint4 *>(out + D) = make_uint4(o[0], o[1], o[2], o[3]);
                    } else {
#pragma unroll
                        for (int t = 0; t < 16; t++)
                            if (D + t >= run && D + t < dend) out[D + t] = (char)((o[t >> 2] >> (8 * (t & 3))) & 0xFFu);
                    }
                }
            }
        }
        // the group's other walkers, the whole wave each
        uint64_t dm = __ballot(gl == 0 && have && !clean);
        while (dm) {
            const int k = __builtin_ctzll(dm);
            dm &= dm - 1ull;
            const int64_t wd = w0 + k / kFmtGroup;
            uint64_t rw = wtoff[wd] + bpre_b[wd / kWScan];
            const uint64_t n = wcount[wd], s0 = (uint64_t)wd * cap_w;
            for (uint64_t i0 = 0; i0 < n; i0 += kWave) {
                const uint64_t i = i0 + lane(), sl = s0 + i;
                const bool in = i < n;
                const uint32_t pl = in ? rowpre_b[sl] : 0u;
                const uint32_t ln = in && status_b[sl] == 1 ? pl + 7u : 0u;
                const uint32_t incl = wave_incl_scan(ln);
                const uint64_t off = rw + incl - ln;
                rw += wave_bcast(incl, kWave - 1);
                if (!ln || off + ln > cap) continue;
                const int64_t ls = i ? (int64_t)le_b[sl - 1] + 1 : (int64_t)wstart[wd];
                char *o = out + off;
                for (uint32_t k2 = 0; k2 < pl; k2++) o[k2] = buf[ls + k2];
                uint32_t flo, fhi;
                af_freq_text(mode, alt_b[sl], tot_b[sl], flo, fhi);
                o += pl;
#pragma unroll
                for (int k2 = 0; k2 < 7; k2++) o[k2] = (char)((k2 < 4 ? flo >> (8 * k2) : fhi >> (8 * (k2 - 4))) & 0xFFu);
            }
        }
    }
}

// =======================================================================================
// launchers
// =======================================================================================
static unsigned grid_for(int64_t n, int64_t per, unsigned cap) {
    int64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

int idx_pos_cap() { return kPosCap; }
int64_t idx_wchunk_bytes() { return kWChunk; }
int64_t idx_wchunks(int64_t lo, int64_t hi) {
    const int64_t a0 = lo & ~(int64_t)15;
    return hi > lo ? (hi - a0 + kWChunk - 1) / kWChunk : 0;
}
hipError_t launch_idx_count(const char *buf, int64_t lo, int64_t hi, uint32_t *counts, uint64_t *pos,
                            unsigned *overflow, hipStream_t s) {
    const int64_t nc = idx_wchunks(lo, hi);
    if (!nc) return hipSuccess;
    hipLaunchKernelGGL(k_idx_sweep<false>, dim3(grid_for(nc, kIdxThreads / kWave, 1u << 20)), dim3(kIdxThreads), 0,
                       s, buf, lo, hi, nc, counts, pos, overflow, nullptr, nullptr);
    return hipGetLastError();
}
hipError_t launch_idx_emit(const char *buf, int64_t lo, int64_t hi, const uint64_t *offs, uint64_t *line_end,
                           hipStream_t s) {
    const int64_t nc = idx_wchunks(lo, hi);
    if (!nc) return hipSuccess;
    hipLaunchKernelGGL(k_idx_sweep<true>, dim3(grid_for(nc, kIdxThreads / kWave, 1u << 20)), dim3(kIdxThreads), 0,
                       s, buf, lo, hi, nc, nullptr, nullptr, nullptr, offs, line_end);
    return hipGetLastError();
}
hipError_t launch_nl_compact(int64_t lo, int64_t hi, const uint32_t *counts, const uint64_t *offs, const uint64_t *pos,
                             uint64_t *line_end, hipStream_t s) {
    const int64_t nc = idx_wchunks(lo, hi);
    if (!nc) return hipSuccess;
    const uint64_t n = (uint64_t)nc * kPosCap;
    hipLaunchKernelGGL(k_nl_compact, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nc, counts, offs, pos,
                       line_end, ~0ull);
    return hipGetLastError();
}
hipError_t launch_af_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int mode, int32_t *alt, int32_t *tot, uint32_t *rowpre,
                             uint8_t *status, unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    unsigned grid = grid_for((int64_t)n_lines_host, kRecWaves, 4096);
    hipLaunchKernelGGL(k_af_records, dim3(grid), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev, mode, alt,
                       tot, rowpre, status, counters);
    return hipGetLastError();
}
size_t af_meta_bytes() { return sizeof(AfMeta); }
// head pass + fixed-stride sweep over the device line range [range[0], range[1]) of one
// pipelined piece (at most max_lines lines: sizes the grids)
hipError_t launch_af_meta_sweep_range(const char *buf, int64_t data_start, const uint64_t *line_end,
                                      const uint64_t *range, uint64_t max_lines, int mode, void *meta, int32_t *alt,
                                      int32_t *tot, uint32_t *rowpre, uint8_t *status, unsigned long long *counters,
                                      hipStream_t s) {
    if (!max_lines) return hipSuccess;
    hipLaunchKernelGGL(k_line_meta, dim3(grid_for((int64_t)max_lines, 256, 2048)), dim3(256), 0, s, buf, data_start,
                       line_end, (uint64_t)0, mode == 0 ? 1 : 0, nullptr, static_cast<AfMeta *>(meta), range);
    unsigned grid = grid_for((int64_t)max_lines, kRecWaves, 4096);
    hipLaunchKernelGGL(k_af_sweep, dim3(grid), dim3(kRecThreads), 0, s, buf, data_start, line_end, range + 1, mode,
                       static_cast<const AfMeta *>(meta), alt, tot, rowpre, status, counters, range);
    return hipGetLastError();
}
hipError_t launch_af_complex(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, const void *meta,
                             int32_t *alt, int32_t *tot, uint32_t *rowpre, uint8_t *status,
                             unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    unsigned gridc = grid_for((int64_t)((n_lines_host + kWave - 1) / kWave), kRecWaves, 2048);
    hipLaunchKernelGGL(k_af_complex, dim3(gridc), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                       mode, static_cast<const AfMeta *>(meta), alt, tot, rowpre, status, counters);
    return hipGetLastError();
}
hipError_t launch_af_meta_sweep(const char *buf, int64_t data_start, const uint64_t *line_end,
                                const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, void *meta, int32_t *alt,
                                int32_t *tot, uint32_t *rowpre, uint8_t *status, unsigned long long *counters,
                                hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_line_meta, dim3((unsigned)((n_lines_host + 255) / 256)), dim3(256), 0, s, buf, data_start,
                       line_end, n_lines_host, mode == 0 ? 1 : 0, nullptr, static_cast<AfMeta *>(meta), nullptr);
    unsigned grid = grid_for((int64_t)n_lines_host, kRecWaves, 4096);
    hipLaunchKernelGGL(k_af_sweep, dim3(grid), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev, mode,
                       static_cast<const AfMeta *>(meta), alt, tot, rowpre, status, counters, nullptr);
    unsigned gridc = grid_for((int64_t)((n_lines_host + kWave - 1) / kWave), kRecWaves, 2048);
    hipLaunchKernelGGL(k_af_complex, dim3(gridc), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                       mode, static_cast<const AfMeta *>(meta), alt, tot, rowpre, status, counters);
    return hipGetLastError();
}
hipError_t launch_nr_complex(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, uint8_t *status,
                             unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    unsigned grid = grid_for((int64_t)((n_lines_host + kWave - 1) / kWave), kRecWaves, 1024);
    hipLaunchKernelGGL(k_nr_complex, dim3(grid), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                       mode, status, counters);
    return hipGetLastError();
}
hipError_t launch_nr_records(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, uint8_t *status,
                             unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    unsigned grid = grid_for((int64_t)n_lines_host, kRecWaves, 4096);
    hipLaunchKernelGGL(k_nr_records, dim3(grid), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                       mode, status, counters);
    return hipGetLastError();
}
hipError_t launch_gq_records(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int strip_cr, const char *q_dev,
                             int qlen, int strict, int qa, int qb, uint8_t *status, unsigned long long *counters,
                             hipStream_t s, const uint8_t *gate, void *meta) {
    if (!n_lines_host) return hipSuccess;
    GqQuery Q{q_dev, qlen, strict, qa, qb};
    unsigned grid = grid_for((int64_t)n_lines_host, kRecWaves, 4096);
    if (!meta) {
        hipLaunchKernelGGL(k_gq_records, dim3(grid), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                           strip_cr, Q, status, counters, gate);
        return hipGetLastError();
    }
    LineMeta *lm = static_cast<LineMeta *>(meta);
    hipLaunchKernelGGL(k_line_meta, dim3((unsigned)((n_lines_host + 255) / 256)), dim3(256), 0, s, buf, data_start,
                       line_end, n_lines_host, strip_cr, gate, lm, nullptr);
    hipLaunchKernelGGL(k_gq_sweep, dim3(grid), dim3(kRecThreads), 0, s, buf, line_end, n_lines_dev, Q, lm, status,
                       counters, gate);
    unsigned gridc = grid_for((int64_t)((n_lines_host + kWave - 1) / kWave), kRecWaves, 1024);
    hipLaunchKernelGGL(k_gq_complex, dim3(gridc), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                       strip_cr, Q, lm, status, counters, gate);
    return hipGetLastError();
}
hipError_t launch_gq_complex(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int strip_cr, const char *q_dev,
                             int qlen, int strict, int qa, int qb, const void *meta, uint8_t *status,
                             unsigned long long *counters, const uint8_t *gate, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    GqQuery Q{q_dev, qlen, strict, qa, qb};
    unsigned gridc = grid_for((int64_t)((n_lines_host + kWave - 1) / kWave), kRecWaves, 1024);
    hipLaunchKernelGGL(k_gq_complex, dim3(gridc), dim3(kRecThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                       strip_cr, Q, static_cast<const LineMeta *>(meta), status, counters, gate);
    return hipGetLastError();
}
hipError_t launch_nl_compact_cap(int64_t lo, int64_t hi, const uint32_t *counts, const uint64_t *offs,
                                 const uint64_t *pos, uint64_t *line_end, uint64_t cap, hipStream_t s) {
    const int64_t nc = idx_wchunks(lo, hi);
    if (!nc) return hipSuccess;
    const uint64_t n = (uint64_t)nc * kPosCap;
    hipLaunchKernelGGL(k_nl_compact, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nc, counts, offs, pos,
                       line_end, cap);
    return hipGetLastError();
}
hipError_t launch_idx_finish(const uint64_t *offs, int64_t nchunks, const unsigned *idx_overflow, int tail, int64_t hi,
                             uint64_t cap, uint64_t *line_end, uint64_t *n_lines, unsigned *fail, hipStream_t s) {
    hipLaunchKernelGGL(k_idx_finish, dim3(1), dim3(1), 0, s, offs, nchunks, idx_overflow, tail, hi, cap, line_end,
                       n_lines, fail);
    return hipGetLastError();
}
hipError_t launch_af_summary(const uint64_t *n_lines, const uint64_t *rowoff, const unsigned long long *counters,
                             const unsigned *fail, uint64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_af_summary, dim3(1), dim3(1), 0, s, n_lines, rowoff, counters, fail, out);
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
                            hipStream_t s, uint64_t text_cap) {
    if (!n_lines_host) return hipSuccess;
    hipLaunchKernelGGL(k_af_format, dim3(grid_for((int64_t)n_lines_host, 256, 4096)), dim3(256), 0, s, buf, data_start,
                       line_end, n_lines_dev, mode, alt, tot, rowpre, status, off, out, text_cap);
    return hipGetLastError();
}

hipError_t launch_af_cx(const char *buf, int mode, uint64_t cap_w, const uint64_t *list, const unsigned long long *list_n,
                        uint64_t list_cap, uint64_t list_cap_host, const uint64_t *wstart, const uint64_t *le_b,
                        const void *meta_b, int32_t *alt_b, int32_t *tot_b, uint32_t *rowpre_b, uint8_t *status_b,
                        uint64_t *wtext, unsigned long long *counters, hipStream_t s) {
    // the list is short (the walk's leftovers); a wave per entry, grid-stride
    const unsigned grid = grid_for((int64_t)std::max<uint64_t>(list_cap_host, 1), kRecWaves, 2048);
    hipLaunchKernelGGL(k_af_cx, dim3(grid), dim3(kRecThreads), 0, s, buf, mode, cap_w, list, list_n, list_cap, wstart,
                       le_b, static_cast<const LineMeta *>(meta_b), alt_b, tot_b, rowpre_b, status_b, wtext, counters);
    return hipGetLastError();
}
hipError_t launch_walker_scan(int64_t nw, const uint64_t *wcount, const uint64_t *wtext, const uint32_t *wgt,
                              uint64_t *woff, uint64_t *wtoff, uint64_t *bpre_a, uint64_t *bpre_b, uint64_t *bsum,
                              unsigned *done, unsigned long long *counters, const unsigned *fail, uint64_t *n_lines,
                              uint64_t *summary, hipStream_t s, uint64_t *reset) {
    const int64_t nb = std::max<int64_t>((nw + kWScan - 1) / kWScan, 1);
    hipLaunchKernelGGL(k_walker_scan, dim3((unsigned)nb), dim3(kWScan), 0, s, nw, wcount, wtext, wgt, woff, wtoff,
                       bpre_a, bpre_b, bsum, done, counters, fail, n_lines, summary, reset);
    return hipGetLastError();
}
hipError_t launch_af_format_w(const char *buf, int mode, int64_t nw, uint64_t cap_w, const uint64_t *wcount,
                              const uint64_t *wtoff, const uint64_t *bpre_b, const uint64_t *wstart,
                              const uint64_t *le_b, const int32_t *alt_b, const int32_t *tot_b, const uint32_t *rowpre_b,
                              const uint8_t *status_b, char *out, uint64_t cap, hipStream_t s, const WalkTail *tail) {
    if (nw <= 0) return hipSuccess;
    const WalkTail t = tail ? *tail : WalkTail{};
    hipLaunchKernelGGL(k_af_format_w, dim3(grid_for(nw, kFmtWaves * kFmtPerWave, 16384)), dim3(kFmtWaves * kWave), 0, s, buf, mode, nw, cap_w,
                       wcount, wtoff, bpre_b, wstart, le_b, alt_b, tot_b, rowpre_b, status_b, out, cap, t.stage,
                       t.stage_cap, t.wdirty, t.wtext);
    return hipGetLastError();
}

// occurrences of one byte value in input bytes [lo, hi): 16 B per lane and step (aligned
// loads; the input buffer is padded past n), exact zero-byte counts of x ^ pattern per dword,
// a wave reduction and one atomic per wave.  HBM-bound; used by the fused chain's checks.
__global__ void __launch_bounds__(256) k_count_byte(const uint8_t *__restrict__ buf, uint64_t lo, uint64_t hi,
                                                    uint32_t pat, unsigned long long *out) {
    const uint64_t a0 = lo & ~15ull;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * 16;
    uint32_t cnt = 0;
    for (uint64_t b = a0 + ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; b < hi; b += step) {
        const uint4 v = *reinterpret_cast<const uint4 *>(buf + b);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const uint32_t x = w[d] ^ pat;
            uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // 0x80 per zero byte
            const uint64_t base = b + 4 * (uint64_t)d;
            if (base < lo || base + 4 > hi) {  // a partial dword at either end
                uint32_t keep = 0;
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (base + k >= lo && base + k < hi) keep |= 0x80u << (8 * k);
                z &= keep;
            }
            cnt += __popc(z);
        }
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(out, (unsigned long long)cnt);
}

hipError_t launch_count_byte(const uint8_t *buf, uint64_t lo, uint64_t hi, uint8_t byte, unsigned long long *out,
                             hipStream_t s) {
    if (hi <= lo) return hipSuccess;
    const uint64_t blocks16 = ((hi - (lo & ~15ull)) + 15) / 16;
    const unsigned grid = (unsigned)std::min<uint64_t>((blocks16 + 255) / 256, 4096);
    hipLaunchKernelGGL(k_count_byte, dim3(grid), dim3(256), 0, s, buf, lo, hi, 0x01010101u * byte, out);
    return hipGetLastError();
}

}  // namespace vcfxg
