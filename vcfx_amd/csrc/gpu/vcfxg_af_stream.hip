// vcfxg_af_stream.hip -- VCFX_allele_freq_calc's record pass in ONE sweep of the input.
//
// A persistent block per CU owns a contiguous range of 32 KiB chunks and streams them
// through a 4-chunk LDS ring with global_load_lds (two chunks in flight while it works on
// one).  Per chunk it
//   1. finds the chunk's newlines (lines are owned by the chunk holding their '\n'; the first
//      line ending here may start in the previous chunk, which is still in the ring),
//   2. runs the head pass of every such line out of LDS (vcfxg_meta.h: kind, sample start,
//      separator, row prefix -- processMmap / processStdin :355-470 / :490-556),
//   3. sweeps the fixed-stride sample regions out of LDS, split into 1 KiB wave-steps that
//      all 8 waves share (vcfxg_gt.h fast_dword: the reference's parseGenotypeAndCount
//      :262-293 on single-digit diploid GT-only records), and
//   4. writes each line's end offset, counts, status and head record to the block's region.
// So every input byte is read from HBM once (the two-sweep schedule reads it twice).  Lines
// that start more than one chunk back, lines whose sweep leaves the fixed-stride layout and
// non-GT-first records go to k_af_complex (the exact per-line path, from global memory),
// exactly as after the two-sweep schedule.  k_af_stream_compact then concatenates the
// blocks' regions in file order.  A chunk ending more than kMaxL lines, or a block over its
// line capacity (lines shorter than ~512 B on average), raises `overflow` and the caller
// reruns the two-sweep schedule.
#include <algorithm>

#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"
#include "vcfxg_meta.h"

namespace vcfxg {

namespace {

constexpr int kSC = 32768;                     // chunk bytes
constexpr int kRingN = 4;                      // ring slots: chunk q lives in slot q & 3
constexpr int kRingBytes = kSC * kRingN;       // 128 KiB
constexpr int64_t kRingMask = kRingBytes - 1;
constexpr int kStThreads = 512;
constexpr int kStWaves = kStThreads / kWave;   // 8
constexpr int kMaxL = 512;                     // lines ending in one chunk
constexpr int kGldsPerWave = kSC / 1024 / kStWaves;  // 1 KiB glds instructions per wave per chunk
static_assert(kGldsPerWave == 4, "vmcnt counts below assume 4 staging loads per wave per chunk");

struct RingSrc {
    const char *lds;
    int64_t a0;  // file offset of the chunk grid origin (ring offset 0 of chunk 0)
    __device__ __forceinline__ uint4 load16(int64_t x) const {
        return *reinterpret_cast<const uint4 *>(lds + ((x - a0) & kRingMask));
    }
    __device__ __forceinline__ uint32_t load4(int64_t x) const {
        return *reinterpret_cast<const uint32_t *>(lds + ((x - a0) & kRingMask));
    }
    __device__ __forceinline__ uint32_t byte(int64_t x) const { return (uint8_t)lds[(x - a0) & kRingMask]; }
};

// per line ending in the current chunk (LDS)
struct LMeta {
    int32_t s;       // sample start - C (GT-first lines)
    int32_t ls;      // line start - C (may be negative: started in the previous chunk)
    uint32_t rowpre;
    uint8_t kind, sep, cr, fast;  // fast: eligible for the fixed-stride sweep
};

struct StreamLds {
    char ring[kRingBytes];
    LMeta lm[kMaxL];
    uint32_t segpre[kMaxL + 1];
    uint32_t acc_alt[kMaxL], acc_tot[kMaxL], acc_err[kMaxL];
    uint16_t ends[kMaxL + 1];   // line end - C, ascending
    uint32_t wsum[kStWaves];
    int64_t carry_nl[kStWaves];  // block max of a newline position
    uint32_t cnt[4];             // block counters (rows, data lines, warn, general)
};

__device__ __forceinline__ void glds16(const char *src, char *lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

// raw barrier: LDS writes of this wave done, every wave here; staging loads stay in flight
__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// exclusive block scan of one value per thread (kStThreads); returns the prefix, *total
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *wsum, uint32_t &total) {
    const int w = threadIdx.x / kWave;
    const uint32_t incl = wave_incl_scan(v);
    if (lane() == kWave - 1) wsum[w] = incl;
    bar();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < kStWaves; k++) {
        const uint32_t x = wsum[k];
        if (k < w) before += x;
        total += x;
    }
    bar();  // wsum reusable
    return before + incl - v;
}

}  // namespace

__global__ __launch_bounds__(kStThreads) void k_af_stream(const char *__restrict__ buf, int64_t lo, int64_t hi,
                                                          int64_t a0, int64_t nchunks, int64_t n_alloc, int mode,
                                                          int tail, uint64_t cap_b, uint64_t *__restrict__ le_o,
                                                          int32_t *__restrict__ alt_o, int32_t *__restrict__ tot_o,
                                                          uint32_t *__restrict__ rowpre_o,
                                                          uint8_t *__restrict__ status_o,
                                                          LineMeta *__restrict__ meta_o,
                                                          uint64_t *__restrict__ bcount, unsigned *overflow,
                                                          unsigned long long *__restrict__ counters) {
    __shared__ __attribute__((aligned(16))) StreamLds L;
    const int t = threadIdx.x, w = t / kWave, l = lane();
    const int64_t G = gridDim.x, b = blockIdx.x;
    const int64_t q0 = b * nchunks / G, q1 = (b + 1) * nchunks / G;
    const RingSrc src{L.ring, a0};
    const int strip_cr = mode == 0 ? 1 : 0;
    if (t < 4) L.cnt[t] = 0;
    // chunk q -> ring slot q & 3; out-of-range chunks load a harmless clamped slice into a
    // slot nobody reads any more, so every wave issues exactly 4 staging loads per chunk
    auto stage = [&](int64_t q) {
#pragma unroll
        for (int i = 0; i < kGldsPerWave; i++) {
            const int idx = kGldsPerWave * w + i;  // 1 KiB slice of the chunk
            int64_t sa = a0 + q * kSC + idx * 1024 + 16 * l;
            if (sa < 0) sa = 0;
            if (sa > n_alloc - 16) sa = (n_alloc - 16) & ~(int64_t)15;
            glds16(buf + sa, L.ring + ((q & (kRingN - 1)) * kSC) + idx * 1024);
        }
    };
    stage(q0 - 1);
    stage(q0);
    stage(q0 + 1);
    stage(q0 + 2);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // chunks q0-1 and q0 landed (this wave)
    bar();
    // start of the first line ending in chunk q0: after the last newline of chunk q0 - 1
    // (or lo); -1: it started before chunk q0 - 1 (the far path)
    int64_t carry;
    {
        const int64_t C = a0 + q0 * kSC, P = C - kSC;
        int64_t best = -1;
        if (q0 > 0) {
            const int64_t blk = P + 64 * t;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t x = blk + 16 * k;
                uint32_t m = eq_mask16(src.load16(x), kRepNl) & range_mask16(x, lo > P ? lo : P, C < hi ? C : hi);
                if (m) best = x + 31 - __builtin_clz(m);
            }
        }
        for (int o = 32; o > 0; o >>= 1) {
            const int64_t y = __shfl_xor(best, o);
            best = y > best ? y : best;
        }
        if (l == 0) L.carry_nl[w] = best;
        bar();
        best = -1;
#pragma unroll
        for (int k = 0; k < kStWaves; k++) best = L.carry_nl[k] > best ? L.carry_nl[k] : best;
        if (best >= 0) carry = best + 1;
        else carry = lo >= P ? lo : -1;  // (q0 == 0: P < a0 <= lo)
        if (carry >= 0 && carry < lo) carry = lo;
        bar();
    }
    uint64_t base = 0;  // lines written by this block
    bool ovf = false;
    for (int64_t q = q0; q < q1; q++) {
        const int64_t C = a0 + q * kSC;
        // chunk q's staging loads are older than the 8 of chunks q+1, q+2
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        bar();
        // 1. newlines of chunk q (64 B per thread), in file order
        uint32_t nl[4];
        uint32_t c = 0;
        {
            const int64_t blk = C + 64 * t;
            const int64_t rlo = lo > C ? lo : C;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t x = blk + 16 * k;
                nl[k] = eq_mask16(src.load16(x), kRepNl) & range_mask16(x, rlo, hi);
                c += __popc(nl[k]);
            }
        }
        uint32_t n_nl;
        uint32_t at = block_excl(c, L.wsum, n_nl);
        if (n_nl > (uint32_t)kMaxL) {
            ovf = true;
            break;  // block-uniform
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t m = nl[k];
            while (m) {
                const int j = __builtin_ctz(m);
                m &= m - 1u;
                L.ends[at++] = (uint16_t)(64 * t + 16 * k + j);
            }
        }
        bar();
        uint32_t n_end = n_nl;
        // the input's last line without '\n' ends at hi (as after the two-sweep index)
        if (tail && q == nchunks - 1) {  // (the input does not end in '\n': that line exists)
            if (n_nl + 1 > (uint32_t)kMaxL) {
                ovf = true;
                break;
            }
            if (t == 0) L.ends[n_nl] = (uint16_t)(hi - C);
            n_end = n_nl + 1;
            bar();
        }
        if (base + n_end > cap_b) {
            ovf = true;
            break;
        }
        // 2. heads
        uint32_t nseg_mine = 0;
        for (uint32_t i = t; i < (uint32_t)kMaxL; i += kStThreads) {
            if (i >= n_end) continue;
            const int64_t e = C + L.ends[i];
            const int64_t ls = i ? C + L.ends[i - 1] + 1 : carry;
            LMeta x{};
            x.ls = (int32_t)(ls - C);
            uint32_t nseg = 0;
            if (ls < 0 || ls < C - kSC) {
                x.kind = kMetaFull;  // started before the ring: the full per-line path
                x.ls = 0;
            } else {
                const LineMeta m = head_meta(src, ls, e, strip_cr);
                x.kind = m.kind;
                x.cr = m.cr;
                x.rowpre = m.rowpre;
                x.sep = m.sep;
                if (m.kind == kMetaGt) {
                    x.s = (int32_t)((int64_t)m.S - C);
                    const int64_t S = (int64_t)m.S, AE = e - m.cr, Ln = AE - S;
                    const bool ok = Ln >= 3 && !((Ln + 1) & 3) && (m.sep == '/' || m.sep == '|');
                    x.fast = ok ? 1 : 0;
                    if (ok) nseg = (uint32_t)((AE - (S & ~(int64_t)15) + kWaveStep - 1) / kWaveStep);
                }
            }
            L.lm[i] = x;
            L.acc_alt[i] = L.acc_tot[i] = L.acc_err[i] = 0;
            nseg_mine = nseg;  // kMaxL == kStThreads: one line per thread
        }
        uint32_t nseg_total;
        const uint32_t sp = block_excl(nseg_mine, L.wsum, nseg_total);
        if ((uint32_t)t < n_end) L.segpre[t] = sp;
        if (t == 0) L.segpre[n_end] = nseg_total;
        bar();
        // 3. fixed-stride sweeps, 1 KiB wave-steps shared by the 8 waves
        for (uint32_t g = w; g < nseg_total; g += kStWaves) {
            uint32_t lo_i = 0, hi_i = n_end;  // last line with segpre <= g
            while (hi_i - lo_i > 1) {
                const uint32_t mid = (lo_i + hi_i) / 2;
                if (L.segpre[mid] <= g) lo_i = mid;
                else hi_i = mid;
            }
            const uint32_t i = lo_i;
            const LMeta x = L.lm[i];
            const int64_t S = C + x.s, AE = C + L.ends[i] - x.cr;
            const uint32_t sepc = x.sep;
            const uint32_t exp_xor = 0x09000000u | (sepc << 8) | 0x00300030u;
            const uint32_t neutral = 0x092E002Eu | (sepc << 8);
            const int s = (int)(S & 3);
            const int64_t wstep = (S & ~(int64_t)15) + (int64_t)(g - L.segpre[i]) * kWaveStep;
            const int64_t blk = wstep + 16 * (int64_t)l;
            AfOp op{buf, AE, 0};
            uint32_t err = 0;
            if (blk < AE) {
                const uint4 v = src.load16(blk);
                const uint32_t x4 = src.load4(blk + 16);
                uint32_t d[4] = {__builtin_amdgcn_alignbyte(v.y, v.x, s), __builtin_amdgcn_alignbyte(v.z, v.y, s),
                                 __builtin_amdgcn_alignbyte(v.w, v.z, s), __builtin_amdgcn_alignbyte(x4, v.w, s)};
                bool real[4] = {true, true, true, true};
                const bool interior = (wstep + s >= S) && (wstep + kWaveStep - 4 + s + 3 < AE);
                if (!interior) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int64_t p = blk + s + 4 * k;
                        if (p < S || p + 3 > AE) {
                            d[k] = neutral;
                            real[k] = false;
                        } else if (p + 3 == AE) d[k] = (d[k] & 0x00FFFFFFu) | 0x09000000u;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; k++) fast_dword(d[k], exp_xor, err, op, real[k], blk + s + 4 * k);
            }
            const uint32_t sa = wave_sum(op.alt), st = wave_sum(op.tot);
            const bool bad = __any(err != 0u);
            if (l == 0) {
                if (sa) atomicAdd(&L.acc_alt[i], sa);
                if (st) atomicAdd(&L.acc_tot[i], st);
                if (bad) L.acc_err[i] = 1;
            }
        }
        bar();
        // 4. outputs (one line per thread)
        if ((uint32_t)t < n_end) {
            const uint32_t i = t;
            const LMeta x = L.lm[i];
            const uint64_t o = (uint64_t)b * cap_b + base + i;
            LineMeta m{};
            m.kind = x.kind;
            m.cr = x.cr;
            m.sep = x.sep;
            m.rowpre = x.rowpre;
            m.S = x.kind == kMetaGt ? (uint64_t)(C + x.s) : 0;
            uint8_t st = 0;
            uint32_t alt = 0, tot = 0, rowpre = 0;
            if (x.kind == kMetaGt) {
                atomicAdd(&L.cnt[1], 1u);
                atomicAdd(&L.cnt[0], 1u);
                rowpre = x.rowpre;
                if (x.fast && !L.acc_err[i]) {
                    st = 1;
                    alt = L.acc_alt[i];
                    tot = L.acc_tot[i];
                } else {
                    st = kAfPending;  // k_af_complex runs the general sweep
                }
            }
            le_o[o] = (uint64_t)(C + L.ends[i]);
            alt_o[o] = (int32_t)alt;
            tot_o[o] = (int32_t)tot;
            rowpre_o[o] = rowpre;
            status_o[o] = st;
            meta_o[o] = m;
        }
        if (n_nl) carry = C + L.ends[n_nl - 1] + 1;
        base += n_end;
        bar();  // chunk q-1 no longer read: its slot takes chunk q+3
        stage(q + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ovf && t == 0) atomicOr(overflow, 1u);
    __syncthreads();
    if (t == 0) bcount[b] = base;
    if (t < 4 && L.cnt[t]) atomicAdd(&counters[t], (unsigned long long)L.cnt[t]);
}

// the blocks' regions -> dense per-line arrays in file order (each block sums the counts of
// the blocks before it); the last block publishes the line count
__global__ __launch_bounds__(256) void k_af_stream_compact(uint64_t cap_b, const uint64_t *__restrict__ bcount,
                                                           const uint64_t *__restrict__ le_b,
                                                           const int32_t *__restrict__ alt_b,
                                                           const int32_t *__restrict__ tot_b,
                                                           const uint32_t *__restrict__ rowpre_b,
                                                           const uint8_t *__restrict__ status_b,
                                                           const LineMeta *__restrict__ meta_b, uint64_t *line_end,
                                                           int32_t *alt, int32_t *tot, uint32_t *rowpre,
                                                           uint8_t *status, LineMeta *meta, uint64_t *n_lines) {
    __shared__ uint64_t red[256 / kWave];
    const int64_t b = blockIdx.x;
    uint64_t pre = 0;
    for (int64_t k = threadIdx.x; k < b; k += blockDim.x) pre += bcount[k];
    pre = wave_sum(pre);
    if (lane() == 0) red[threadIdx.x / kWave] = pre;
    __syncthreads();
    uint64_t gb = 0;
    for (int k = 0; k < (int)(blockDim.x / kWave); k++) gb += red[k];
    const uint64_t n = bcount[b];
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t s = (uint64_t)b * cap_b + i, d = gb + i;
        line_end[d] = le_b[s];
        alt[d] = alt_b[s];
        tot[d] = tot_b[s];
        rowpre[d] = rowpre_b[s];
        status[d] = status_b[s];
        meta[d] = meta_b[s];
    }
    if (b == (int64_t)gridDim.x - 1 && threadIdx.x == 0) *n_lines = gb + n;
}

int64_t af_stream_chunks(int64_t lo, int64_t hi) {
    const int64_t a0 = lo & ~(int64_t)15;
    return hi > lo ? (hi - a0 + kSC - 1) / kSC : 0;
}

hipError_t launch_af_stream(const char *buf, int64_t lo, int64_t hi, int64_t n_alloc, int mode, int tail, int grid,
                            uint64_t cap_b, uint64_t *le_b, int32_t *alt_b, int32_t *tot_b, uint32_t *rowpre_b,
                            uint8_t *status_b, void *meta_b, uint64_t *bcount, unsigned *overflow,
                            unsigned long long *counters, hipStream_t s) {
    const int64_t a0 = lo & ~(int64_t)15;
    const int64_t nc = af_stream_chunks(lo, hi);
    if (!nc || grid <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_af_stream, dim3(grid), dim3(kStThreads), 0, s, buf, lo, hi, a0, nc, n_alloc, mode, tail, cap_b,
                       le_b, alt_b, tot_b, rowpre_b, status_b, static_cast<LineMeta *>(meta_b), bcount, overflow,
                       counters);
    return hipGetLastError();
}

hipError_t launch_af_stream_compact(int grid, uint64_t cap_b, const uint64_t *bcount, const uint64_t *le_b,
                                    const int32_t *alt_b, const int32_t *tot_b, const uint32_t *rowpre_b,
                                    const uint8_t *status_b, const void *meta_b, uint64_t *line_end, int32_t *alt,
                                    int32_t *tot, uint32_t *rowpre, uint8_t *status, void *meta, uint64_t *n_lines,
                                    hipStream_t s) {
    hipLaunchKernelGGL(k_af_stream_compact, dim3(grid), dim3(256), 0, s, cap_b, bcount, le_b, alt_b, tot_b, rowpre_b,
                       status_b, static_cast<const LineMeta *>(meta_b), line_end, alt, tot, rowpre, status,
                       static_cast<LineMeta *>(meta), n_lines);
    return hipGetLastError();
}

}  // namespace vcfxg
