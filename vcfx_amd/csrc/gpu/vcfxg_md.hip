// vcfxg_md.hip -- VCFX_missing_detector's per-record test (a per-sample GT
// predicate on the record path).
//
// One wave per indexed line: the head's first 9 tabs (INFO span, sample start), then a sweep
// of the sample bytes 16 B per lane for '.'.  Each '.' found is tested against the rule of
// hasMissingGenotypeInSamples (VCFX_missing_detector.cpp:290-336): it lies in its sample's
// first ':' sub-field (no ':' between the sample start and it) and starts or ends that
// sub-field or touches a '/' or '|'.  The sweep stops at the first such '.'.  Besides the
// flag, every line reports whether its sample bytes hold any '.' at all: the file path's
// pre-scan (sampleColumnsHaveAnyDots :371-445) sends the whole input through unchanged when
// no line that ends in '\n' has one.
//
// Semantics per mode: file (processMmapZeroCopy :450-589): a trailing '\r' is dropped before
// the line is tested, an empty line or a '#' line is copied; stdin (detectMissingGenotypes
// :860-911): the line as getline gives it.  Output of a flagged line (the host writes it):
// INFO becomes "MISSING_GENOTYPES=1" when empty or ".", else gains ";MISSING_GENOTYPES=1".
#include "vcfxg_device.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

constexpr int kMdThreads = 256;
constexpr int kMdWaves = kMdThreads / kWave;
constexpr uint32_t kRepDot = 0x2E2E2E2Eu;

__device__ __forceinline__ bool md_gt_sep(uint32_t c) { return c == '/' || c == '|'; }

// the '.' at q (sp <= q < ae) makes its sample missing
__device__ __forceinline__ bool md_dot_missing(const char *__restrict__ buf, int64_t sp, int64_t ae, int64_t q) {
    const uint32_t pv = q > sp ? byte_at(buf, q - 1) : (uint32_t)'\t';
    const uint32_t nx = q + 1 < ae ? byte_at(buf, q + 1) : (uint32_t)'\t';
    if (!(pv == '\t' || md_gt_sep(pv) || nx == ':' || nx == '\t' || md_gt_sep(nx))) return false;
    // in the GT sub-field: no ':' back to the sample start
    for (int64_t p = q - 1; p >= sp; p--) {
        const uint32_t c = byte_at(buf, p);
        if (c == '\t') break;
        if (c == ':') return false;
    }
    return true;
}

// sweep of [sp, ae): any '.', and the first missing sample (wave-uniform results)
__device__ __forceinline__ void md_sweep(const char *__restrict__ buf, int64_t sp, int64_t ae, bool &dot,
                                         bool &miss) {
    constexpr int kU = 4;
    const int64_t b0 = sp & ~(int64_t)15;
    const int64_t lastblk = (ae - 1) & ~(int64_t)15;
    for (int64_t w0 = b0; w0 < ae; w0 += kU * kWaveStep) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {  // branch-free: lanes past the line re-read its last block
            const int64_t blk = w0 + u * kWaveStep + lane() * kBlockBytes;
            v[u] = load16(buf, blk < ae ? blk : lastblk);
        }
        bool m = false;
        uint32_t any = 0;
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int64_t blk = w0 + u * kWaveStep + lane() * kBlockBytes;
            uint32_t dm = blk < ae ? eq_mask16(v[u], kRepDot) & range_mask16(blk, sp, ae) : 0u;
            any |= dm;
            while (dm && !m) {
                const int j = __builtin_ctz(dm);
                dm &= dm - 1u;
                m = md_dot_missing(buf, sp, ae, blk + j);
            }
        }
        dot = dot || __any(any != 0u);
        if (__any(m)) {
            miss = true;
            return;
        }
    }
}

__global__ __launch_bounds__(kMdThreads) void k_md_lines(const char *__restrict__ buf, int64_t data_start,
                                                         int64_t n_input, const uint64_t *__restrict__ line_end,
                                                         const uint64_t *n_lines_p, int mode, int walk,
                                                         uint8_t *__restrict__ status, int32_t *__restrict__ info_s,
                                                         int32_t *__restrict__ info_e,
                                                         unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kMdWaves][16];
    __shared__ uint32_t red[3][kMdWaves];
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    uint32_t data = 0, flagged = 0, dots = 0;  // (wave-uniform)
    // one line with the whole wave
    auto one = [&](uint64_t li) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start, le = (int64_t)line_end[li];
        int64_t ae = le;
        if (mode == 0 && ae > ls && byte_at(buf, ae - 1) == '\r') ae--;
        uint8_t st = 0;
        int32_t is = 0, ie = 0;
        bool dot = false, miss = false;
        const uint8_t ws = walk ? status[li] : (uint8_t)0xFF;
        if (ws == kMdFlag) {  // the walk found a missing sample: the INFO span
            int64_t t[9];
            const int nt = head_tabs(buf, ls, ae, 9, t, lds);
            (void)nt;  // (a fixed-stride record has its 9 tabs)
            data++;
            flagged++;
            st = kMdFlag;
            is = (int32_t)(t[6] + 1 - ls);
            ie = (int32_t)(t[7] - ls);
            dots += le < n_input;
        } else if (ae > ls) {
            const bool hash = byte_at(buf, ls) == '#';
            int64_t t[9];
            // a '#' line is copied, but the file pre-scan looks at its "sample" bytes too
            const int nt = (!hash || mode == 0) ? head_tabs(buf, ls, ae, 9, t, lds) : 0;
            const int64_t sp = nt >= 9 ? t[8] + 1 : ae;
            if (sp < ae) md_sweep(buf, sp, ae, dot, miss);
            if (hash) st = 4;
            else {
                data++;
                st = 1;
                if (miss) {
                    st = kMdFlag;
                    flagged++;
                    is = (int32_t)(t[6] + 1 - ls);
                    ie = (int32_t)(t[7] - ls);
                }
            }
            // the pre-scan reads only lines that end in '\n'
            dots += dot && le < n_input;
        }
        if (lane() == 0) {
            status[li] = st;
            info_s[li] = is;
            info_e[li] = ie;
        }
    };
    if (walk) {
        // 64 lines per step, a lane each: the walk's fixed-stride records without a '.' allele
        // (status 1: no '.' at all) are counted by the lanes; the wave takes the others in turn
        for (uint64_t b0 = wid * kWave; b0 < n_lines; b0 += nw * kWave) {
            const uint64_t li = b0 + lane();
            const uint8_t st = li < n_lines ? status[li] : (uint8_t)0;
            const bool plain = li < n_lines && st == 1;
            if (plain) {
                info_s[li] = 0;
                info_e[li] = 0;
            }
            data += (uint32_t)__popcll(__ballot(plain));
            uint64_t todo = __ballot(li < n_lines && st != 1);
            while (todo) {
                const int j = __builtin_ctzll(todo);
                todo &= todo - 1;
                one(b0 + j);
            }
        }
    } else
        for (uint64_t li = wid; li < n_lines; li += nw) one(li);
    if (lane() == 0) {
        red[0][threadIdx.x / kWave] = data;
        red[1][threadIdx.x / kWave] = flagged;
        red[2][threadIdx.x / kWave] = dots;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint32_t t = 0;
        for (int k = 0; k < kMdWaves; k++) t += red[threadIdx.x][k];
        if (t) atomicAdd(&counters[threadIdx.x], (unsigned long long)t);
    }
}

hipError_t launch_md_lines(const char *buf, int64_t data_start, int64_t n_input, const uint64_t *line_end,
                           const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, uint8_t *status,
                           int32_t *info_s, int32_t *info_e, unsigned long long *counters, hipStream_t s, int walk) {
    if (!n_lines_host) return hipSuccess;
    int64_t g = ((int64_t)n_lines_host + kMdWaves - 1) / kMdWaves;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_md_lines, dim3((unsigned)g), dim3(kMdThreads), 0, s, buf, data_start, n_input, line_end,
                       n_lines_dev, mode, walk, status, info_s, info_e, counters);
    return hipGetLastError();
}

}  // namespace vcfxg
