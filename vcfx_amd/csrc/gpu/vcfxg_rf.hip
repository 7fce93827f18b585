// vcfxg_rf.hip -- VCFX_record_filter predicates on the device: one thread per line.
//
// Per data line (evaluateLine, VCFX_record_filter.cpp:383-401): AND / OR over compiled
// criteria on POS (field 1), QUAL (field 5), FILTER (field 6) or an INFO key (field 7).
// Field extraction restates extractField (:207-229) -- fewer tabs than the index gives an
// empty field -- and extractInfoValue (:234-267) -- first ';' token whose '='-key (or, for
// a flag, whole token) equals the key.  Numbers are strtod-exact via vcfxg_num.h.
#include "vcfxg_device.h"
#include "vcfxg_num.h"
#include "vcfxg_rf.h"

namespace vcfxg {

// status: 0 empty (after '\r' strip; printed as "\n"), 4 header, 1 kept, 2 dropped, 5 to be
// decided on the host (an RF_QUAL_LENIENT criterion met an unparsable QUAL)
__global__ __launch_bounds__(256) void k_rf_records(const char *__restrict__ buf, int64_t data_start,
                                                    const uint64_t *__restrict__ line_end, const uint64_t *n_lines_p,
                                                    const RfCrit *__restrict__ crit, int ncrit, int and_logic,
                                                    const char *__restrict__ pool, uint8_t *__restrict__ status,
                                                    unsigned long long *__restrict__ counters, int keep_cr) {
    __shared__ uint32_t cnt[2];
    if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t n = *n_lines_p;
    uint32_t kept = 0, data = 0;
    for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < n; li += gridDim.x * (uint64_t)blockDim.x) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
        int64_t ae = (int64_t)line_end[li];
        if (!keep_cr && ae > ls && buf[ae - 1] == '\r') ae--;  // :454-456 / :509-511
        uint8_t st;
        if (ae == ls) st = 0;
        else if (buf[ls] == '#') st = 4;
        else {
            data++;
            bool recheck = false;
            const bool res = rf_line(buf, ls, ae, crit, ncrit, and_logic, pool, &recheck);
            st = recheck ? 5 : (res ? 1 : 2);
            kept += res && !recheck;
        }
        status[li] = st;
    }
    kept = wave_sum(kept);
    data = wave_sum(data);
    if (lane() == 0) {
        if (kept) atomicAdd(&cnt[0], kept);
        if (data) atomicAdd(&cnt[1], data);
    }
    __syncthreads();
    if (threadIdx.x < 2 && cnt[threadIdx.x]) atomicAdd(&counters[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

// VCFX_variant_counter per line (countVariantsMmap :352-388 / processLine :182-202):
// status 0 = empty or '#', 1 = counted (>= 7 tabs, hasEightColumnsFast :31-44), 3 = fewer
// columns.  strip_cr: the file path drops a trailing '\r' before the column check.
__global__ __launch_bounds__(256) void k_vc_records(const char *__restrict__ buf, int64_t data_start,
                                                    const uint64_t *__restrict__ line_end, const uint64_t *n_lines_p,
                                                    int strip_cr, uint8_t *__restrict__ status,
                                                    unsigned long long *__restrict__ counters) {
    __shared__ uint32_t cnt[2];
    if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t n = *n_lines_p;
    uint32_t good = 0, bad = 0;
    for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < n; li += gridDim.x * (uint64_t)blockDim.x) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
        int64_t ae = (int64_t)line_end[li];
        uint8_t st = 0;
        if (ae > ls && buf[ls] != '#') {
            if (strip_cr && buf[ae - 1] == '\r') ae--;
            int nt = 0;
            for (int64_t p = ls; p < ae && nt < 7; p++) nt += buf[p] == '\t';
            st = nt >= 7 ? 1 : 3;
        }
        good += st == 1;
        bad += st == 3;
        status[li] = st;
    }
    good = wave_sum(good);
    bad = wave_sum(bad);
    if (lane() == 0) {
        if (good) atomicAdd(&cnt[0], good);
        if (bad) atomicAdd(&cnt[1], bad);
    }
    __syncthreads();
    if (threadIdx.x < 2 && cnt[threadIdx.x]) atomicAdd(&counters[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

hipError_t launch_vc_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int strip_cr, uint8_t *status, unsigned long long *counters,
                             hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    int64_t g = ((int64_t)n_lines_host + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_vc_records, dim3((unsigned)g), dim3(256), 0, s, buf, data_start, line_end, n_lines_dev,
                       strip_cr, status, counters);
    return hipGetLastError();
}

hipError_t launch_rf_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, const RfCrit *crit, int ncrit, int and_logic, const char *pool,
                             uint8_t *status, unsigned long long *counters, hipStream_t s, int keep_cr) {
    if (!n_lines_host) return hipSuccess;
    int64_t g = ((int64_t)n_lines_host + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_rf_records, dim3((unsigned)g), dim3(256), 0, s, buf, data_start, line_end, n_lines_dev, crit,
                       ncrit, and_logic, pool, status, counters, keep_cr);
    return hipGetLastError();
}

}  // namespace vcfxg
