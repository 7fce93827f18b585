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

struct Field {
    int64_t p, e;
};

// extractField(line, i) for i <= 7 given the first nt (<= 8) tab offsets
__device__ __forceinline__ Field field_of(const int64_t *t, int nt, int64_t ls, int64_t ae, int i) {
    if (nt < i) return {ae, ae};  // "not enough fields" -> empty
    int64_t p = i ? t[i - 1] + 1 : ls;
    int64_t e = nt > i ? t[i] : ae;
    return {p, e};
}

__device__ __forceinline__ bool bytes_eq(const char *buf, int64_t p, int64_t n, const char *pool, uint32_t off,
                                         uint32_t len) {
    if ((uint64_t)n != len) return false;
    for (uint32_t k = 0; k < len; k++)
        if (buf[p + k] != pool[off + k]) return false;
    return true;
}

__device__ bool eval_crit(const char *__restrict__ buf, const int64_t *t, int nt, int64_t ls, int64_t ae,
                          const RfCrit &c, const char *__restrict__ pool) {
    bool parsed;
    switch (c.target) {
    case RF_POS: {
        Field f = field_of(t, nt, ls, ae, 1);
        if (f.e <= f.p) return false;
        return num_compare(buf, f.p, f.e, c.T, c.op, pool, &parsed);
    }
    case RF_QUAL: {
        Field f = field_of(t, nt, ls, ae, 5);
        if (f.e <= f.p || (f.e - f.p == 1 && buf[f.p] == '.')) return cmp_double(0.0, c.op, c.T.t);
        return num_compare(buf, f.p, f.e, c.T, c.op, pool, &parsed);
    }
    case RF_FILTER: {
        if (c.numeric) return false;
        Field f = field_of(t, nt, ls, ae, 6);
        bool eq = bytes_eq(buf, f.p, f.e - f.p, pool, c.str_off, c.str_len);
        return c.op == OPN_EQ ? eq : (c.op == OPN_NE ? !eq : false);
    }
    default: {
        Field f = field_of(t, nt, ls, ae, 7);
        if (f.e <= f.p || (f.e - f.p == 1 && buf[f.p] == '.')) return false;
        // token scan
        int64_t p = f.p;
        int64_t vp = -1, ve = -1;
        while (p < f.e) {
            int64_t te = p;
            while (te < f.e && buf[te] != ';') te++;
            int64_t eq = p;
            while (eq < te && buf[eq] != '=') eq++;
            if (eq < te) {
                if (bytes_eq(buf, p, eq - p, pool, c.key_off, c.key_len)) {
                    vp = eq + 1;
                    ve = te;
                    break;
                }
            } else if (bytes_eq(buf, p, te - p, pool, c.key_off, c.key_len)) {
                vp = p;
                ve = te;
                break;
            }
            p = te + 1;
        }
        if (vp < 0) return false;
        if (c.numeric) {
            if (ve <= vp) return false;
            return num_compare(buf, vp, ve, c.T, c.op, pool, &parsed);
        }
        bool eq = bytes_eq(buf, vp, ve - vp, pool, c.str_off, c.str_len);
        return c.op == OPN_EQ ? eq : (c.op == OPN_NE ? !eq : false);
    }
    }
}

// status: 0 empty (after '\r' strip; printed as "\n"), 4 header, 1 kept, 2 dropped
__global__ __launch_bounds__(256) void k_rf_records(const char *__restrict__ buf, int64_t data_start,
                                                    const uint64_t *__restrict__ line_end, const uint64_t *n_lines_p,
                                                    const RfCrit *__restrict__ crit, int ncrit, int and_logic,
                                                    const char *__restrict__ pool, uint8_t *__restrict__ status,
                                                    unsigned long long *__restrict__ counters) {
    __shared__ uint32_t cnt[2];
    if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t n = *n_lines_p;
    uint32_t kept = 0, data = 0;
    for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < n; li += gridDim.x * (uint64_t)blockDim.x) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
        int64_t ae = (int64_t)line_end[li];
        if (ae > ls && buf[ae - 1] == '\r') ae--;  // :454-456 / :509-511
        uint8_t st;
        if (ae == ls) st = 0;
        else if (buf[ls] == '#') st = 4;
        else {
            data++;
            int64_t t[8];
            int nt = 0;
            for (int64_t p = ls; p < ae && nt < 8; p++)
                if (buf[p] == '\t') t[nt++] = p;
            bool res;
            if (and_logic) {
                res = true;
                for (int k = 0; k < ncrit && res; k++) res = eval_crit(buf, t, nt, ls, ae, crit[k], pool);
            } else {
                res = false;
                for (int k = 0; k < ncrit && !res; k++) res = eval_crit(buf, t, nt, ls, ae, crit[k], pool);
            }
            st = res ? 1 : 2;
            kept += res;
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
                             uint8_t *status, unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    int64_t g = ((int64_t)n_lines_host + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_rf_records, dim3((unsigned)g), dim3(256), 0, s, buf, data_start, line_end, n_lines_dev, crit,
                       ncrit, and_logic, pool, status, counters);
    return hipGetLastError();
}

}  // namespace vcfxg
