// vcfxg_rf.h -- compiled record_filter criterion (device layout) and launcher.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vcfxg_num.h"

namespace vcfxg {

// RF_QUAL_LENIENT: the legacy free function recordPasses in OR mode (VCFX_record_filter.cpp:
// 736-739) compares whatever strtod made of an unparsable QUAL; the device flags such lines
// for the host (vcfxg_record_filter_ex status VCFXG_LINE_RECHECK) instead of restating strtod's
// prefix rules
enum { RF_POS = 0, RF_QUAL = 1, RF_FILTER = 2, RF_INFO = 3, RF_QUAL_LENIENT = 4 };

struct RfCrit {
    int target, op, numeric;
    NumThreshold T;
    uint32_t key_off, key_len;  // INFO key in the pool
    uint32_t str_off, str_len;  // string value in the pool
};

// ---- device evaluation (restating VCFX_record_filter.cpp; shared by k_rf_records and the walk)
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

template <class B, class PB>
__device__ __forceinline__ bool bytes_eq(const B &buf, int64_t p, int64_t n, const PB &pool, uint32_t off,
                                         uint32_t len) {
    if ((uint64_t)n != len) return false;
    for (uint32_t k = 0; k < len; k++)
        if (buf[p + k] != pool[off + k]) return false;
    return true;
}

template <class B, class PB>
__device__ inline bool eval_crit(const B &buf, const int64_t *t, int nt, int64_t ls, int64_t ae, const RfCrit &c,
                                 const PB &pool, bool *recheck = nullptr) {
    bool parsed;
    switch (c.target) {
    case RF_POS: {
        Field f = field_of(t, nt, ls, ae, 1);
        if (f.e <= f.p) return false;
        return num_compare(buf, f.p, f.e, c.T, c.op, pool, &parsed);
    }
    case RF_QUAL:
    case RF_QUAL_LENIENT: {
        Field f = field_of(t, nt, ls, ae, 5);
        if (f.e <= f.p || (f.e - f.p == 1 && buf[f.p] == '.')) return cmp_double(0.0, c.op, c.T.t);
        const bool res = num_compare(buf, f.p, f.e, c.T, c.op, pool, &parsed);
        if (c.target == RF_QUAL_LENIENT && !parsed && recheck) *recheck = true;
        return res;
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


// evaluateLine (:383-401) given the line's first nt (<= 8) tab offsets: AND short-circuits
// on the first false criterion, OR on the first true one.  CS: criteria source (crit[k] ->
// RfCrit), B / PB: byte sources as in vcfxg_num.h
template <class B, class CS, class PB>
__device__ inline bool rf_eval(const B &buf, const int64_t *t, int nt, int64_t ls, int64_t ae, const CS &crit,
                               int ncrit, int and_logic, const PB &pool, bool *recheck = nullptr) {
    bool res = and_logic ? true : false;
    for (int k = 0; k < ncrit && res == (bool)and_logic; k++) {
        const RfCrit c = crit[k];
        res = eval_crit(buf, t, nt, ls, ae, c, pool, recheck);
    }
    return res;
}
// the same for the data line [ls, ae) ('\r' already stripped): one thread, byte loop
__device__ inline bool rf_line(const char *__restrict__ buf, int64_t ls, int64_t ae, const RfCrit *__restrict__ crit,
                               int ncrit, int and_logic, const char *__restrict__ pool, bool *recheck = nullptr) {
    int64_t t[8];
    int nt = 0;
    for (int64_t p = ls; p < ae && nt < 8; p++)
        if (buf[p] == '\t') t[nt++] = p;
    return rf_eval(buf, t, nt, ls, ae, crit, ncrit, and_logic, pool, recheck);
}

hipError_t launch_vc_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int strip_cr, uint8_t *status, unsigned long long *counters,
                             hipStream_t s);
// keep_cr: evaluate each line with its trailing '\r' (the legacy processVCF's getline lines)
hipError_t launch_rf_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, const RfCrit *crit, int ncrit, int and_logic, const char *pool,
                             uint8_t *status, unsigned long long *counters, hipStream_t s, int keep_cr = 0);

// ---- the filter / query walk (vcfxg_fq_walk.hip): record_filter (kFqRF), genotype_query
// (kFqGQ) or the fused pipeline (kFqBoth) in one pass without a separate line index
enum { kFqRF = 1, kFqGQ = 2, kFqBoth = 3, kFqNR = 4, kFqMD = 5 };  // kFqNR: VCFX_nonref_filter, kFqMD: VCFX_missing_detector
struct RfArgs {
    const RfCrit *crit;
    int ncrit, and_logic;
    const char *pool;
    int pool_len;
};
hipError_t launch_fq_walk(int what, const char *buf, int64_t lo, int64_t hi, int64_t chunk, int strip_cr,
                          int64_t span0, uint64_t cap_w, const RfArgs &rf, const char *q_dev, int qlen, int strict,
                          int qa, int qb, uint64_t *le_b, uint8_t *status_b, void *meta_b, void *tabs_b,
                          uint64_t *wcount, unsigned *overflow, hipStream_t s);
// tabs: per line 16 B, the first 8 tab offsets (u16 from the line start, 0xFFFF = none)
hipError_t launch_fq_compact(int what, int64_t n_walkers, uint64_t cap_w, const uint64_t *offs, const uint64_t *le_b,
                             const uint8_t *status_b, const void *meta_b, const void *tabs_b, uint64_t *line_end,
                             uint8_t *status, void *meta, void *tabs, uint64_t *n_lines, hipStream_t s);
// k_fq_done: counters [0..7], *n_lines and the 8-byte overflow slot into out[0..9] (mapped
// host memory), the counters and the slot zeroed after being read
hipError_t launch_fq_done(unsigned long long *cnt, const uint64_t *n_lines, uint64_t *ovf, uint64_t *out,
                          hipStream_t s);
hipError_t launch_fq_finish(int what, const char *buf, int64_t data_start, const uint64_t *line_end,
                            const uint64_t *n_lines_dev, uint64_t n_lines_host, const RfArgs &rf, uint8_t *status,
                            void *meta, const void *tabs, unsigned long long *rf_cnt, unsigned long long *gq_cnt,
                            hipStream_t s);

}  // namespace vcfxg
