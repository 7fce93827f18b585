// vcfxg_rf.h -- compiled record_filter criterion (device layout) and launcher.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vcfxg_num.h"

namespace vcfxg {

enum { RF_POS = 0, RF_QUAL = 1, RF_FILTER = 2, RF_INFO = 3 };

struct RfCrit {
    int target, op, numeric;
    NumThreshold T;
    uint32_t key_off, key_len;  // INFO key in the pool
    uint32_t str_off, str_len;  // string value in the pool
};

hipError_t launch_vc_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int strip_cr, uint8_t *status, unsigned long long *counters,
                             hipStream_t s);
hipError_t launch_rf_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, const RfCrit *crit, int ncrit, int and_logic, const char *pool,
                             uint8_t *status, unsigned long long *counters, hipStream_t s);

}  // namespace vcfxg
