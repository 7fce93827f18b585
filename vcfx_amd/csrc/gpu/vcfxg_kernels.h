// vcfxg_kernels.h -- host-visible launchers of the record kernels (vcfxg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vcfxg {

int64_t idx_nchunks(int64_t lo, int64_t hi);
hipError_t launch_nl_count(const char *buf, int64_t lo, int64_t hi, uint32_t *counts, hipStream_t s);
hipError_t launch_nl_emit(const char *buf, int64_t lo, int64_t hi, const uint64_t *offs, uint64_t *line_end,
                          uint64_t cap, hipStream_t s);
hipError_t launch_af_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int mode, int32_t *alt, int32_t *tot, uint32_t *rowpre,
                             uint8_t *status, unsigned long long *counters, hipStream_t s);
// fused index + AF (one sweep): chunks for data_start / n (0 = use the two-pass path)
uint64_t af_fused_chunks(int64_t ds, int64_t n);
hipError_t launch_af_fused(const char *buf, int64_t ds, int64_t n, int mode, unsigned long long *state, uint64_t *line_end, uint64_t *n_lines_dev, uint64_t cap,
                           int32_t *alt, int32_t *tot, uint32_t *rowpre, uint8_t *status,
                           unsigned long long *counters, hipStream_t s, int dbg = 0);
hipError_t launch_gq_records(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int strip_cr, const char *q_dev,
                             int qlen, int strict, int qa, int qb, uint8_t *status, unsigned long long *counters,
                             hipStream_t s, const uint8_t *gate);
hipError_t launch_af_rowlen(const uint32_t *rowpre, const uint8_t *status, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, uint64_t *len, hipStream_t s);
hipError_t launch_af_format(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, int mode, const int32_t *alt, const int32_t *tot,
                            const uint32_t *rowpre, const uint8_t *status, const uint64_t *off, char *out,
                            hipStream_t s);

}  // namespace vcfxg
