// vcfxg_api.hip -- the C ABI (include/vcfx_gpu.h): device context, device-resident input,
// and the host-side sequencing of the record kernels on one HIP stream.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstring>
#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "vcfx_gpu.h"
#include "vcfxg_decimal.h"
#include "vcfxg_kernels.h"
#include "vcfxg_rf.h"

namespace {

constexpr size_t kPad = 256;  // zeroed bytes after the input: 16 B loads may run past n

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

}  // namespace

struct vcfxg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // input
    DevBuf input;
    size_t n = 0;
    int last_byte = -1;  // input[n-1] (host copy), -1 if empty
    bool loaded = false;
    // index
    DevBuf idx_counts, idx_offs, line_end, d_nlines, scan_tmp;
    size_t data_start = 0;
    uint64_t n_lines = 0;
    bool indexed = false;
    // per-line results
    DevBuf alt, tot, rowpre, status, rowlen, rowoff, text, counters, query, crit, pool;
    std::string query_host, crit_host, pool_host;  // host sources of in-flight async copies
    uint64_t text_bytes = 0;
    // profiling
    bool profiling = false;
    std::map<std::string, std::pair<hipEvent_t, hipEvent_t>> ev;
    std::map<std::string, float> ms;           // last launch
    std::map<std::string, std::pair<double, uint64_t>> acc;  // sum ms, launches
    std::vector<std::string> pending;
};

namespace {

int fail(vcfxg_ctx *c, hipError_t e, const char *what) {
    if (c) {
        c->err = std::string(what) + ": " + hipGetErrorString(e);
    }
    return e == hipErrorOutOfMemory ? VCFXG_E_NOMEM : VCFXG_E_HIP;
}

#define HIPCHK(ctx, x)                                   \
    do {                                                 \
        hipError_t e_ = (x);                             \
        if (e_ != hipSuccess) return fail(ctx, e_, #x);  \
    } while (0)

int ensure(vcfxg_ctx *c, DevBuf &b, size_t bytes) {
    if (bytes <= b.cap) return VCFXG_OK;
    size_t nc = bytes < 4096 ? 4096 : bytes + bytes / 8;
    if (b.p) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
    }
    HIPCHK(c, hipMalloc(&b.p, nc));
    b.cap = nc;
    return VCFXG_OK;
}

template <typename T>
T *P(DevBuf &b) {
    return reinterpret_cast<T *>(b.p);
}

void prof_begin(vcfxg_ctx *c, const char *name) {
    if (!c->profiling) return;
    auto &e = c->ev[name];
    if (!e.first) {
        (void)hipEventCreate(&e.first);
        (void)hipEventCreate(&e.second);
    }
    (void)hipEventRecord(e.first, c->stream);
}
void prof_end(vcfxg_ctx *c, const char *name) {
    if (!c->profiling) return;
    (void)hipEventRecord(c->ev[name].second, c->stream);
    c->pending.push_back(name);
}
// after a stream sync: harvest elapsed times
void prof_collect(vcfxg_ctx *c) {
    for (auto &nm : c->pending) {
        auto &e = c->ev[nm];
        float t = 0.f;
        if (hipEventElapsedTime(&t, e.first, e.second) == hipSuccess) {
            c->ms[nm] = t;
            auto &a = c->acc[nm];
            a.first += t;
            a.second += 1;
        }
    }
    c->pending.clear();
}

template <typename InT>
int exclusive_scan(vcfxg_ctx *c, const InT *in, uint64_t *out, size_t n) {
    size_t tmp = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)n, c->stream));
    int r = ensure(c, c->scan_tmp, tmp);
    if (r) return r;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tmp, in, out, (int)n, c->stream));
    return VCFXG_OK;
}

}  // namespace

extern "C" {

const char *vcfxg_version(void) { return "vcfx_amd 0.1 (gfx950)"; }

int vcfxg_device_count(int *n) {
    int k = 0;
    if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
    if (n) *n = k;
    return VCFXG_OK;
}

int vcfxg_open(int device, vcfxg_ctx **out) {
    if (!out) return VCFXG_E_ARG;
    *out = nullptr;
    int k = 0;
    if (hipGetDeviceCount(&k) != hipSuccess || k <= 0 || device < 0 || device >= k) return VCFXG_E_NODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return VCFXG_E_NODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return VCFXG_E_NODEV;
    vcfxg_ctx *c = new vcfxg_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return VCFXG_E_HIP;
    }
    int r = ensure(c, c->d_nlines, 64);
    if (!r) r = ensure(c, c->counters, 64);
    if (r) {
        vcfxg_close(c);
        return r;
    }
    *out = c;
    return VCFXG_OK;
}

void vcfxg_close(vcfxg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (DevBuf *b : {&c->input, &c->idx_counts, &c->idx_offs, &c->line_end, &c->d_nlines, &c->scan_tmp, &c->alt,
                      &c->tot, &c->rowpre, &c->status, &c->rowlen, &c->rowoff, &c->text, &c->counters, &c->query, &c->crit, &c->pool})
        if (b->p) (void)hipFree(b->p);
    for (auto &kv : c->ev) {
        (void)hipEventDestroy(kv.second.first);
        (void)hipEventDestroy(kv.second.second);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *vcfxg_last_error(const vcfxg_ctx *c) { return c ? c->err.c_str() : "no context"; }
void *vcfxg_stream(vcfxg_ctx *c) { return c ? (void *)c->stream : nullptr; }

int vcfxg_set_profiling(vcfxg_ctx *c, int enable) {
    if (!c) return VCFXG_E_ARG;
    c->profiling = enable != 0;
    return VCFXG_OK;
}

int vcfxg_kernel_ms(vcfxg_ctx *c, const char *kernel, float *ms) {
    if (!c || !kernel || !ms) return VCFXG_E_ARG;
    auto it = c->ms.find(kernel);
    if (it == c->ms.end()) return VCFXG_E_STATE;
    *ms = it->second;
    return VCFXG_OK;
}

int vcfxg_kernel_stats(vcfxg_ctx *c, const char *kernel, double *total_ms, uint64_t *launches) {
    if (!c || !kernel) return VCFXG_E_ARG;
    auto it = c->acc.find(kernel);
    if (total_ms) *total_ms = it == c->acc.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == c->acc.end() ? 0 : it->second.second;
    return VCFXG_OK;
}

int vcfxg_reset_kernel_stats(vcfxg_ctx *c) {
    if (!c) return VCFXG_E_ARG;
    c->acc.clear();
    return VCFXG_OK;
}

int vcfxg_load_host(vcfxg_ctx *c, const char *host, size_t n) {
    if (!c || (!host && n)) return VCFXG_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int r = ensure(c, c->input, n + kPad);
    if (r) return r;
    if (n) HIPCHK(c, hipMemcpyAsync(c->input.p, host, n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(static_cast<char *>(c->input.p) + n, 0, kPad, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->n = n;
    c->last_byte = n ? (unsigned char)host[n - 1] : -1;
    c->loaded = true;
    c->indexed = false;
    return VCFXG_OK;
}

const void *vcfxg_input_device_ptr(vcfxg_ctx *c) { return c && c->loaded ? c->input.p : nullptr; }

int vcfxg_index(vcfxg_ctx *c, size_t data_start, uint64_t *n_lines) {
    if (!c) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n;
    const int64_t nc = vcfxg::idx_nchunks(lo, hi);
    int r = ensure(c, c->idx_counts, sizeof(uint32_t) * (size_t)(nc + 1));
    if (!r) r = ensure(c, c->idx_offs, sizeof(uint64_t) * (size_t)(nc + 1));
    if (r) return r;
    const char *buf = P<char>(c->input);
    prof_begin(c, "line_count");
    HIPCHK(c, vcfxg::launch_nl_count(buf, lo, hi, P<uint32_t>(c->idx_counts), c->stream));
    prof_end(c, "line_count");
    HIPCHK(c, hipMemsetAsync(P<uint32_t>(c->idx_counts) + nc, 0, sizeof(uint32_t), c->stream));
    r = exclusive_scan(c, P<uint32_t>(c->idx_counts), P<uint64_t>(c->idx_offs), (size_t)nc + 1);
    if (r) return r;
    uint64_t total = 0;
    HIPCHK(c, hipMemcpyAsync(&total, P<uint64_t>(c->idx_offs) + nc, sizeof total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const bool tail = hi > lo && c->last_byte != '\n';
    const uint64_t nl = total + (tail ? 1 : 0);
    r = ensure(c, c->line_end, sizeof(uint64_t) * (size_t)(nl + 1));
    if (r) return r;
    prof_begin(c, "line_emit");
    HIPCHK(c, vcfxg::launch_nl_emit(buf, lo, hi, P<uint64_t>(c->idx_offs), P<uint64_t>(c->line_end), total,
                                    c->stream));
    prof_end(c, "line_emit");
    static thread_local uint64_t tail_end, nl_host;
    tail_end = (uint64_t)hi;
    nl_host = nl;
    if (tail)
        HIPCHK(c, hipMemcpyAsync(P<uint64_t>(c->line_end) + total, &tail_end, sizeof(uint64_t), hipMemcpyHostToDevice,
                                 c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_nlines.p, &nl_host, sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->data_start = data_start;
    c->n_lines = nl;
    c->indexed = true;
    if (n_lines) *n_lines = nl;
    return VCFXG_OK;
}

int vcfxg_line_ends(vcfxg_ctx *c, uint64_t first, uint64_t count, uint64_t *out) {
    if (!c || (!out && count)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    if (first + count > c->n_lines) return VCFXG_E_ARG;
    if (!count) return VCFXG_OK;
    HIPCHK(c, hipMemcpyAsync(out, P<uint64_t>(c->line_end) + first, count * sizeof(uint64_t), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

int vcfxg_allele_freq(vcfxg_ctx *c, int mode, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t L = c->n_lines;
    int r = ensure(c, c->alt, 4 * (L + 1));
    if (!r) r = ensure(c, c->tot, 4 * (L + 1));
    if (!r) r = ensure(c, c->rowpre, 4 * (L + 1));
    if (!r) r = ensure(c, c->status, L + 1);
    if (!r) r = ensure(c, c->rowlen, 8 * (L + 1));
    if (!r) r = ensure(c, c->rowoff, 8 * (L + 1));
    if (r) return r;
    const char *buf = P<char>(c->input);
    const uint64_t *nl_dev = P<uint64_t>(c->d_nlines);
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    prof_begin(c, "af_records");
    HIPCHK(c, vcfxg::launch_af_records(buf, (int64_t)c->data_start, P<uint64_t>(c->line_end), nl_dev, L, mode,
                                       P<int32_t>(c->alt), P<int32_t>(c->tot), P<uint32_t>(c->rowpre),
                                       P<uint8_t>(c->status), P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "af_records");
    prof_begin(c, "af_rows");
    HIPCHK(c, vcfxg::launch_af_rowlen(P<uint32_t>(c->rowpre), P<uint8_t>(c->status), nl_dev, L, P<uint64_t>(c->rowlen),
                                      c->stream));
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->rowlen) + L, 0, 8, c->stream));
    r = exclusive_scan(c, P<uint64_t>(c->rowlen), P<uint64_t>(c->rowoff), (size_t)L + 1);
    if (r) return r;
    prof_end(c, "af_rows");
    static thread_local uint64_t host_tail[5];
    HIPCHK(c, hipMemcpyAsync(&host_tail[0], P<uint64_t>(c->rowoff) + L, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&host_tail[1], c->counters.p, 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t text = host_tail[0];
    r = ensure(c, c->text, text + 1);
    if (r) return r;
    prof_begin(c, "af_format");
    HIPCHK(c, vcfxg::launch_af_format(buf, (int64_t)c->data_start, P<uint64_t>(c->line_end), nl_dev, L, mode,
                                      P<int32_t>(c->alt), P<int32_t>(c->tot), P<uint32_t>(c->rowpre),
                                      P<uint8_t>(c->status), P<uint64_t>(c->rowoff), P<char>(c->text), c->stream));
    prof_end(c, "af_format");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->text_bytes = text;
    if (out) {
        out->n_lines = L;
        out->rows = host_tail[1];
        out->data_lines = host_tail[2];
        out->warn_lines = host_tail[3];
        out->general_records = host_tail[4];
        out->text_bytes = text;
    }
    return VCFXG_OK;
}

// parseDiploidAlleles (VCFX_genotype_query.cpp:246-272) incl. its partial assignment on
// failure, then the swap of main :641-645
static void gq_parse_query(const char *q, size_t n, int &qa, int &qb) {
    qa = qb = -1;
    size_t sep = (size_t)-1;
    for (size_t i = 0; i < n; i++)
        if (q[i] == '|' || q[i] == '/') { sep = i; break; }
    if (sep == (size_t)-1 || sep == 0 || sep == n - 1) return;
    if (sep == 1 && q[0] == '.') return;
    unsigned v = 0;
    qa = 0;
    bool ok = true;
    for (size_t i = 0; i < sep && ok; i++) {
        if (q[i] < '0' || q[i] > '9') ok = false;
        else qa = (int)(v = v * 10u + (unsigned)(q[i] - '0'));
    }
    if (ok) {
        if (!(n - sep - 1 == 1 && q[sep + 1] == '.')) {
            v = 0;
            qb = 0;
            for (size_t i = sep + 1; i < n; i++) {
                if (q[i] < '0' || q[i] > '9') break;
                qb = (int)(v = v * 10u + (unsigned)(q[i] - '0'));
            }
        }
    }
    if (qa > qb) std::swap(qa, qb);
}

int vcfxg_genotype_query(vcfxg_ctx *c, const char *query, size_t qlen, int strict, int strip_cr, vcfxg_summary *out) {
    if (!c || (!query && qlen)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t L = c->n_lines;
    int r = ensure(c, c->status, L + 1);
    if (!r) r = ensure(c, c->query, qlen + 1);
    if (r) return r;
    int qa = -1, qb = -1;
    if (!strict) gq_parse_query(query, qlen, qa, qb);
    c->query_host.assign(query, qlen);
    if (qlen)
        HIPCHK(c, hipMemcpyAsync(c->query.p, c->query_host.data(), qlen, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    prof_begin(c, "gq_records");
    HIPCHK(c, vcfxg::launch_gq_records(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                       P<uint64_t>(c->d_nlines), L, strip_cr, P<char>(c->query), (int)qlen, strict,
                                       qa, qb, P<uint8_t>(c->status), P<unsigned long long>(c->counters), c->stream,
                                       nullptr));
    prof_end(c, "gq_records");
    static thread_local uint64_t host_cnt[4];
    HIPCHK(c, hipMemcpyAsync(host_cnt, c->counters.p, 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->text_bytes = 0;
    if (out) {
        out->n_lines = L;
        out->rows = host_cnt[0];
        out->data_lines = host_cnt[1];
        out->warn_lines = host_cnt[2];
        out->general_records = host_cnt[3];
        out->text_bytes = 0;
    }
    return VCFXG_OK;
}

static vcfxg::DecRef put_dec(const vcfxg::DecHost &d, std::string &pool) {
    vcfxg::DecRef r;
    r.sign = d.sign;
    r.exp = d.exp;
    r.off = (uint32_t)pool.size();
    r.n = (uint32_t)d.digits.size();
    r.inf = d.inf;
    pool += d.digits;
    return r;
}

static int compile_criteria(vcfxg_ctx *c, const vcfxg_criterion *crit, int n) {
    std::vector<vcfxg::RfCrit> dev((size_t)n);
    std::string pool;
    for (int i = 0; i < n; i++) {
        const vcfxg_criterion &h = crit[i];
        vcfxg::RfCrit &d = dev[(size_t)i];
        std::memset(&d, 0, sizeof d);
        d.target = h.target;
        d.op = h.op;
        d.numeric = h.numeric;
        d.key_off = (uint32_t)pool.size();
        d.key_len = (uint32_t)h.key_len;
        pool.append(h.key ? h.key : "", h.key_len);
        d.str_off = (uint32_t)pool.size();
        d.str_len = (uint32_t)h.str_len;
        pool.append(h.str ? h.str : "", h.str_len);
        vcfxg::ThresholdHost th;
        vcfxg::threshold_bounds(h.numeric ? h.value : 0.0, th);
        d.T.t = h.numeric ? h.value : 0.0;
        d.T.kind = th.kind;
        d.T.lo = put_dec(th.lo, pool);
        d.T.hi = put_dec(th.hi, pool);
        d.T.lo_to_t = th.lo_to_t;
        d.T.hi_to_t = th.hi_to_t;
    }
    int r = ensure(c, c->crit, sizeof(vcfxg::RfCrit) * (size_t)(n + 1));
    if (!r) r = ensure(c, c->pool, pool.size() + 16);
    if (r) return r;
    c->crit_host.assign((const char *)dev.data(), sizeof(vcfxg::RfCrit) * (size_t)n);
    c->pool_host = pool;
    if (n)
        HIPCHK(c, hipMemcpyAsync(c->crit.p, c->crit_host.data(), c->crit_host.size(), hipMemcpyHostToDevice, c->stream));
    if (!pool.empty())
        HIPCHK(c, hipMemcpyAsync(c->pool.p, c->pool_host.data(), pool.size(), hipMemcpyHostToDevice, c->stream));
    return VCFXG_OK;
}

static int run_rf(vcfxg_ctx *c, const vcfxg_criterion *crit, int n, int and_logic) {
    int r = ensure(c, c->status, c->n_lines + 1);
    if (!r) r = compile_criteria(c, crit, n);
    if (r) return r;
    prof_begin(c, "rf_records");
    HIPCHK(c, vcfxg::launch_rf_records(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                       P<uint64_t>(c->d_nlines), c->n_lines, P<vcfxg::RfCrit>(c->crit), n, and_logic,
                                       P<char>(c->pool), P<uint8_t>(c->status), P<unsigned long long>(c->counters),
                                       c->stream));
    prof_end(c, "rf_records");
    return VCFXG_OK;
}

int vcfxg_record_filter(vcfxg_ctx *c, const vcfxg_criterion *crit, int n, int and_logic, vcfxg_summary *out) {
    if (!c || n < 0 || (n && !crit)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    int r = run_rf(c, crit, n, and_logic);
    if (r) return r;
    static thread_local uint64_t host_cnt[2];
    HIPCHK(c, hipMemcpyAsync(host_cnt, c->counters.p, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = c->n_lines;
        out->rows = host_cnt[0];
        out->data_lines = host_cnt[1];
    }
    return VCFXG_OK;
}

int vcfxg_filter_query(vcfxg_ctx *c, const vcfxg_criterion *crit, int n, int and_logic, const char *query, size_t qlen,
                       int strict, vcfxg_summary *out) {
    if (!c || n < 0 || (n && !crit) || (!query && qlen)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    int r = run_rf(c, crit, n, and_logic);
    if (!r) r = ensure(c, c->query, qlen + 1);
    if (r) return r;
    int qa = -1, qb = -1;
    if (!strict) gq_parse_query(query, qlen, qa, qb);
    c->query_host.assign(query, qlen);
    if (qlen)
        HIPCHK(c, hipMemcpyAsync(c->query.p, c->query_host.data(), qlen, hipMemcpyHostToDevice, c->stream));
    prof_begin(c, "gq_records");
    HIPCHK(c, vcfxg::launch_gq_records(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                       P<uint64_t>(c->d_nlines), c->n_lines, 1, P<char>(c->query), (int)qlen, strict,
                                       qa, qb, P<uint8_t>(c->status), P<unsigned long long>(c->counters) + 4,
                                       c->stream, P<uint8_t>(c->status)));
    prof_end(c, "gq_records");
    static thread_local uint64_t host_cnt[8];
    HIPCHK(c, hipMemcpyAsync(host_cnt, c->counters.p, 64, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = c->n_lines;
        out->rows = host_cnt[4];        // kept by both stages
        out->data_lines = host_cnt[0];  // kept by record_filter
        out->warn_lines = host_cnt[6];
        out->general_records = host_cnt[7];
    }
    return VCFXG_OK;
}

int vcfxg_variant_count(vcfxg_ctx *c, int strip_cr, vcfxg_summary *out) {
    if (!c) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    int r = ensure(c, c->status, c->n_lines + 1);
    if (r) return r;
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    prof_begin(c, "vc_records");
    HIPCHK(c, vcfxg::launch_vc_records(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                       P<uint64_t>(c->d_nlines), c->n_lines, strip_cr, P<uint8_t>(c->status),
                                       P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "vc_records");
    static thread_local uint64_t host_cnt[2];
    HIPCHK(c, hipMemcpyAsync(host_cnt, c->counters.p, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = c->n_lines;
        out->rows = host_cnt[0];
        out->warn_lines = host_cnt[1];
    }
    return VCFXG_OK;
}

int vcfxg_fetch_text(vcfxg_ctx *c, char *host, size_t cap) {
    if (!c || (!host && c->text_bytes)) return VCFXG_E_ARG;
    if (cap < c->text_bytes) return VCFXG_E_CAP;
    if (!c->text_bytes) return VCFXG_OK;
    HIPCHK(c, hipMemcpyAsync(host, c->text.p, c->text_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

int vcfxg_fetch_lines(vcfxg_ctx *c, uint64_t first, uint64_t count, int32_t *alt, int32_t *total, uint8_t *status) {
    if (!c) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    if (first + count > c->n_lines) return VCFXG_E_ARG;
    if (!count) return VCFXG_OK;
    if (alt) HIPCHK(c, hipMemcpyAsync(alt, P<int32_t>(c->alt) + first, 4 * count, hipMemcpyDeviceToHost, c->stream));
    if (total) HIPCHK(c, hipMemcpyAsync(total, P<int32_t>(c->tot) + first, 4 * count, hipMemcpyDeviceToHost, c->stream));
    if (status) HIPCHK(c, hipMemcpyAsync(status, P<uint8_t>(c->status) + first, count, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

}  // extern "C"
