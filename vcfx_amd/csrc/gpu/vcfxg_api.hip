// vcfxg_api.hip -- the C ABI (include/vcfx_gpu.h): device context, device-resident input,
// and the host-side sequencing of the record kernels on one HIP stream.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>  // declarations only: librccl is dlopen'd by the rank cliques

#include <dlfcn.h>
#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <map>
#include <string>
#include <vector>

#include "vcfx_gpu.h"
#include "vcfxg_decimal.h"
#include "vcfxg_kernels.h"
#include "vcfxg_ld.h"
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
    bool ingesting = false;               // between vcfxg_ingest_begin and the final chunk
    bool hints_pending = false;           // no ingested chunk has held a data line yet
    const char *last_schedule = "";       // the schedule of the last region call (note_schedule)
    std::vector<std::pair<size_t, hipEvent_t>> ingest_ev;  // (input bytes copied once it fires, event)
    std::vector<hipEvent_t> ingest_ev_free;
    // index
    DevBuf idx_counts, idx_offs, idx_pos, line_end, d_nlines, scan_tmp;
    size_t data_start = 0;
    uint64_t n_lines = 0;
    bool indexed = false;
    // per-line results
    DevBuf alt, tot, rowpre, status, rowlen, rowoff, text, counters, query, crit, pool;
    std::string query_host, crit_host, pool_host;  // host sources of in-flight async copies
    // LD
    DevBuf ld_G, ld_lines, ld_vidx, ld_valid, ld_Gc, ld_vars, ld_plen, ld_poff, ld_prefix, ld_cid, ld_blocks, ld_cnt,
        ld_off, ld_pairs, ld_fast, ld_gflag, ld_Gp, ld_rowoff, ld_Gv, ld_Gq, dose_meta;
    // LD walk (vcfxg_ld_prepare_region): walker counts, valid-line counts and their scan, flags +
    // summary; ld_gc_ready: ld_Gc holds the compact int8 rows (the walk gathers them only when
    // some variant misses a call)
    DevBuf ld_wcnt, ld_wval, ld_vbase, ld_small, ld_pend;
    // vcfxg_bgzf_stage: the compressed stream's size and the bytes staged so far (into bgz_in, on
    // copy_stream); vcfxg_bgzf_inflate: members already launched and their output bytes
    size_t bgz_total = 0, bgz_staged = 0;
    uint64_t bgz_handed = 0;  // members of the last BGZF ingest the lane decoder handed over
    uint64_t bgz_launched = 0, bgz_out = 0;
    hipStream_t copy_stream = nullptr;
    hipEvent_t bgz_copy_ev = nullptr;  // the latest staged copy
    // the inflate batches run round robin on their own streams (one stream would serialise each
    // batch's tail), joined before the device input completes; two: batches are 32,768 members
    // (hostio.cpp), and a fresh context pays ~7 ms to create a stream
    static constexpr int kBgzStreams = 2;
    hipStream_t bgz_stream[kBgzStreams] = {};
    hipEvent_t bgz_ev[kBgzStreams] = {};
    int bgz_next = 0;
    bool ld_gc_ready = false;
    bool ld_vq = false;  // ld_Gv / ld_Gq (valid-mask and squared-dosage FP4 planes) are current
    int n_cu = 0;
    DevBuf async_small;         // asynchronous AF path: line range {0, n}, failure flags, summary
    DevBuf ld_temp, ld_quarters, ld_stage_ctr;  // LD: pairs staged by the count pass
    uint64_t ld_temp_cap = 0;
    // test hook: a fixed (small) staging capacity exercises the overflow -> emit-pass path
    uint64_t ld_stage_cap_fixed = getenv("VCFXG_LD_STAGE_CAP") ? strtoull(getenv("VCFXG_LD_STAGE_CAP"), nullptr, 10) : 0;
    DevBuf af_meta;             // AF head pass output (k_af_meta)
    // walk AF path (vcfxg_af_walk.hip): per-walker regions, counts, scan, flags
    DevBuf wk_le, wk_alt, wk_tot, wk_rowpre, wk_status, wk_meta, wk_count, wk_offs, wk_gt, wk_small;
    DevBuf wk_tabs, rf_tabs;    // filter / query walk: per-line tab offsets (per walker, dense)
    // AF walk region tail: per walker row bytes, text offsets, first line start; leftover list
    DevBuf wk_text, wk_toff, wk_start, wk_cx, wk_bs, scratch_small, byte_cnt;
    // AF walk: flags / counters that k_walker_scan zeroes after reading them (af_small_dirty: a
    // call did not get that far, so the next one clears them first), and the call summary the
    // same kernel writes straight into mapped host memory (no copy before the synchronisation)
    DevBuf af_small;
    bool af_small_dirty = true;
    DevBuf wk_stage, wk_dirty;  // AF walk: each walker's rows as text (kStageCap bytes), its clean flag
    uint64_t *sum_host = nullptr, *sum_dev = nullptr;
    uint64_t cx_hint = ~0ull;  // leftover lines of the previous AF walk (sizes k_af_cx's grid)
    // filter / query walk: overflow slot + 8 counters, zeroed by k_fq_done after each call
    // (fq_small_dirty as af_small_dirty); its summary goes to sum_host[8..17]
    DevBuf fq_small;
    bool fq_small_dirty = true;
    uint64_t fq_lines_hint = 0;  // lines of the previous filter / query walk (sizes k_fq_finish's grid)
    // the bytes last uploaded to query / crit / pool and the buffer they went to: an unchanged
    // query or criteria list is not copied again (any other writer resets the pointer)
    std::string query_dev, crit_dev, pool_dev;
    void *query_dev_p = nullptr, *crit_dev_p = nullptr, *pool_dev_p = nullptr;
    // the last AF walk left its per-line results in walker regions only (ensure_dense)
    bool dense_pending = false;
    int64_t dense_nw = 0;
    uint64_t dense_cap_w = 0;
    // VCFX_hwe_tester: hom-alt counts (dense, per walker), the host-recheck list and its length
    DevBuf hwe_aux, wk_aux, hwe_rc;
    // VCFX_allele_counter: slots' sample indices, name offsets and bytes, per-wave sample tables
    DevBuf ac_eff, ac_noff, ac_names, ac_scratch, ac_etab, ac_nib;
    std::vector<uint32_t> ac_eff_host;
    std::vector<uint64_t> ac_noff_host;
    std::string ac_names_host;
    std::vector<uint8_t> ac_etab_host;
    // VCFX_haplotype_phaser: genotype rows (by line), per-line info, variant -> line, pair flags
    DevBuf ph_G, ph_isvar, ph_info, ph_vnum, ph_vline, ph_flags, ph_r2;
    uint64_t ph_nvar = 0;
    uint64_t hwe_rc_n = 0;
    // ulps either side of the device p-value that must print the same digits (test hook: a
    // huge value sends every exp()-derived row to the host)
    int64_t hwe_ulps = getenv("VCFXG_HWE_ULPS") ? atoll(getenv("VCFXG_HWE_ULPS")) : 16;
    // (an override is clamped to [4 KiB, 8 MiB]: the AF walk packs a walker's GT-line count in
    // 16 bits, and its line capacity 2 * chunk / hint_line + 16 stays below 2^15 for the
    // >= 512 B records the walk takes)
    int64_t walk_chunk = getenv("VCFXG_WALK_CHUNK")
                             ? std::min<int64_t>(std::max<int64_t>(atol(getenv("VCFXG_WALK_CHUNK")), 4096), 8 << 20)
                             : 128 * 1024;
    bool walk_overflowed = false;  // the last walk run overflowed: two-sweep schedule
    bool dose_head_failed = false;  // a dosage head walk's rows failed the check (this input)
    bool ph_head_failed = false;    // a phaser head-walk index failed the parse's check (this input)
    // host hints taken at load time from the first data line: its '\n' distance from the
    // sample start (the walk's first prediction) and the mean length of the first lines
    int64_t hint_span = 0, hint_line = 0;
    // the first data line's FORMAT is exactly "GT" (fixed-stride records: the walk's predicted
    // ends pay; "GT:AD:DP"-like records are scanned faster by the index sweep)
    bool hint_gt_only = false;
    // ... or starts with "GT:" (GT:AD:DP-like records: the GT-first walk, gt_first finding each
    // record's end in its one sweep)
    bool hint_gt_first = false;
    uint64_t af_line_cap = 0;   // two-sweep AF: line capacity the last run needed
    // region AF schedule: 0 = default (the walk schedule 7 when the first records average
    // >= 512 B, else 3 with one host synchronisation: single-sweep index + head pass +
    // fixed-stride sweep), 1 = one-sweep look-back kernel (k_af_fused),
    // 2 = chunk count + chunk sweep (k_af_chunks), 4 = one sweep with byte-class segment
    // counts (k_af_scan); the single-sweep alternatives are correct and tested but slower
    // today, kept selectable for measurement; 7 = walk (k_af_walk: predicted
    // record ends validated by the sweep, one HBM pass); 8 = the two-sweep schedule always
    int af_path = getenv("VCFXG_AF_FUSED") ? atoi(getenv("VCFXG_AF_FUSED")) : 0;
    // record_filter / genotype_query region schedule: 0 = the walk (vcfxg_fq_walk.hip) when
    // the first records average >= 512 B, 1 = the walk always, -1 = index + per-tool kernels
    int fq_path = getenv("VCFXG_FQ_WALK") ? atoi(getenv("VCFXG_FQ_WALK")) : 0;
    std::vector<uint8_t> ld_gflag_host;  // per 128-variant group: all complete
    uint64_t ld_m = 0, ld_prefix_bytes = 0, ld_np = 0;
    int ld_kpad = 64, ld_ns = 0, ld_kp4 = 64;
    bool ld_chrom_ids = false;
    std::vector<uint32_t> ld_cid_host, ld_blocks_host;
    // the last streaming call's block lists: key (j0, j1, window, M, masked kernel), group
    // flags, list sizes (fast, masked, int8), the ld_blocks buffer they were copied to
    uint64_t ld_plan_key[5] = {0, 0, 0, 0, 0};
    std::vector<uint8_t> ld_plan_gf;
    uint32_t ld_plan_n[4] = {0, 0, 0, 0};
    // the sparse-missing LD kernel's data (ld_sp: some 256-group qualifies): CSR of each
    // variant's missing samples and the sample-major contribution plane
    bool ld_sp = false;
    uint64_t ld_mp = 0;
    DevBuf ld_moff, ld_midx, ld_mvar, ld_gt16, ld_sprec, ld_midx16;
    // device BGZF inflate (vcfxg_ingest_bgzf): compressed bytes, member table, output offsets,
    // per-member status, first bad member
    DevBuf bgz_in, bgz_mem, bgz_off, bgz_stat, bgz_small, bgz_perm;
    // the lane decoder's token buffers (and hand-over lists): one per inflate stream and one for
    // `stream`; its side stream (the hand-overs') and events
    DevBuf bgz_tok[kBgzStreams + 1];
    vcfxg::InflateSide bgz_side;
    void *ld_plan_dev = nullptr;
    uint64_t text_bytes = 0;
    uint64_t text_hint = 0;  // AF walk: text bytes of the previous call (the next call's capacity)
    // profiling: an event pair per launch from a pool, harvested only when the figures are
    // read (or the pending list is long): no event queries between the calls of a timed loop
    bool profiling = false;
    std::string prof_only;  // non-empty: only this kernel is timed
    struct ProfRec {
        const char *name;
        hipEvent_t a, b;
    };
    std::vector<hipEvent_t> ev_free;
    std::vector<ProfRec> ev_open, pending;
    std::map<std::string, float> ms;           // last launch
    std::map<std::string, std::pair<double, uint64_t>> acc;  // sum ms, launches
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

static hipEvent_t prof_event(vcfxg_ctx *c) {
    hipEvent_t e = nullptr;
    if (!c->ev_free.empty()) {
        e = c->ev_free.back();
        c->ev_free.pop_back();
    } else {
        (void)hipEventCreate(&e);
    }
    return e;
}
static bool prof_on(vcfxg_ctx *c, const char *name) {
    return c->profiling && (c->prof_only.empty() || c->prof_only == name);
}
void prof_begin(vcfxg_ctx *c, const char *name) {
    if (!prof_on(c, name)) return;
    hipEvent_t e = prof_event(c);
    (void)hipEventRecord(e, c->stream);
    c->ev_open.push_back({name, e, nullptr});
}
void prof_end(vcfxg_ctx *c, const char *name) {
    if (!prof_on(c, name)) return;
    for (size_t k = c->ev_open.size(); k-- > 0;) {
        if (strcmp(c->ev_open[k].name, name)) continue;
        vcfxg_ctx::ProfRec r = c->ev_open[k];
        c->ev_open.erase(c->ev_open.begin() + k);
        r.b = prof_event(c);
        (void)hipEventRecord(r.b, c->stream);
        c->pending.push_back(r);
        return;
    }
}
// elapsed times of the recorded launches (synchronises with the stream first)
static void prof_harvest(vcfxg_ctx *c) {
    if (c->pending.empty()) return;
    (void)hipStreamSynchronize(c->stream);
    for (auto &r : c->pending) {
        float t = 0.f;
        if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
            c->ms[r.name] = t;
            auto &a = c->acc[r.name];
            a.first += t;
            a.second += 1;
        }
        c->ev_free.push_back(r.a);
        c->ev_free.push_back(r.b);
    }
    c->pending.clear();
}
// after a call: harvest only when many launches are pending (bounded event pool)
void prof_collect(vcfxg_ctx *c) {
    if (c->pending.size() >= 4096) prof_harvest(c);
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

static int ensure_dense(vcfxg_ctx *c);
// per-line calls on the indexed context read the dense arrays
#define DENSE(c)                       \
    do {                               \
        int rd_ = ensure_dense(c);     \
        if (rd_) return rd_;           \
    } while (0)

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
    c->n_cu = prop.multiProcessorCount;
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
    for (DevBuf *b : {&c->input, &c->idx_counts, &c->idx_offs, &c->idx_pos, &c->line_end, &c->d_nlines, &c->scan_tmp, &c->alt,
                      &c->tot, &c->rowpre, &c->status, &c->rowlen, &c->rowoff, &c->text, &c->counters, &c->query, &c->crit, &c->pool, &c->ld_G, &c->ld_lines,
                      &c->ld_vidx, &c->ld_valid, &c->ld_Gc, &c->ld_wcnt, &c->ld_wval, &c->ld_vbase, &c->ld_small, &c->ld_pend, &c->ld_vars, &c->ld_plen, &c->ld_poff, &c->ld_prefix,
                      &c->ld_cid, &c->ld_blocks, &c->ld_cnt, &c->ld_off, &c->ld_pairs, &c->ld_fast, &c->ld_gflag, &c->ld_Gp, &c->ld_Gv, &c->ld_Gq, &c->dose_meta, &c->af_meta, &c->ld_temp, &c->ld_quarters, &c->ld_stage_ctr, &c->ld_rowoff, &c->async_small, &c->wk_le, &c->wk_alt, &c->wk_tot, &c->wk_rowpre, &c->wk_status, &c->wk_meta, &c->wk_count, &c->wk_offs, &c->wk_gt, &c->wk_small, &c->wk_tabs, &c->rf_tabs, &c->hwe_aux, &c->wk_aux, &c->hwe_rc, &c->wk_text, &c->wk_toff, &c->wk_start, &c->wk_cx, &c->wk_bs, &c->scratch_small, &c->byte_cnt, &c->ld_moff, &c->ld_midx, &c->ld_mvar, &c->ld_gt16, &c->ld_sprec, &c->ld_midx16, &c->bgz_in, &c->bgz_mem, &c->bgz_off, &c->bgz_stat, &c->bgz_small, &c->bgz_perm})
        if (b->p) (void)hipFree(b->p);
    for (DevBuf &b : c->bgz_tok)
        if (b.p) (void)hipFree(b.p);
    if (c->af_small.p) (void)hipFree(c->af_small.p);
    if (c->wk_stage.p) (void)hipFree(c->wk_stage.p);
    if (c->wk_dirty.p) (void)hipFree(c->wk_dirty.p);
    if (c->fq_small.p) (void)hipFree(c->fq_small.p);
    if (c->sum_host) (void)hipHostFree(c->sum_host);
    for (auto &pe : c->ingest_ev) (void)hipEventDestroy(pe.second);
    for (hipEvent_t e : c->ingest_ev_free) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_free) (void)hipEventDestroy(e);
    for (auto &r : c->pending) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    for (auto &r : c->ev_open) (void)hipEventDestroy(r.a);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    for (int k = 0; k < vcfxg_ctx::kBgzStreams; k++) {
        if (c->bgz_stream[k]) (void)hipStreamDestroy(c->bgz_stream[k]);
        if (c->bgz_ev[k]) (void)hipEventDestroy(c->bgz_ev[k]);
    }
    if (c->bgz_copy_ev) (void)hipEventDestroy(c->bgz_copy_ev);
    if (c->bgz_side.aux) (void)hipStreamDestroy(c->bgz_side.aux);
    for (hipEvent_t e : c->bgz_side.ev)
        if (e) (void)hipEventDestroy(e);
    delete c;
}

const char *vcfxg_last_error(const vcfxg_ctx *c) { return c ? c->err.c_str() : "no context"; }
void *vcfxg_stream(vcfxg_ctx *c) { return c ? (void *)c->stream : nullptr; }

int vcfxg_set_profiling(vcfxg_ctx *c, int enable) {
    if (!c) return VCFXG_E_ARG;
    c->profiling = enable != 0;
    return VCFXG_OK;
}

int vcfxg_set_profiling_only(vcfxg_ctx *c, const char *kernel) {
    if (!c) return VCFXG_E_ARG;
    c->prof_only = kernel ? kernel : "";
    return VCFXG_OK;
}

int vcfxg_kernel_ms(vcfxg_ctx *c, const char *kernel, float *ms) {
    if (!c || !kernel || !ms) return VCFXG_E_ARG;
    prof_harvest(c);
    auto it = c->ms.find(kernel);
    if (it == c->ms.end()) return VCFXG_E_STATE;
    *ms = it->second;
    return VCFXG_OK;
}

int vcfxg_kernel_stats(vcfxg_ctx *c, const char *kernel, double *total_ms, uint64_t *launches) {
    if (!c || !kernel) return VCFXG_E_ARG;
    prof_harvest(c);
    auto it = c->acc.find(kernel);
    if (total_ms) *total_ms = it == c->acc.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == c->acc.end() ? 0 : it->second.second;
    return VCFXG_OK;
}

int vcfxg_reset_kernel_stats(vcfxg_ctx *c) {
    if (!c) return VCFXG_E_ARG;
    prof_harvest(c);
    c->acc.clear();
    return VCFXG_OK;
}

// the walk paths' hints from the host bytes of the input's first chunk holding data lines:
// skip '#' lines, then the first data line's '\n' distance from the byte after its 9th tab and
// the mean length of up to 256 lines.  Called on each ingested chunk until one holds data: a
// chunk of '#' lines only that ends at a line end (a shard view's header [0, H), a pipe's head)
// returns false and the next chunk is looked at.  Chunks are read while the caller still owns
// them (a pipe's staging slot is reused after the call).
static void reset_hints(vcfxg_ctx *c) {
    c->hint_span = 0;
    c->hint_line = 0;
    c->hint_gt_only = false;
    c->hint_gt_first = false;
    c->walk_overflowed = false;
    c->dose_head_failed = false;
    c->ph_head_failed = false;
    if (!getenv("VCFXG_WALK_CHUNK")) c->walk_chunk = 128 * 1024;
}

// the schedule a region call took (vcfxg_last_schedule; VCFXG_SCHEDULE_LOG=path appends one
// line per call: tests check which path sharded ranks and fresh contexts run)
// VCFX_TIMING=1: "[vcfxg-timing] <what> <ms>" on stderr at the steps of a fresh context's first
// BGZF stage (ms since the library loaded; the host's own phases are hostio.cpp phase())
static void lib_phase(const char *what) {
    static const auto t0 = std::chrono::steady_clock::now();
    static const bool on = getenv("VCFX_TIMING") && atoi(getenv("VCFX_TIMING")) > 0;
    if (!on) return;
    fprintf(stderr, "[vcfxg-timing] %s %.2f ms\n", what,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

static void note_schedule(vcfxg_ctx *c, const char *what) {
    c->last_schedule = what;
    const char *log = getenv("VCFXG_SCHEDULE_LOG");  // (read per call: tests set it in-process)
    if (!log) return;
    const int fd = ::open(log, O_WRONLY | O_APPEND | O_CREAT | O_CLOEXEC, 0644);
    if (fd < 0) return;
    const std::string l = std::string(what) + "\n";
    (void)!::write(fd, l.data(), l.size());
    ::close(fd);
}

static bool load_hints(vcfxg_ctx *c, const char *h, size_t n) {
    size_t p = 0;
    while (p < n && h[p] == '#') {
        const void *q = memchr(h + p, '\n', n - p);
        if (!q) return true;  // a '#' line cut by the chunk end: no hints
        p = (size_t)((const char *)q - h) + 1;
    }
    if (p >= n) return false;  // header lines only: the data starts in a later chunk
    const size_t first = p;
    int lines = 0;
    while (p < n && lines < 256) {
        const char *q = (const char *)memchr(h + p, '\n', n - p);
        const size_t e = q ? (size_t)(q - h) : n;
        if (lines == 0) {
            int tabs = 0;
            size_t x = p, f8 = 0;
            while (x < e && tabs < 9) {
                const char *t = (const char *)memchr(h + x, '\t', e - x);
                if (!t) break;
                if (tabs == 8) {
                    c->hint_gt_only = (size_t)(t - h) - f8 == 2 && h[f8] == 'G' && h[f8 + 1] == 'T';
                    c->hint_gt_first = (size_t)(t - h) - f8 > 3 && h[f8] == 'G' && h[f8 + 1] == 'T' && h[f8 + 2] == ':';
                }
                x = (size_t)(t - h) + 1;
                tabs++;
                if (tabs == 8) f8 = x;
            }
            if (tabs == 9) c->hint_span = (int64_t)(e - x);
        }
        lines++;
        p = e + 1;
    }
    if (lines) c->hint_line = (int64_t)((std::min(p, n) - first) / (size_t)lines);
    // the walkers' chunk: 128 KiB, or about 12 records (rounded up to 64 KiB, at most 4 MiB) for
    // records over 16 KiB: each walker's two backward boundary scans read about one record, so
    // long records want longer chunks (GT:AD:DP, 30 KB records: 128 KiB 5.03 ms, 512 KiB 4.76,
    // 1 MiB 5.10; r03 sweep; r05, XCD-contiguous walker blocks: 256 KiB 3.73 ms, 384 KiB 3.65,
    // 512 KiB 3.69, 768 KiB 3.89).  VCFXG_WALK_CHUNK overrides.
    if (!getenv("VCFXG_WALK_CHUNK"))
        c->walk_chunk = c->hint_line > 16 * 1024
                            ? std::min<int64_t>(((12 * c->hint_line + 65535) / 65536) * 65536, 4 << 20)
                            : 128 * 1024;
    return true;
}

int vcfxg_load_host(vcfxg_ctx *c, const char *host, size_t n) {
    if (!c || (!host && n)) return VCFXG_E_ARG;
    int r = vcfxg_ingest_begin(c, n);
    if (!r) r = vcfxg_ingest(c, host, n, 1);
    return r;
}

int vcfxg_ingest_begin(vcfxg_ctx *c, size_t size_hint) {
    if (c) c->dense_pending = false;  // a new index / regions replace the pending ones
    if (!c) return VCFXG_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    // (a staged BGZF stream abandoned before vcfxg_ingest_bgzf may still have copies and inflate
    // batches in flight on their own streams: they finish before the input is written again)
    if (c->copy_stream) HIPCHK(c, hipStreamSynchronize(c->copy_stream));
    for (int k = 0; k < vcfxg_ctx::kBgzStreams; k++)
        if (c->bgz_stream[k]) HIPCHK(c, hipStreamSynchronize(c->bgz_stream[k]));
    if (c->bgz_side.aux) HIPCHK(c, hipStreamSynchronize(c->bgz_side.aux));
    c->bgz_total = c->bgz_staged = 0;
    // (a hint past half of the memory the input could take -- free memory plus its buffer now --
    // is cut to that half: the walk's, LD's and the inflate's buffers keep the rest, and the
    // ingest grows the buffer if the bytes need more)
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && size_hint > (fr + c->input.cap) / 2)
        size_hint = (fr + c->input.cap) / 2;
    int r = ensure(c, c->input, size_hint + kPad);
    if (r) return r;
    c->loaded = false;
    c->indexed = false;
    c->n = 0;
    c->ingesting = true;
    reset_hints(c);
    c->hints_pending = true;
    return VCFXG_OK;
}

static int ingest_mark(vcfxg_ctx *c, size_t upto);

int vcfxg_ingest(vcfxg_ctx *c, const char *host, size_t n, int is_final_chunk) {
    if (!c || (!host && n)) return VCFXG_E_ARG;
    if (!c->ingesting) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    if (c->n + n + kPad > c->input.cap) {
        // grow: a larger buffer, the bytes so far copied on the device
        size_t nc = std::max(c->input.cap * 2, c->n + n + kPad);
        void *np = nullptr;
        HIPCHK(c, hipMalloc(&np, nc));
        if (c->n) HIPCHK(c, hipMemcpyAsync(np, c->input.p, c->n, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->input.p));
        c->input.p = np;
        c->input.cap = nc;
    }
    // pageable host memory: the runtime's staged DMA runs at the PCIe rate (measured
    // 50-56 GB/s on MI355X, tools/microbench/h2d_ingest.cpp), asynchronous to the caller
    // up to its staging depth
    if (n) HIPCHK(c, hipMemcpyAsync(static_cast<char *>(c->input.p) + c->n, host, n, hipMemcpyHostToDevice, c->stream));
    if (n && !is_final_chunk) {  // completion marker for vcfxg_ingest_wait
        int r = ingest_mark(c, c->n + n);
        if (r) return r;
    }
    if (n && c->hints_pending) c->hints_pending = !load_hints(c, host, n);
    c->n += n;
    if (n) c->last_byte = (unsigned char)host[n - 1];
    if (!is_final_chunk) return VCFXG_OK;
    if (!c->n) c->last_byte = -1;
    HIPCHK(c, hipMemsetAsync(static_cast<char *>(c->input.p) + c->n, 0, kPad, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (auto &pe : c->ingest_ev) c->ingest_ev_free.push_back(pe.second);
    c->ingest_ev.clear();
    c->hints_pending = false;
    c->ingesting = false;
    c->loaded = true;
    c->indexed = false;
    return VCFXG_OK;
}

static_assert(sizeof(vcfxg_bgzf_member) == sizeof(vcfxg::BgzfMember), "BGZF member layout");
constexpr size_t kCompPad = 8192;  // the inflate reader's ring loads run up to 3 KiB past a stream

// a completion marker for vcfxg_ingest_wait at stream offset `upto`
static int ingest_mark(vcfxg_ctx *c, size_t upto) {
    hipEvent_t e = nullptr;
    if (!c->ingest_ev_free.empty()) {
        e = c->ingest_ev_free.back();
        c->ingest_ev_free.pop_back();
    } else {
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    HIPCHK(c, hipEventRecord(e, c->stream));
    c->ingest_ev.push_back({upto, e});
    return VCFXG_OK;
}

// (a member holds >= 20 compressed bytes: at most this many members in a stream)
static uint64_t bgz_max_members(size_t comp_total) { return comp_total / 20 + 2; }

// The member tables (members, output offsets, verdicts, the lane order) of a staged stream hold
// `want` members, keeping the first `keep` (the entries the launched batches wrote; every batch
// is complete -- the caller made `stream` wait for them).  Sized at the stage's start for members
// of >= 1 KiB compressed (a genotype VCF's are ~4 KiB): 28 B a member where the worst case
// (20-byte members) would be ~1.4x the compressed bytes; a stream of smaller members stops
// batching (E_CAP) and grows them at the end.
static int bgz_tables(vcfxg_ctx *c, uint64_t want, uint64_t keep) {
    struct Tab {
        DevBuf *b;
        size_t w;
    } t[] = {{&c->bgz_mem, sizeof(vcfxg_bgzf_member)}, {&c->bgz_off, 8}, {&c->bgz_stat, 4}, {&c->bgz_perm, 4}};
    bool need = false;
    for (const Tab &x : t) need = need || x.b->cap < x.w * want;
    if (!need) return VCFXG_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (const Tab &x : t) {
        if (x.b->cap >= x.w * want) continue;
        const size_t nc = x.w * want + x.w * want / 8;
        void *np = nullptr;
        HIPCHK(c, hipMalloc(&np, nc));
        if (keep && x.b->p) HIPCHK(c, hipMemcpyAsync(np, x.b->p, x.w * keep, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (x.b->p) HIPCHK(c, hipFree(x.b->p));
        x.b->p = np;
        x.b->cap = nc;
    }
    return VCFXG_OK;
}
static uint64_t bgz_table_members(const vcfxg_ctx *c) { return c->bgz_mem.cap / sizeof(vcfxg_bgzf_member); }

int vcfxg_bgzf_stage(vcfxg_ctx *c, const void *host, size_t n, size_t offset, size_t comp_total) {
    if (!c || (!host && n) || offset > comp_total || n > comp_total - offset) return VCFXG_E_ARG;
    if (!c->ingesting) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    if (offset == 0) {
        static const uint64_t tset = [] {  // (VCFXG_BGZF_TABLE: the members sized for; tests: tiny)
            const char *e = getenv("VCFXG_BGZF_TABLE");
            return e && *e ? std::max<uint64_t>(2, strtoull(e, nullptr, 10)) : (uint64_t)0;
        }();
        const uint64_t mm = std::min<uint64_t>(bgz_max_members(comp_total),
                                               tset ? tset : std::max<uint64_t>(65536, comp_total / 1024));
        lib_phase("bgzf stage: begin");
        int r = ensure(c, c->bgz_in, comp_total + kCompPad);
        lib_phase("bgzf stage: compressed buffer");
        if (!r) r = bgz_tables(c, mm, 0);
        if (!r) r = ensure(c, c->bgz_small, 64);
        if (r) return r;
        lib_phase("bgzf stage: member tables");
        if (!c->copy_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
        if (!c->bgz_copy_ev) HIPCHK(c, hipEventCreateWithFlags(&c->bgz_copy_ev, hipEventDisableTiming));
        for (int k = 0; k < vcfxg_ctx::kBgzStreams; k++) {
            if (!c->bgz_stream[k]) HIPCHK(c, hipStreamCreateWithFlags(&c->bgz_stream[k], hipStreamNonBlocking));
            if (!c->bgz_ev[k]) HIPCHK(c, hipEventCreateWithFlags(&c->bgz_ev[k], hipEventDisableTiming));
        }
        c->bgz_next = 0;
        lib_phase("bgzf stage: streams");
        // (the first-bad marker and the hand-over count, then the stream's earlier work -- buffers
        // just reallocated, the last call's kernels: every batch is ordered after this event)
        HIPCHK(c, hipMemsetAsync(c->bgz_small.p, 0xFF, 8, c->stream));
        HIPCHK(c, hipMemsetAsync(P<uint8_t>(c->bgz_small) + 8, 0, 56, c->stream));
        HIPCHK(c, hipEventRecord(c->bgz_copy_ev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->bgz_copy_ev, 0));
        c->bgz_total = comp_total;
        c->bgz_staged = 0;
        c->bgz_launched = 0;
        c->bgz_out = 0;
    }
    if (comp_total != c->bgz_total || offset != c->bgz_staged) return VCFXG_E_ARG;  // (in order)
    if (!n) return VCFXG_OK;
    // the copies on their own stream, so they overlap the inflate batches (vcfxg_bgzf_inflate)
    HIPCHK(c, hipMemcpyAsync(P<uint8_t>(c->bgz_in) + offset, host, n, hipMemcpyHostToDevice, c->copy_stream));
    c->bgz_staged = offset + n;
    if (c->bgz_staged == comp_total)
        HIPCHK(c, hipMemsetAsync(P<uint8_t>(c->bgz_in) + comp_total, 0, kCompPad, c->copy_stream));
    HIPCHK(c, hipEventRecord(c->bgz_copy_ev, c->copy_stream));
    // (the completion marker for vcfxg_ingest_wait: recorded on the copy stream)
    hipEvent_t e = nullptr;
    if (!c->ingest_ev_free.empty()) {
        e = c->ingest_ev_free.back();
        c->ingest_ev_free.pop_back();
    } else {
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    HIPCHK(c, hipEventRecord(e, c->copy_stream));
    c->ingest_ev.push_back({offset + n, e});
    return VCFXG_OK;
}

// launch the inflate of members [first, first + count) of the staged stream: their table entries
// and output offsets (from the running output count) to the device, k_inflate after the copies
// staged so far
// the token buffer of stream slot k (kBgzStreams: c->stream) for `count` members: at most 69,632 at
// a time (2.3 GB: the bench shard's 65,834 members in one launch), fewer when the device cannot
// spare that (down to 4,096; launches of more members run in pieces); 0 members when even that
// cannot be had (every member then on the wave decoder)
static uint64_t bgz_tokens(vcfxg_ctx *c, int k, uint64_t count, hipStream_t st) {
    DevBuf &b = c->bgz_tok[k];
    const size_t per = (size_t)vcfxg::kTokCap * 4 + 4;  // (the tokens, and a hand-over list entry)
    for (uint64_t want = std::min<uint64_t>(count, 69632);; want /= 2) {
        if (b.cap >= want * per + 4) return want;
        if (b.p) {  // (the stream's earlier batches may still read it)
            if (hipStreamSynchronize(st) != hipSuccess) return 0;
            (void)hipFree(b.p);
            b.p = nullptr;
            b.cap = 0;
        }
        // (rounded up to 8,192 members: a batch a few members past the last one's size reuses it)
        const uint64_t alloc = std::min<uint64_t>((want + 8191) / 8192 * 8192, std::max<uint64_t>(want, 69632));
        if (hipMalloc(&b.p, alloc * per + 4) == hipSuccess) {
            b.cap = alloc * per + 4;
            return want;
        }
        (void)hipGetLastError();
        b.p = nullptr;
        if (want <= 4096) return 0;
    }
}

// the lane decoder's member order for `count` members: largest compressed first (a counting sort
// on 64-byte buckets: the lanes of a wave then decode similar amounts, and the largest go first)
static std::vector<uint32_t> bgz_order(const vcfxg_bgzf_member *mem, uint64_t count) {
    constexpr uint32_t kB = 1026;  // (src_len <= 65,536 + header slack: buckets of 64 B)
    std::vector<uint32_t> cnt(kB + 1, 0), perm(count);
    auto bucket = [&](uint64_t i) { return kB - 1 - std::min<uint32_t>(mem[i].src_len >> 6, kB - 1); };
    for (uint64_t i = 0; i < count; i++) cnt[bucket(i) + 1]++;
    for (uint32_t b = 0; b < kB; b++) cnt[b + 1] += cnt[b];
    for (uint64_t i = 0; i < count; i++) perm[cnt[bucket(i)]++] = (uint32_t)i;
    return perm;
}

// the lane decoder's side stream and events (created once)
static int bgz_aux(vcfxg_ctx *c) {
    vcfxg::InflateSide &d = c->bgz_side;
    if (!d.aux) HIPCHK(c, hipStreamCreateWithFlags(&d.aux, hipStreamNonBlocking));
    for (hipEvent_t &e : d.ev)
        if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return VCFXG_OK;
}

// the CRC-32 pass's "1 KiB of zeros" basis
static const vcfxg::Crc1k &crc_basis() {
    static const vcfxg::Crc1k z = [] {
        vcfxg::Crc1k b;
        vcfxg::crc32_zero1k_basis(&b);
        return b;
    }();
    return z;
}

// members [first, first + count) of a staged stream: the tables, the inflate and its CRC-32 pass
// on `st` (so the last batch's check does not wait for a pass over every member)
static int bgz_launch(vcfxg_ctx *c, const vcfxg_bgzf_member *mem, uint64_t first, uint64_t count,
                      hipStream_t st, int slot) {
    if (!count) return VCFXG_OK;
    const std::vector<uint32_t> perm = bgz_order(mem, count);
    HIPCHK(c, hipMemcpyAsync(P<uint32_t>(c->bgz_perm) + first, perm.data(), 4 * count, hipMemcpyHostToDevice, st));
    std::vector<uint64_t> off(count);
    uint64_t o = c->bgz_out;
    for (uint64_t i = 0; i < count; i++) {
        off[i] = o;
        o += mem[i].out_len;
    }
    HIPCHK(c, hipMemcpyAsync(P<vcfxg_bgzf_member>(c->bgz_mem) + first, mem, sizeof(vcfxg_bgzf_member) * count,
                             hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(P<uint64_t>(c->bgz_off) + first, off.data(), 8 * count, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipStreamWaitEvent(st, c->bgz_copy_ev, 0));
    const uint64_t tm = bgz_tokens(c, slot, count, st);
    if (int r = bgz_aux(c)) return r;
    for (int which = 0; which < 2; which++)
        HIPCHK(c, vcfxg::launch_inflate(which, P<uint8_t>(c->bgz_in), P<vcfxg::BgzfMember>(c->bgz_mem) + first,
                                        P<uint64_t>(c->bgz_off) + first, count, P<uint8_t>(c->input) + c->n,
                                        P<uint32_t>(c->bgz_stat) + first, P<unsigned long long>(c->bgz_small),
                                        crc_basis(), st, first, P<uint32_t>(c->bgz_tok[slot]), tm,
                                        P<uint32_t>(c->bgz_perm) + first, &c->bgz_side));
    c->bgz_launched = first + count;
    c->bgz_out = o;
    return VCFXG_OK;
}

int vcfxg_bgzf_inflate(vcfxg_ctx *c, const vcfxg_bgzf_member *mem, size_t count) {
    if (!c || (!mem && count)) return VCFXG_E_ARG;
    if (!c->ingesting || !c->bgz_total) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    uint64_t out = 0;
    for (size_t i = 0; i < count; i++) {
        if (mem[i].src_off > c->bgz_staged || mem[i].src_len > c->bgz_staged - mem[i].src_off || mem[i].src_len < 20 ||
            mem[i].out_len > 65536)
            return VCFXG_E_ARG;  // (not staged yet, or out of range)
        out += mem[i].out_len;
    }
    if (c->bgz_launched + count > bgz_max_members(c->bgz_total)) return VCFXG_E_ARG;
    if (c->bgz_launched + count + 1 > bgz_table_members(c)) return VCFXG_E_CAP;  // (the rest at the end)
    // the output must fit the input buffer as it is (growing it here would move the bytes the
    // launched batches are writing): the rest waits for vcfxg_ingest_bgzf, which grows it
    if (c->n + c->bgz_out + out + kPad > c->input.cap) return VCFXG_E_CAP;
    const int k = c->bgz_next;
    c->bgz_next = (k + 1) % vcfxg_ctx::kBgzStreams;
    int r = bgz_launch(c, mem, c->bgz_launched, count, c->bgz_stream[k], k);
    if (r) return r;
    HIPCHK(c, hipEventRecord(c->bgz_ev[k], c->bgz_stream[k]));
    return VCFXG_OK;
}

int vcfxg_ingest_bgzf(vcfxg_ctx *c, const void *comp, size_t comp_n, const vcfxg_bgzf_member *mem, size_t nm,
                      const char *head, size_t head_n, uint64_t *bad_member) {
    // comp = NULL: the compressed bytes were staged by vcfxg_bgzf_stage (all comp_n of them), and
    // members [0, bgz_launched) were launched by vcfxg_bgzf_inflate (mem[] must begin with them)
    const bool staged = !comp;
    if (!c || (staged && comp_n && (c->bgz_total != comp_n || c->bgz_staged != comp_n)) || (!mem && nm) ||
        (!head && head_n))
        return VCFXG_E_ARG;
    if (!c->ingesting) return VCFXG_E_STATE;
    if (bad_member) *bad_member = ~0ull;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t done = staged ? c->bgz_launched : 0;  // members launched already
    if (done > nm || (staged && nm > bgz_max_members(comp_n))) return VCFXG_E_ARG;
    std::vector<uint64_t> off(nm + 1);
    uint64_t tot = 0;
    for (size_t i = 0; i < nm; i++) {
        // (the kernel reads the header's XLEN and the trailer inside the member)
        if (mem[i].src_off > comp_n || mem[i].src_len > comp_n - mem[i].src_off || mem[i].src_len < 20 ||
            mem[i].out_len > 65536) {
            c->err = "vcfxg_ingest_bgzf: member " + std::to_string(i) + " out of range";
            return VCFXG_E_ARG;
        }
        off[i] = tot;
        tot += mem[i].out_len;
    }
    off[nm] = tot;
    if (staged && done && off[done] != c->bgz_out) return VCFXG_E_ARG;  // (not the launched members)
    if (staged) {
        // every staged copy and every launched batch before anything below (the grow copies the
        // batches' output; the kernels below read the staged bytes)
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->bgz_copy_ev, 0));
        if (done)
            for (int k = 0; k < vcfxg_ctx::kBgzStreams; k++) HIPCHK(c, hipStreamWaitEvent(c->stream, c->bgz_ev[k], 0));
        if (int rt = bgz_tables(c, nm + 1, done)) return rt;  // (more members than the stage sized for)
    }
    if (c->n + tot + kPad > c->input.cap) {  // grow as vcfxg_ingest does (keeping launched output)
        const size_t keep = c->n + (size_t)(staged ? c->bgz_out : 0);
        size_t ncap = std::max(c->input.cap * 2, c->n + tot + kPad);
        void *np = nullptr;
        HIPCHK(c, hipMalloc(&np, ncap));
        if (keep) HIPCHK(c, hipMemcpyAsync(np, c->input.p, keep, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->input.p));
        c->input.p = np;
        c->input.cap = ncap;
    }
    int r = VCFXG_OK;
    if (!staged) {
        r = ensure(c, c->bgz_in, comp_n + kCompPad);
        if (!r) r = ensure(c, c->bgz_mem, sizeof(vcfxg_bgzf_member) * (nm + 1));
        if (!r) r = ensure(c, c->bgz_off, 8 * (nm + 1));
        if (!r) r = ensure(c, c->bgz_stat, 4 * (nm + 1));
        if (!r) r = ensure(c, c->bgz_small, 64);
        if (!r) r = ensure(c, c->bgz_perm, 4 * (nm + 1));
        if (r) return r;
    }
    const vcfxg::Crc1k &z1k = crc_basis();
    if (staged) {
        // the members not launched yet
        prof_begin(c, "bgzf_inflate");
        r = bgz_launch(c, mem + done, done, nm - done, c->stream, vcfxg_ctx::kBgzStreams);
        prof_end(c, "bgzf_inflate");
        if (r) return r;
    } else {
        prof_begin(c, "bgzf_h2d");
        if (comp_n) HIPCHK(c, hipMemcpyAsync(c->bgz_in.p, comp, comp_n, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemsetAsync(P<uint8_t>(c->bgz_in) + comp_n, 0, kCompPad, c->stream));
        if (nm) {
            HIPCHK(c, hipMemcpyAsync(c->bgz_mem.p, mem, sizeof(vcfxg_bgzf_member) * nm, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipMemcpyAsync(c->bgz_off.p, off.data(), 8 * nm, hipMemcpyHostToDevice, c->stream));
        }
        HIPCHK(c, hipMemsetAsync(c->bgz_small.p, 0xFF, 8, c->stream));
        HIPCHK(c, hipMemsetAsync(P<uint8_t>(c->bgz_small) + 8, 0, 56, c->stream));
        prof_end(c, "bgzf_h2d");
        const uint64_t tm = bgz_tokens(c, vcfxg_ctx::kBgzStreams, nm, c->stream);
        if (int ra = bgz_aux(c)) return ra;
        const std::vector<uint32_t> perm = bgz_order(mem, nm);
        if (nm) HIPCHK(c, hipMemcpyAsync(c->bgz_perm.p, perm.data(), 4 * nm, hipMemcpyHostToDevice, c->stream));
        prof_begin(c, "bgzf_inflate");
        HIPCHK(c, vcfxg::launch_inflate(0, P<uint8_t>(c->bgz_in), P<vcfxg::BgzfMember>(c->bgz_mem),
                                        P<uint64_t>(c->bgz_off), nm, P<uint8_t>(c->input) + c->n,
                                        P<uint32_t>(c->bgz_stat), P<unsigned long long>(c->bgz_small), z1k, c->stream, 0,
                                        P<uint32_t>(c->bgz_tok[vcfxg_ctx::kBgzStreams]), tm, P<uint32_t>(c->bgz_perm), &c->bgz_side));
        prof_end(c, "bgzf_inflate");
    }
    prof_begin(c, "bgzf_crc32");
    if (!staged)  // (a staged stream's batches checked their own members, bgz_launch)
        HIPCHK(c, vcfxg::launch_inflate(1, P<uint8_t>(c->bgz_in), P<vcfxg::BgzfMember>(c->bgz_mem),
                                        P<uint64_t>(c->bgz_off), nm, P<uint8_t>(c->input) + c->n,
                                        P<uint32_t>(c->bgz_stat), P<unsigned long long>(c->bgz_small), z1k, c->stream));
    prof_end(c, "bgzf_crc32");
    // the first bad member, the hand-over count and its reasons (32-bit words 3..14)
    static thread_local uint64_t small[8];
    static thread_local uint8_t lastb;
    uint64_t &bad = small[0];
    HIPCHK(c, hipMemcpyAsync(small, c->bgz_small.p, 64, hipMemcpyDeviceToHost, c->stream));
    if (tot) HIPCHK(c, hipMemcpyAsync(&lastb, P<uint8_t>(c->input) + c->n + tot - 1, 1, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->bgz_total = c->bgz_staged = 0;
    c->bgz_launched = c->bgz_out = 0;
    c->bgz_handed = (uint32_t)small[1];
    if (c->bgz_handed && getenv("VCFX_BGZF_DIAG")) {  // (why the lane decoder handed members over)
        const uint32_t *w = reinterpret_cast<const uint32_t *>(small) + 2;
        fprintf(stderr, "vcfxg: BGZF members handed to the wave decoder: %u (by reason 1-12:", w[0]);
        for (int k = 1; k <= 12; k++) fprintf(stderr, " %u", w[k]);
        fprintf(stderr, ")\n");
    }
    if (bad != ~0ull) {
        uint32_t why = 0;
        (void)hipMemcpy(&why, P<uint32_t>(c->bgz_stat) + bad, 4, hipMemcpyDeviceToHost);
        if (bad_member) *bad_member = bad;
        c->err = "BGZF member " + std::to_string(bad) + " does not inflate (check " + std::to_string(why) + ")";
        c->ingesting = false;
        c->loaded = false;
        c->n = 0;
        return VCFXG_E_DATA;
    }
    if (head_n && c->hints_pending) c->hints_pending = !load_hints(c, head, head_n);
    note_schedule(c, staged ? "bgzf_inflate_staged" : "bgzf_inflate");
    c->n += tot;
    if (tot) c->last_byte = lastb;
    return VCFXG_OK;
}

int vcfxg_ingest_wait(vcfxg_ctx *c, size_t upto) {
    if (!c) return VCFXG_E_ARG;
    size_t k = 0;
    while (k < c->ingest_ev.size() && c->ingest_ev[k].first <= upto) k++;
    if (k == 0) return VCFXG_OK;
    HIPCHK(c, hipEventSynchronize(c->ingest_ev[k - 1].second));
    for (size_t i = 0; i < k; i++) c->ingest_ev_free.push_back(c->ingest_ev[i].second);
    c->ingest_ev.erase(c->ingest_ev.begin(), c->ingest_ev.begin() + (long)k);
    return VCFXG_OK;
}

int vcfxg_count_byte(vcfxg_ctx *c, uint64_t from, int byte, uint64_t *count) {
    if (!c || !count || byte < 0 || byte > 255) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    HIPCHK(c, hipSetDevice(c->device));
    *count = 0;
    if (from >= c->n) return VCFXG_OK;
    int r = ensure(c, c->byte_cnt, 8);
    if (r) return r;
    HIPCHK(c, hipMemsetAsync(c->byte_cnt.p, 0, 8, c->stream));
    prof_begin(c, "count_byte");
    HIPCHK(c, vcfxg::launch_count_byte(P<uint8_t>(c->input), from, c->n, (uint8_t)byte,
                                       P<unsigned long long>(c->byte_cnt), c->stream));
    prof_end(c, "count_byte");
    static thread_local uint64_t h;
    HIPCHK(c, hipMemcpyAsync(&h, c->byte_cnt.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    *count = h;
    return VCFXG_OK;
}

int vcfxg_host_alloc(vcfxg_ctx *c, size_t n, void **out) {
    if (!c || !out) return VCFXG_E_ARG;
    *out = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipHostMalloc(out, n ? n : 1, hipHostMallocDefault));
    return VCFXG_OK;
}

void vcfxg_host_free(vcfxg_ctx *c, void *p) {
    if (c && p) (void)hipHostFree(p);
}

int vcfxg_input_fetch(vcfxg_ctx *c, uint64_t offset, size_t n, void *host) {
    if (!c || (!host && n)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (offset > c->n || n > c->n - offset) return VCFXG_E_ARG;
    if (!n) return VCFXG_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(host, static_cast<const char *>(c->input.p) + offset, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

const void *vcfxg_input_device_ptr(vcfxg_ctx *c) { return c && c->loaded ? c->input.p : nullptr; }

int vcfxg_index(vcfxg_ctx *c, size_t data_start, uint64_t *n_lines) {
    if (c) c->dense_pending = false;  // a new index / regions replace the pending ones
    if (!c) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n;
    const int64_t nc = vcfxg::idx_wchunks(lo, hi);
    int r = ensure(c, c->idx_counts, sizeof(uint32_t) * (size_t)(nc + 1));
    if (!r) r = ensure(c, c->idx_offs, sizeof(uint64_t) * (size_t)(nc + 1));
    if (!r) r = ensure(c, c->idx_pos, sizeof(uint64_t) * (size_t)nc * vcfxg::idx_pos_cap() + 64);
    if (r) return r;
    const char *buf = P<char>(c->input);
    unsigned *overflow = reinterpret_cast<unsigned *>(P<uint64_t>(c->idx_pos) + (size_t)nc * vcfxg::idx_pos_cap());
    HIPCHK(c, hipMemsetAsync(overflow, 0, 8, c->stream));
    prof_begin(c, "line_count");
    HIPCHK(c, vcfxg::launch_idx_count(buf, lo, hi, P<uint32_t>(c->idx_counts), P<uint64_t>(c->idx_pos), overflow,
                                      c->stream));
    prof_end(c, "line_count");
    HIPCHK(c, hipMemsetAsync(P<uint32_t>(c->idx_counts) + nc, 0, sizeof(uint32_t), c->stream));
    r = exclusive_scan(c, P<uint32_t>(c->idx_counts), P<uint64_t>(c->idx_offs), (size_t)nc + 1);
    if (r) return r;
    static thread_local uint64_t total;
    static thread_local unsigned ovf;
    HIPCHK(c, hipMemcpyAsync(&total, P<uint64_t>(c->idx_offs) + nc, sizeof total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&ovf, overflow, sizeof ovf, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const bool tail = hi > lo && c->last_byte != '\n';
    const uint64_t nl = total + (tail ? 1 : 0);
    r = ensure(c, c->line_end, sizeof(uint64_t) * (size_t)(nl + 1));
    if (r) return r;
    if (ovf) {  // some chunk has more newlines than the scratch holds: the emit sweep
        prof_begin(c, "line_emit");
        HIPCHK(c, vcfxg::launch_idx_emit(buf, lo, hi, P<uint64_t>(c->idx_offs), P<uint64_t>(c->line_end), c->stream));
        prof_end(c, "line_emit");
    } else {
        prof_begin(c, "line_compact");
        HIPCHK(c, vcfxg::launch_nl_compact(lo, hi, P<uint32_t>(c->idx_counts), P<uint64_t>(c->idx_offs),
                                           P<uint64_t>(c->idx_pos), P<uint64_t>(c->line_end), c->stream));
        prof_end(c, "line_compact");
    }
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
    DENSE(c);
    if (first + count > c->n_lines) return VCFXG_E_ARG;
    if (!count) return VCFXG_OK;
    HIPCHK(c, hipMemcpyAsync(out, P<uint64_t>(c->line_end) + first, count * sizeof(uint64_t), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

static int af_buffers(vcfxg_ctx *c, uint64_t L) {
    int r = ensure(c, c->alt, 4 * (L + 1));
    if (!r) r = ensure(c, c->tot, 4 * (L + 1));
    if (!r) r = ensure(c, c->rowpre, 4 * (L + 1));
    if (!r) r = ensure(c, c->status, L + 1);
    if (!r) r = ensure(c, c->rowlen, 8 * (L + 1));
    if (!r) r = ensure(c, c->rowoff, 8 * (L + 1));
    return r;
}

static int af_rows(vcfxg_ctx *c, int mode, vcfxg_summary *out);

int vcfxg_allele_freq(vcfxg_ctx *c, int mode, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t L = c->n_lines;
    int r = af_buffers(c, L);
    if (r) return r;
    const char *buf = P<char>(c->input);
    const uint64_t *nl_dev = P<uint64_t>(c->d_nlines);
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    r = ensure(c, c->af_meta, vcfxg::af_meta_bytes() * (L + 1));
    if (r) return r;
    prof_begin(c, "af_records");
    HIPCHK(c, vcfxg::launch_af_meta_sweep(buf, (int64_t)c->data_start, P<uint64_t>(c->line_end), nl_dev, L, mode,
                                          c->af_meta.p, P<int32_t>(c->alt), P<int32_t>(c->tot), P<uint32_t>(c->rowpre),
                                          P<uint8_t>(c->status), P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "af_records");
    return af_rows(c, mode, out);
}


// Default region path, asynchronous: the two-sweep schedule (index sweep + scan +
// compaction, head pass + fixed-stride sweep + the per-line rest, row lengths + scan) runs
// with the line count kept on the device -- buffers sized by the count of the previous call
// (else the no-overflow bound of idx_pos_cap() lines per 16 KiB chunk), compaction and
// kernels guarded by it -- and ONE host synchronisation reads a small summary (lines, text
// bytes, counters, failure) before the formatting kernel.  A failure (a chunk with more
// newlines than the scratch keeps, or more lines than the capacity) reruns the call on the
// synchronous path.
static int af_region_async(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out) {
    if (c) c->dense_pending = false;  // a new index / regions replace the pending ones
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n;
    const int64_t nc = vcfxg::idx_wchunks(lo, hi);
    if (!nc) {
        int r = vcfxg_index(c, data_start, nullptr);
        return r ? r : vcfxg_allele_freq(c, mode, out);
    }
    const size_t pcap = (size_t)vcfxg::idx_pos_cap();
    const uint64_t bound = (uint64_t)nc * pcap + 2;
    const uint64_t cap = c->af_line_cap ? std::min<uint64_t>(c->af_line_cap + 1, bound) : bound;
    int r = ensure(c, c->idx_counts, sizeof(uint32_t) * (size_t)(nc + 1));
    if (!r) r = ensure(c, c->idx_offs, sizeof(uint64_t) * (size_t)(nc + 1));
    if (!r) r = ensure(c, c->idx_pos, sizeof(uint64_t) * (size_t)nc * pcap + 64);
    if (!r) r = ensure(c, c->line_end, 8 * (cap + 1));
    if (!r) r = af_buffers(c, cap);
    if (!r) r = ensure(c, c->af_meta, vcfxg::af_meta_bytes() * (cap + 1));
    if (!r) r = ensure(c, c->async_small, 128);
    if (r) return r;
    const char *buf = P<char>(c->input);
    uint64_t *small = P<uint64_t>(c->async_small);  // [0] 0, [1] n, [2] flags, [4..10] summary
    unsigned *idx_ovf = reinterpret_cast<unsigned *>(small + 2), *failf = idx_ovf + 1;
    HIPCHK(c, hipMemsetAsync(small, 0, 32, c->stream));
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    prof_begin(c, "line_count");
    HIPCHK(c, vcfxg::launch_idx_count(buf, lo, hi, P<uint32_t>(c->idx_counts), P<uint64_t>(c->idx_pos), idx_ovf,
                                      c->stream));
    prof_end(c, "line_count");
    HIPCHK(c, hipMemsetAsync(P<uint32_t>(c->idx_counts) + nc, 0, sizeof(uint32_t), c->stream));
    r = exclusive_scan(c, P<uint32_t>(c->idx_counts), P<uint64_t>(c->idx_offs), (size_t)nc + 1);
    if (r) return r;
    prof_begin(c, "line_compact");
    HIPCHK(c, vcfxg::launch_nl_compact_cap(lo, hi, P<uint32_t>(c->idx_counts), P<uint64_t>(c->idx_offs),
                                           P<uint64_t>(c->idx_pos), P<uint64_t>(c->line_end), cap, c->stream));
    HIPCHK(c, vcfxg::launch_idx_finish(P<uint64_t>(c->idx_offs), nc, idx_ovf, c->last_byte != '\n' ? 1 : 0, hi, cap,
                                       P<uint64_t>(c->line_end), small + 1, failf, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_nlines.p, small + 1, 8, hipMemcpyDeviceToDevice, c->stream));
    prof_end(c, "line_compact");
    prof_begin(c, "af_records");
    HIPCHK(c, vcfxg::launch_af_meta_sweep_range(buf, lo, P<uint64_t>(c->line_end), small, cap, mode, c->af_meta.p,
                                                P<int32_t>(c->alt), P<int32_t>(c->tot), P<uint32_t>(c->rowpre),
                                                P<uint8_t>(c->status), P<unsigned long long>(c->counters), c->stream));
    HIPCHK(c, vcfxg::launch_af_complex(buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), cap, mode,
                                       c->af_meta.p, P<int32_t>(c->alt), P<int32_t>(c->tot), P<uint32_t>(c->rowpre),
                                       P<uint8_t>(c->status), P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "af_records");
    prof_begin(c, "af_rows");
    HIPCHK(c, vcfxg::launch_af_rowlen(P<uint32_t>(c->rowpre), P<uint8_t>(c->status), P<uint64_t>(c->d_nlines), cap,
                                      P<uint64_t>(c->rowlen), c->stream));
    r = exclusive_scan(c, P<uint64_t>(c->rowlen), P<uint64_t>(c->rowoff), (size_t)cap + 1);
    if (r) return r;
    HIPCHK(c, vcfxg::launch_af_summary(P<uint64_t>(c->d_nlines), P<uint64_t>(c->rowoff),
                                       P<unsigned long long>(c->counters), failf, small + 4, c->stream));
    prof_end(c, "af_rows");
    static thread_local uint64_t sm[7];
    HIPCHK(c, hipMemcpyAsync(sm, small + 4, sizeof sm, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (sm[6]) {  // rerun synchronously (and learn the exact line count)
        prof_collect(c);
        c->af_line_cap = 0;
        r = vcfxg_index(c, data_start, nullptr);
        if (!r) r = vcfxg_allele_freq(c, mode, out);
        if (!r) c->af_line_cap = c->n_lines;
        return r;
    }
    const uint64_t L = sm[0], text = sm[1];
    c->af_line_cap = std::max<uint64_t>(c->af_line_cap, L);
    r = ensure(c, c->text, text + 1);
    if (r) return r;
    prof_begin(c, "af_format");
    HIPCHK(c, vcfxg::launch_af_format(buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), L, mode,
                                      P<int32_t>(c->alt), P<int32_t>(c->tot), P<uint32_t>(c->rowpre),
                                      P<uint8_t>(c->status), P<uint64_t>(c->rowoff), P<char>(c->text), c->stream));
    prof_end(c, "af_format");
    prof_collect(c);
    c->data_start = data_start;
    c->n_lines = L;
    c->indexed = true;
    c->text_bytes = text;
    if (out) {
        out->n_lines = L;
        out->rows = sm[2];
        out->data_lines = sm[3];
        out->warn_lines = sm[4];
        out->general_records = sm[5];
        out->text_bytes = text;
    }
    return VCFXG_OK;
}

// Walk region path (default when the first data lines average >= 512 B): no separate
// index sweep.  k_af_walk reads each chunk's lines once, predicting fixed-stride record ends
// and validating them by the sample sweep itself, and leaves per walker its lines' results,
// its rows' bytes and a list of the lines for the exact per-line path.  The tail works on the
// walkers' regions directly: k_af_cx (the listed lines), k_walker_scan (one block: walker line
// and text offsets + the call summary), k_af_format_w (rows, into the previous call's text
// capacity), then ONE host synchronisation.  The dense per-line arrays (line ends, counts,
// statuses) are compacted from the regions only when a later call asks for them
// (ensure_dense).  A walker over its line capacity, or an overlong leftover list, reruns the
// call on the two-sweep schedule (and later calls on this input use it directly).
// the mapped host words the tail kernels write the call summaries into (AF walk [0..7],
// filter / query walk [8..17])
static int ensure_sum_host(vcfxg_ctx *c) {
    if (c->sum_host) return VCFXG_OK;
    HIPCHK(c, hipHostMalloc(reinterpret_cast<void **>(&c->sum_host), 256, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(c->sum_host, 0, 256);
    HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void **>(&c->sum_dev), c->sum_host, 0));
    return VCFXG_OK;
}

static int af_region_walk(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out, bool gf = false) {
    if (c) c->dense_pending = false;  // a new index / regions replace the pending ones
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n;
    const int64_t C = c->walk_chunk;
    const int64_t nw = vcfxg::af_walkers(lo, hi, C);
    if (!nw) {
        int r = vcfxg_index(c, data_start, nullptr);
        return r ? r : vcfxg_allele_freq(c, mode, out);
    }
    const uint64_t cap_w = (uint64_t)(2 * C / std::max<int64_t>(c->hint_line, 64)) + 16;
    if (cap_w > 0xFFFF) {
        // (wgt packs the GT-line count in 16 bits: short records in a large VCFXG_WALK_CHUNK, or a
        // forced walk on them) the two-sweep schedule, as after a walk that ran out of line slots
        c->walk_overflowed = true;
        return note_schedule(c, "af_two_sweep"), af_region_async(c, data_start, mode, out);
    }
    const uint64_t cap = (uint64_t)nw * cap_w;
    int r = ensure(c, c->wk_le, 8 * cap);
    if (!r) r = ensure(c, c->wk_alt, 4 * cap);
    if (!r) r = ensure(c, c->wk_tot, 4 * cap);
    if (!r) r = ensure(c, c->wk_rowpre, 4 * cap);
    if (!r) r = ensure(c, c->wk_status, cap);
    if (!r) r = ensure(c, c->wk_meta, vcfxg::af_meta_bytes() * cap);
    if (!r) r = ensure(c, c->wk_count, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_offs, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_gt, 4 * (size_t)nw);
    if (!r) r = ensure(c, c->wk_text, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_toff, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_start, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_cx, 8 * cap);
    const int64_t nbs = (nw + vcfxg::kWalkerScanBlock - 1) / vcfxg::kWalkerScanBlock;
    if (!r) r = ensure(c, c->wk_bs, 8 * (size_t)(5 * nbs + 4));
    if (!r) r = ensure(c, c->af_small, 128);
    // a walker's rows as text: ~ 13 rows x 31 B on the config 2 shard; a walker whose rows
    // outgrow its stage is formatted from the arrays instead
    constexpr uint32_t kStageCap = 2048;
    if (!r) r = ensure(c, c->wk_stage, (size_t)kStageCap * (size_t)nw);
    if (!r) r = ensure(c, c->wk_dirty, (size_t)nw);
    if (r) return r;
    r = ensure_sum_host(c);
    if (r) return r;
    const char *buf = P<char>(c->input);
    // [0] walk overflow flag (u32), [1] leftover count, [2..5] counters: zero on entry (k_walker_scan
    // clears them for the next call); [6] walker-scan arrivals (u32, reset by its last block)
    uint64_t *bpre_a = P<uint64_t>(c->wk_bs), *bpre_b = bpre_a + nbs + 1, *bsum = bpre_b + nbs + 1;
    uint64_t *small = P<uint64_t>(c->af_small);
    unsigned *ovf = reinterpret_cast<unsigned *>(small);
    unsigned long long *cx_n = reinterpret_cast<unsigned long long *>(small + 1);
    unsigned long long *cnt = reinterpret_cast<unsigned long long *>(small + 2);
    if (c->af_small_dirty) HIPCHK(c, hipMemsetAsync(small, 0, 128, c->stream));
    c->af_small_dirty = true;  // until the call has synchronised
    vcfxg::WalkTail tail;
    tail.wtext = P<uint64_t>(c->wk_text);
    tail.wstart = P<uint64_t>(c->wk_start);
    tail.cx_list = P<uint64_t>(c->wk_cx);
    tail.cx_n = cx_n;
    tail.cx_cap = cap;
    tail.stage = P<char>(c->wk_stage);
    tail.stage_cap = kStageCap;
    tail.wdirty = P<uint8_t>(c->wk_dirty);
    prof_begin(c, "af_walk");
    HIPCHK(c, vcfxg::launch_af_walk(buf, lo, hi, C, mode, c->hint_span, cap_w, P<uint64_t>(c->wk_le),
                                    P<int32_t>(c->wk_alt), P<int32_t>(c->wk_tot), P<uint32_t>(c->wk_rowpre),
                                    P<uint8_t>(c->wk_status), c->wk_meta.p, P<uint64_t>(c->wk_count),
                                    P<uint32_t>(c->wk_gt), ovf, c->stream, nullptr, &tail, false, gf));
    prof_end(c, "af_walk");
    prof_begin(c, "af_complex");
    // the grid: a wave per leftover line of the previous call (usually none; 16 blocks at least)
    const uint64_t cx_grid_lines = std::min<uint64_t>(cap, std::max<uint64_t>(c->cx_hint, 64));
    HIPCHK(c, vcfxg::launch_af_cx(buf, mode, cap_w, tail.cx_list, cx_n, cap, cx_grid_lines, tail.wstart,
                                  P<uint64_t>(c->wk_le), c->wk_meta.p, P<int32_t>(c->wk_alt), P<int32_t>(c->wk_tot),
                                  P<uint32_t>(c->wk_rowpre), P<uint8_t>(c->wk_status), tail.wtext, cnt, c->stream));
    prof_end(c, "af_complex");
    prof_begin(c, "af_rows");
    uint64_t *sm = c->sum_host;  // lines, text bytes, counters[0..3], walk overflow, leftovers
    HIPCHK(c, vcfxg::launch_walker_scan(nw, P<uint64_t>(c->wk_count), tail.wtext, P<uint32_t>(c->wk_gt),
                                        P<uint64_t>(c->wk_offs), P<uint64_t>(c->wk_toff), bpre_a, bpre_b, bsum,
                                        reinterpret_cast<unsigned *>(small + 6), cnt, ovf, P<uint64_t>(c->d_nlines),
                                        c->sum_dev, c->stream, small));
    prof_end(c, "af_rows");
    // the rows go out before the host has seen their total: into the text capacity of the
    // previous call (rows past it are skipped, and all are written again below once it has
    // grown), so the call synchronises with the host once
    const uint64_t tcap = std::max<uint64_t>(c->text_hint, 1u << 16);
    r = ensure(c, c->text, tcap + 1);
    if (r) return r;
    prof_begin(c, "af_format");
    HIPCHK(c, vcfxg::launch_af_format_w(buf, mode, nw, cap_w, P<uint64_t>(c->wk_count), P<uint64_t>(c->wk_toff),
                                        bpre_b, tail.wstart, P<uint64_t>(c->wk_le), P<int32_t>(c->wk_alt),
                                        P<int32_t>(c->wk_tot), P<uint32_t>(c->wk_rowpre), P<uint8_t>(c->wk_status),
                                        P<char>(c->text), tcap, c->stream, &tail));
    prof_end(c, "af_format");
    // (the leftover list holds every slot at most once: it cannot overflow its capacity)
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->af_small_dirty = false;
    c->cx_hint = sm[7];
    if (sm[6]) {  // a walker ran out of line slots (short lines): the two-sweep schedule
        prof_collect(c);
        c->walk_overflowed = true;
        return af_region_async(c, data_start, mode, out);
    }
    const uint64_t L = sm[0], text = sm[1];
    c->text_hint = text;
    if (text > tcap) {  // the text outgrew the previous capacity: all rows again
        r = ensure(c, c->text, text + 1);
        if (r) return r;
        prof_begin(c, "af_format");
        HIPCHK(c, vcfxg::launch_af_format_w(buf, mode, nw, cap_w, P<uint64_t>(c->wk_count), P<uint64_t>(c->wk_toff),
                                            bpre_b, tail.wstart, P<uint64_t>(c->wk_le), P<int32_t>(c->wk_alt),
                                            P<int32_t>(c->wk_tot), P<uint32_t>(c->wk_rowpre),
                                            P<uint8_t>(c->wk_status), P<char>(c->text), ~0ull, c->stream, &tail));
        prof_end(c, "af_format");
    }
    prof_collect(c);
    c->data_start = data_start;
    c->n_lines = L;
    c->indexed = true;
    c->text_bytes = text;
    c->dense_nw = nw;  // the dense arrays come from the regions on demand
    c->dense_cap_w = cap_w;
    c->dense_pending = true;
    if (out) {
        out->n_lines = L;
        out->rows = sm[2];
        out->data_lines = sm[3];
        out->warn_lines = sm[4];
        out->general_records = sm[5];
        out->text_bytes = text;
    }
    return VCFXG_OK;
}

// the dense per-line arrays (line_end, alt, tot, rowpre, status, meta) of the last walk
// region call, compacted from its walker regions (k_walk_compact; counters discarded)
static int ensure_dense(vcfxg_ctx *c) {
    if (!c->dense_pending) return VCFXG_OK;
    c->dense_pending = false;
    const uint64_t L = c->n_lines;
    int r = ensure(c, c->line_end, 8 * (L + 1));
    if (!r) r = af_buffers(c, L);
    if (!r) r = ensure(c, c->af_meta, vcfxg::af_meta_bytes() * (L + 1));
    if (!r) r = ensure(c, c->scratch_small, 64);
    if (r) return r;
    HIPCHK(c, vcfxg::launch_walk_compact(c->dense_nw, c->dense_cap_w, P<uint64_t>(c->wk_offs), P<uint32_t>(c->wk_gt),
                                         P<uint64_t>(c->wk_le), P<int32_t>(c->wk_alt), P<int32_t>(c->wk_tot),
                                         P<uint32_t>(c->wk_rowpre), P<uint8_t>(c->wk_status), c->wk_meta.p,
                                         P<uint64_t>(c->line_end), P<int32_t>(c->alt), P<int32_t>(c->tot),
                                         P<uint32_t>(c->rowpre), P<uint8_t>(c->status), c->af_meta.p,
                                         P<uint64_t>(c->d_nlines), P<unsigned long long>(c->scratch_small),
                                         c->stream, nullptr, nullptr, P<uint64_t>(c->wk_bs)));
    return VCFXG_OK;
}

int vcfxg_allele_freq_region(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    if (c->af_path == 7) return note_schedule(c, "af_walk"), af_region_walk(c, data_start, mode, out);
    if (c->af_path == 8) return note_schedule(c, "af_two_sweep"), af_region_async(c, data_start, mode, out);
    if (c->af_path == 3) {  // synchronous two-sweep schedule: index + record kernels
        note_schedule(c, "af_two_sweep_sync");
        int r = vcfxg_index(c, data_start, nullptr);
        return r ? r : vcfxg_allele_freq(c, mode, out);
    }
    // records of >= 512 B on average (a GT-dense VCF): the walk schedule, no index sweep; the
    // GT-first walk for "GT:..." records (VCFXG_AF_GF_WALK=0: the index sweep + per-line sweep)
    if (c->hint_line >= 512 && c->hint_gt_only && !c->walk_overflowed)
        return note_schedule(c, "af_walk"), af_region_walk(c, data_start, mode, out);
    static const bool gf_ok = [] {
        const char *e = getenv("VCFXG_AF_GF_WALK");
        return !(e && e[0] == '0');
    }();
    if (gf_ok && c->hint_line >= 512 && c->hint_gt_first && !c->walk_overflowed)
        return note_schedule(c, "af_walk_gt_first"), af_region_walk(c, data_start, mode, out, true);
    return note_schedule(c, "af_two_sweep"), af_region_async(c, data_start, mode, out);
}

static int af_rows(vcfxg_ctx *c, int mode, vcfxg_summary *out) {
    const uint64_t L = c->n_lines;
    const char *buf = P<char>(c->input);
    const uint64_t *nl_dev = P<uint64_t>(c->d_nlines);
    int r;
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

int vcfxg_nonref_filter(vcfxg_ctx *c, int mode, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t L = c->n_lines;
    int r = ensure(c, c->status, L + 1);
    if (r) return r;
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    prof_begin(c, "nr_records");
    HIPCHK(c, vcfxg::launch_nr_records(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                       P<uint64_t>(c->d_nlines), L, mode, P<uint8_t>(c->status),
                                       P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "nr_records");
    static thread_local uint64_t host_cnt[4];
    HIPCHK(c, hipMemcpyAsync(host_cnt, c->counters.p, 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->text_bytes = 0;
    if (out) {
        out->n_lines = L;
        out->rows = host_cnt[0];
        out->data_lines = host_cnt[1];
        out->warn_lines = 0;
        out->general_records = host_cnt[3];
        out->text_bytes = 0;
    }
    return VCFXG_OK;
}

int vcfxg_genotype_query(vcfxg_ctx *c, const char *query, size_t qlen, int strict, int strip_cr, vcfxg_summary *out) {
    if (!c || (!query && qlen)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t L = c->n_lines;
    int r = ensure(c, c->status, L + 1);
    if (!r) r = ensure(c, c->query, qlen + 1);
    if (!r) r = ensure(c, c->af_meta, vcfxg::af_meta_bytes() * (L + 1));
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
                                       nullptr, c->af_meta.p));
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

// threshold_bounds memoised by the value's bits: the exact decimal expansion of a boundary
// (up to ~750 digits for the subnormal neighbours of 0.0, which every FILTER criterion asks
// for) cost tens of microseconds per call, paid again for every region call with the same
// criteria (a bounded per-thread table; the result is a pure function of the value)
static void cached_threshold_bounds(double t, vcfxg::ThresholdHost &out) {
    static thread_local std::map<uint64_t, vcfxg::ThresholdHost> memo;
    uint64_t key;
    std::memcpy(&key, &t, sizeof key);
    auto it = memo.find(key);
    if (it != memo.end()) {
        out = it->second;
        return;
    }
    vcfxg::threshold_bounds(t, out);
    if (memo.size() >= 64) memo.clear();
    memo.emplace(key, out);
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
        // FILTER and string INFO criteria never compare numbers: no boundary digits (they
        // would only lengthen the pool the filter walk keeps in registers)
        const bool cmp_num = h.target != vcfxg::RF_FILTER && (h.target != vcfxg::RF_INFO || h.numeric);
        cached_threshold_bounds(cmp_num && h.numeric ? h.value : 0.0, th);
        if (!cmp_num) th.lo.digits.clear(), th.hi.digits.clear();
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
    if (n && !(c->crit_dev_p == c->crit.p && c->crit_dev == c->crit_host)) {
        HIPCHK(c, hipMemcpyAsync(c->crit.p, c->crit_host.data(), c->crit_host.size(), hipMemcpyHostToDevice, c->stream));
        c->crit_dev = c->crit_host;
        c->crit_dev_p = c->crit.p;
    }
    if (!pool.empty() && !(c->pool_dev_p == c->pool.p && c->pool_dev == c->pool_host)) {
        HIPCHK(c, hipMemcpyAsync(c->pool.p, c->pool_host.data(), pool.size(), hipMemcpyHostToDevice, c->stream));
        c->pool_dev = c->pool_host;
        c->pool_dev_p = c->pool.p;
    }
    return VCFXG_OK;
}

static int run_rf(vcfxg_ctx *c, const vcfxg_criterion *crit, int n, int and_logic, int keep_cr = 0) {
    int r = ensure(c, c->status, c->n_lines + 1);
    if (!r) r = compile_criteria(c, crit, n);
    if (r) return r;
    prof_begin(c, "rf_records");
    HIPCHK(c, vcfxg::launch_rf_records(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                       P<uint64_t>(c->d_nlines), c->n_lines, P<vcfxg::RfCrit>(c->crit), n, and_logic,
                                       P<char>(c->pool), P<uint8_t>(c->status), P<unsigned long long>(c->counters),
                                       c->stream, keep_cr));
    prof_end(c, "rf_records");
    return VCFXG_OK;
}

int vcfxg_record_filter(vcfxg_ctx *c, const vcfxg_criterion *crit, int n, int and_logic, vcfxg_summary *out) {
    return vcfxg_record_filter_ex(c, crit, n, and_logic, 0, out);
}

int vcfxg_record_filter_ex(vcfxg_ctx *c, const vcfxg_criterion *crit, int n, int and_logic, int flags,
                           vcfxg_summary *out) {
    if (!c || n < 0 || (n && !crit) || (flags & ~VCFXG_RF_KEEP_CR)) return VCFXG_E_ARG;
    for (int k = 0; k < n; k++)
        if (crit[k].target < 0 || crit[k].target > vcfxg::RF_QUAL_LENIENT) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    int r = run_rf(c, crit, n, and_logic, (flags & VCFXG_RF_KEEP_CR) ? 1 : 0);
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
    DENSE(c);
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
    r = ensure(c, c->af_meta, vcfxg::af_meta_bytes() * (c->n_lines + 1));
    if (r) return r;
    prof_begin(c, "gq_records");
    HIPCHK(c, vcfxg::launch_gq_records(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                       P<uint64_t>(c->d_nlines), c->n_lines, 1, P<char>(c->query), (int)qlen, strict,
                                       qa, qb, P<uint8_t>(c->status), P<unsigned long long>(c->counters) + 4,
                                       c->stream, P<uint8_t>(c->status), c->af_meta.p));
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

// record_filter / genotype_query / the fused pipeline over the data region in one pass
// (vcfxg_fq_walk.hip): k_fq_walk reads each chunk's lines once (no separate index sweep), the
// walkers' regions are concatenated in file order (k_fq_compact), k_fq_finish filters the
// lines whose head did not fit the walk's window and counts, k_gq_complex takes the query's
// general lines; ONE host synchronisation reads the counters.  Short lines (the first lines
// average under 512 B), an earlier walk overflow on this input, or VCFXG_FQ_WALK=-1:
// vcfxg_index + the per-tool call, with identical results.
static int fq_region(vcfxg_ctx *c, size_t data_start, int what, const vcfxg_criterion *crit, int n, int and_logic,
                     const char *query, size_t qlen, int strict, int gq_strip_cr, vcfxg_summary *out) {
    if (!c || n < 0 || (n && !crit) || (!query && qlen)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    c->dense_pending = false;  // its own index replaces pending regions
    if (data_start > c->n) data_start = c->n;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n, C = c->walk_chunk;
    const int64_t nw = vcfxg::af_walkers(lo, hi, C);
    if (!nw || c->fq_path < 0 || c->walk_overflowed || (c->fq_path == 0 && c->hint_line < 512)) {
        note_schedule(c, "fq_two_sweep");
        int r = vcfxg_index(c, data_start, nullptr);
        if (r) return r;
        if (what == vcfxg::kFqRF) return vcfxg_record_filter(c, crit, n, and_logic, out);
        if (what == vcfxg::kFqGQ) return vcfxg_genotype_query(c, query, qlen, strict, gq_strip_cr, out);
        if (what == vcfxg::kFqNR) return vcfxg_nonref_filter(c, gq_strip_cr ? VCFXG_MODE_FILE : VCFXG_MODE_STDIN, out);
        return vcfxg_filter_query(c, crit, n, and_logic, query, qlen, strict, out);
    }
    note_schedule(c, "fq_walk");
    const bool nr = what == vcfxg::kFqNR;  // nonref_filter: the query's walk with its own reducer
    const bool rf = !nr && (what & vcfxg::kFqRF) != 0, gq = nr || (what & vcfxg::kFqGQ) != 0;
    const uint64_t cap_w = (uint64_t)(2 * C / std::max<int64_t>(c->hint_line, 64)) + 16;
    const uint64_t cap = (uint64_t)nw * cap_w;
    const size_t mb = vcfxg::af_meta_bytes();
    int r = ensure(c, c->wk_le, 8 * cap);
    if (!r) r = ensure(c, c->wk_status, cap);
    if (!r && gq) r = ensure(c, c->wk_meta, mb * cap);
    if (!r && rf) r = ensure(c, c->wk_tabs, 16 * cap);
    if (!r && rf) r = ensure(c, c->rf_tabs, 16 * (cap + 1));
    if (!r) r = ensure(c, c->wk_count, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_offs, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->fq_small, 128);
    if (!r) r = ensure(c, c->line_end, 8 * (cap + 1));
    if (!r) r = ensure(c, c->status, cap + 1);
    if (!r && gq) r = ensure(c, c->af_meta, mb * (cap + 1));
    if (!r && gq) r = ensure(c, c->query, qlen + 1);
    if (!r && rf) r = compile_criteria(c, crit, n);
    if (r) return r;
    int qa = -1, qb = -1;
    if (gq) {
        if (!strict) gq_parse_query(query, qlen, qa, qb);
        c->query_host.assign(query, qlen);
        if (qlen && !(c->query_dev_p == c->query.p && c->query_dev == c->query_host)) {
            HIPCHK(c, hipMemcpyAsync(c->query.p, c->query_host.data(), qlen, hipMemcpyHostToDevice, c->stream));
            c->query_dev = c->query_host;
            c->query_dev_p = c->query.p;
        }
    }
    const char *buf = P<char>(c->input);
    r = ensure_sum_host(c);
    if (r) return r;
    unsigned *ovf = P<unsigned>(c->fq_small);
    unsigned long long *cnt = P<unsigned long long>(c->fq_small) + 1;
    unsigned long long *gq_cnt = what == vcfxg::kFqBoth ? cnt + 4 : cnt;
    const int strip_cr = rf ? 1 : gq_strip_cr;  // the pipeline's query sees record_filter's output
    const int pool_len = (int)c->pool_host.size();
    const vcfxg::RfArgs ra{P<vcfxg::RfCrit>(c->crit), n, and_logic ? 1 : 0, P<char>(c->pool), pool_len};
    // (k_fq_done zeroed the slot and the counters after the last call; k_fq_walk zeroes
    // wk_count[nw], the scan's last entry)
    if (c->fq_small_dirty) HIPCHK(c, hipMemsetAsync(c->fq_small.p, 0, 128, c->stream));
    c->fq_small_dirty = true;  // until the call has synchronised
    prof_begin(c, "fq_walk");
    HIPCHK(c, vcfxg::launch_fq_walk(what, buf, lo, hi, C, strip_cr, c->hint_span, cap_w, ra, P<char>(c->query),
                                    (int)qlen, strict, qa, qb, P<uint64_t>(c->wk_le), P<uint8_t>(c->wk_status),
                                    c->wk_meta.p, c->wk_tabs.p, P<uint64_t>(c->wk_count), ovf, c->stream));
    prof_end(c, "fq_walk");
    prof_begin(c, "fq_rest");
    r = exclusive_scan(c, P<uint64_t>(c->wk_count), P<uint64_t>(c->wk_offs), (size_t)nw + 1);
    if (r) return r;
    HIPCHK(c, vcfxg::launch_fq_compact(what, nw, cap_w, P<uint64_t>(c->wk_offs), P<uint64_t>(c->wk_le),
                                       P<uint8_t>(c->wk_status), c->wk_meta.p, c->wk_tabs.p, P<uint64_t>(c->line_end),
                                       P<uint8_t>(c->status), c->af_meta.p, c->rf_tabs.p, P<uint64_t>(c->d_nlines),
                                       c->stream));
    if (nr)
        HIPCHK(c, vcfxg::launch_nr_complex(buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), cap,
                                           strip_cr ? VCFXG_MODE_FILE : VCFXG_MODE_STDIN, P<uint8_t>(c->status), cnt,
                                           c->stream));
    else
        // (a thread per line of the previous call, at most cap: the kernel grid-strides over the
        // device count, so fewer threads than lines is still exact)
        HIPCHK(c, vcfxg::launch_fq_finish(what, buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines),
                                          c->fq_lines_hint ? std::min<uint64_t>(cap, c->fq_lines_hint) : cap, ra,
                                          P<uint8_t>(c->status), c->af_meta.p, c->rf_tabs.p, cnt, gq_cnt, c->stream));
    if (gq && !nr)
        HIPCHK(c, vcfxg::launch_gq_complex(buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), cap, strip_cr,
                                           P<char>(c->query), (int)qlen, strict, qa, qb, c->af_meta.p,
                                           P<uint8_t>(c->status), gq_cnt,
                                           what == vcfxg::kFqBoth ? P<uint8_t>(c->status) : nullptr, c->stream));
    prof_end(c, "fq_rest");
    uint64_t *host = c->sum_host + 8;  // counters[0..7], lines, overflow (k_fq_done)
    HIPCHK(c, vcfxg::launch_fq_done(cnt, P<uint64_t>(c->d_nlines), P<uint64_t>(c->fq_small), c->sum_dev + 8, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->fq_small_dirty = false;
    c->fq_lines_hint = host[8];
    prof_collect(c);
    if (host[9]) {  // a walker ran out of line slots (short lines): index + the per-tool kernels
        c->walk_overflowed = true;
        return fq_region(c, data_start, what, crit, n, and_logic, query, qlen, strict, gq_strip_cr, out);
    }
    c->data_start = data_start;
    c->n_lines = host[8];
    c->indexed = true;
    c->text_bytes = 0;
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = host[8];
        if (what == vcfxg::kFqBoth) {
            out->rows = host[4];        // kept by both stages
            out->data_lines = host[0];  // kept by record_filter
            out->warn_lines = host[6];
            out->general_records = host[7];
        } else {
            out->rows = host[0];
            out->data_lines = host[1];
            if (nr) out->general_records = host[3];
            else if (gq) {
                out->warn_lines = host[2];
                out->general_records = host[3];
            }
        }
    }
    return VCFXG_OK;
}

int vcfxg_record_filter_region(vcfxg_ctx *c, size_t data_start, const vcfxg_criterion *crit, int n, int and_logic,
                               vcfxg_summary *out) {
    return fq_region(c, data_start, vcfxg::kFqRF, crit, n, and_logic, nullptr, 0, 0, 0, out);
}

int vcfxg_genotype_query_region(vcfxg_ctx *c, size_t data_start, const char *query, size_t qlen, int strict,
                                int strip_cr, vcfxg_summary *out) {
    return fq_region(c, data_start, vcfxg::kFqGQ, nullptr, 0, 0, query, qlen, strict, strip_cr, out);
}

int vcfxg_filter_query_region(vcfxg_ctx *c, size_t data_start, const vcfxg_criterion *crit, int n, int and_logic,
                              const char *query, size_t qlen, int strict, vcfxg_summary *out) {
    return fq_region(c, data_start, vcfxg::kFqBoth, crit, n, and_logic, query, qlen, strict, 1, out);
}
int vcfxg_nonref_filter_region(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out) {
    if (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN) return VCFXG_E_ARG;
    return fq_region(c, data_start, vcfxg::kFqNR, nullptr, 0, 0, "", 0, 0, mode == VCFXG_MODE_FILE ? 1 : 0, out);
}

// VCFX_hwe_tester over [data_start, n).  walk: the AF walk with the HWE reducer (records of
// >= 512 B on average), its compaction and k_hwe_lines for the lines it left; else the line
// index and k_hwe_lines on every line.  Then the row rules + lengths, the scan, the rows into
// the previous call's text capacity and ONE host synchronisation (as af_region_walk); rows
// past the capacity are formatted again once it has grown.  A walker over its line capacity
// reruns the call without the walk.
static int hwe_region_impl(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out, bool walk) {
    if (c) c->dense_pending = false;  // a new index / regions replace the pending ones
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n;
    const int64_t C = c->walk_chunk;
    const int64_t nw = walk ? vcfxg::af_walkers(lo, hi, C) : 0;
    walk = walk && nw > 0;
    const char *buf = P<char>(c->input);
    int r = ensure(c, c->wk_small, 128);
    if (r) return r;
    uint64_t *small = P<uint64_t>(c->wk_small);  // [0] overflow flag, [4..10] summary, [11] rechecks
    unsigned *ovf = reinterpret_cast<unsigned *>(small);
    uint64_t cap = 0;
    if (walk) {
        const uint64_t cap_w = (uint64_t)(2 * C / std::max<int64_t>(c->hint_line, 64)) + 16;
        cap = (uint64_t)nw * cap_w;
        r = ensure(c, c->wk_le, 8 * cap);
        if (!r) r = ensure(c, c->wk_alt, 4 * cap);
        if (!r) r = ensure(c, c->wk_tot, 4 * cap);
        if (!r) r = ensure(c, c->wk_aux, 4 * cap);
        if (!r) r = ensure(c, c->wk_rowpre, 4 * cap);
        if (!r) r = ensure(c, c->wk_status, cap);
        if (!r) r = ensure(c, c->wk_meta, vcfxg::af_meta_bytes() * cap);
        if (!r) r = ensure(c, c->wk_count, 8 * (size_t)(nw + 1));
        if (!r) r = ensure(c, c->wk_offs, 8 * (size_t)(nw + 1));
        if (!r) r = ensure(c, c->wk_gt, 4 * (size_t)nw);
        if (!r) r = ensure(c, c->line_end, 8 * (cap + 1));
        if (!r) r = af_buffers(c, cap);
        if (!r) r = ensure(c, c->hwe_aux, 4 * (cap + 1));
        if (!r) r = ensure(c, c->af_meta, vcfxg::af_meta_bytes() * (cap + 1));
        if (!r) r = ensure(c, c->hwe_rc, sizeof(vcfxg_hwe_recheck) * (cap + 1));
        if (r) return r;
        HIPCHK(c, hipMemsetAsync(small, 0, 96, c->stream));
        HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->wk_count) + nw, 0, 8, c->stream));
        prof_begin(c, "hwe_walk");
        // mode 0: both HWE modes strip the trailing '\r' before the record is parsed
        HIPCHK(c, vcfxg::launch_af_walk(buf, lo, hi, C, 0, c->hint_span, cap_w, P<uint64_t>(c->wk_le),
                                        P<int32_t>(c->wk_alt), P<int32_t>(c->wk_tot), P<uint32_t>(c->wk_rowpre),
                                        P<uint8_t>(c->wk_status), c->wk_meta.p, P<uint64_t>(c->wk_count),
                                        P<uint32_t>(c->wk_gt), ovf, c->stream, P<int32_t>(c->wk_aux)));
        prof_end(c, "hwe_walk");
        prof_begin(c, "walk_compact");
        r = exclusive_scan(c, P<uint64_t>(c->wk_count), P<uint64_t>(c->wk_offs), (size_t)nw + 1);
        if (r) return r;
        HIPCHK(c, vcfxg::launch_walk_compact(nw, cap_w, P<uint64_t>(c->wk_offs), P<uint32_t>(c->wk_gt),
                                             P<uint64_t>(c->wk_le), P<int32_t>(c->wk_alt), P<int32_t>(c->wk_tot),
                                             P<uint32_t>(c->wk_rowpre), P<uint8_t>(c->wk_status), c->wk_meta.p,
                                             P<uint64_t>(c->line_end), P<int32_t>(c->alt), P<int32_t>(c->tot),
                                             P<uint32_t>(c->rowpre), P<uint8_t>(c->status), c->af_meta.p,
                                             P<uint64_t>(c->d_nlines), P<unsigned long long>(c->counters), c->stream,
                                             P<int32_t>(c->wk_aux), P<int32_t>(c->hwe_aux)));
        prof_end(c, "walk_compact");
    } else {
        uint64_t L = 0;
        r = vcfxg_index(c, data_start, &L);
        if (r) return r;
        cap = L;
        r = af_buffers(c, cap);
        if (!r) r = ensure(c, c->hwe_aux, 4 * (cap + 1));
        if (!r) r = ensure(c, c->hwe_rc, sizeof(vcfxg_hwe_recheck) * (cap + 1));
        if (r) return r;
        HIPCHK(c, hipMemsetAsync(small, 0, 96, c->stream));
    }
    // (the walk's compaction counts GT lines for AF in counters[0..1]: rows are counted below)
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    prof_begin(c, "hwe_lines");
    HIPCHK(c, vcfxg::launch_hwe_lines(buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), cap, mode,
                                      walk ? c->af_meta.p : nullptr, P<int32_t>(c->alt), P<int32_t>(c->tot),
                                      P<int32_t>(c->hwe_aux), P<uint32_t>(c->rowpre), P<uint8_t>(c->status),
                                      P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "hwe_lines");
    prof_begin(c, "hwe_rows");
    HIPCHK(c, vcfxg::launch_hwe_rowlen(P<uint64_t>(c->d_nlines), cap, mode, walk ? c->af_meta.p : nullptr,
                                       P<uint32_t>(c->rowpre), P<uint8_t>(c->status), P<uint64_t>(c->rowlen),
                                       P<unsigned long long>(c->counters), c->stream));
    r = exclusive_scan(c, P<uint64_t>(c->rowlen), P<uint64_t>(c->rowoff), (size_t)cap + 1);
    if (r) return r;
    HIPCHK(c, vcfxg::launch_af_summary(P<uint64_t>(c->d_nlines), P<uint64_t>(c->rowoff),
                                       P<unsigned long long>(c->counters), ovf, small + 4, c->stream));
    prof_end(c, "hwe_rows");
    const uint64_t tcap = std::max<uint64_t>(c->text_hint, 1u << 16);
    r = ensure(c, c->text, tcap + 1);
    if (r) return r;
    unsigned long long *rc_n = reinterpret_cast<unsigned long long *>(small + 11);
    prof_begin(c, "hwe_format");
    HIPCHK(c, vcfxg::launch_hwe_format(buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), cap, mode,
                                       P<int32_t>(c->alt), P<int32_t>(c->tot), P<int32_t>(c->hwe_aux),
                                       P<uint32_t>(c->rowpre), P<uint8_t>(c->status), P<uint64_t>(c->rowoff),
                                       P<char>(c->text), tcap, c->hwe_ulps, c->hwe_rc.p, rc_n, cap + 1, c->stream));
    prof_end(c, "hwe_format");
    static thread_local uint64_t sm[8];
    HIPCHK(c, hipMemcpyAsync(sm, small + 4, sizeof sm, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (walk && sm[6]) {  // a walker ran out of line slots (short lines): no walk
        prof_collect(c);
        c->walk_overflowed = true;
        return hwe_region_impl(c, data_start, mode, out, false);
    }
    const uint64_t L = sm[0], text = sm[1];
    c->text_hint = text;
    if (text > tcap) {  // the text outgrew the previous capacity: all rows again
        r = ensure(c, c->text, text + 1);
        if (r) return r;
        HIPCHK(c, hipMemsetAsync(rc_n, 0, 8, c->stream));
        prof_begin(c, "hwe_format");
        HIPCHK(c, vcfxg::launch_hwe_format(buf, lo, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), L, mode,
                                           P<int32_t>(c->alt), P<int32_t>(c->tot), P<int32_t>(c->hwe_aux),
                                           P<uint32_t>(c->rowpre), P<uint8_t>(c->status), P<uint64_t>(c->rowoff),
                                           P<char>(c->text), ~0ull, c->hwe_ulps, c->hwe_rc.p, rc_n, cap + 1,
                                           c->stream));
        prof_end(c, "hwe_format");
        HIPCHK(c, hipMemcpyAsync(&sm[7], rc_n, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    prof_collect(c);
    c->data_start = data_start;
    c->n_lines = L;
    c->indexed = true;
    c->text_bytes = text;
    c->hwe_rc_n = sm[7];
    if (out) {
        out->n_lines = L;
        out->rows = sm[2];
        out->data_lines = 0;
        out->warn_lines = 0;
        out->general_records = sm[5];
        out->text_bytes = text;
    }
    return VCFXG_OK;
}

int vcfxg_hwe_region(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    // the AF schedule knob selects here too: 3 / 8 = no walk, 7 = the walk
    const bool walk = c->af_path == 7 || (c->af_path != 3 && c->af_path != 8 && c->hint_line >= 512 && c->hint_gt_only &&
                                          !c->walk_overflowed);
    return hwe_region_impl(c, data_start, mode, out, walk);
}

int vcfxg_hwe_rechecks(vcfxg_ctx *c, vcfxg_hwe_recheck *out, uint64_t cap, uint64_t *n) {
    if (!c || !n || (!out && cap)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    *n = c->hwe_rc_n;
    const uint64_t k = std::min(cap, c->hwe_rc_n);
    if (!k) return VCFXG_OK;
    HIPCHK(c, hipMemcpyAsync(out, c->hwe_rc.p, k * sizeof(vcfxg_hwe_recheck), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

// the dosage walk: line ends + per fixed-stride record its samples / "NA" samples, compacted to
// the dense per-line arrays (line_end, alt = ns, tot = na, status, af_meta = LineMeta); the
// context is indexed afterwards.  *overflow: a walker ran out of line slots (short lines)
static int dose_walk_index(vcfxg_ctx *c, size_t data_start, int mode, uint64_t *L_out, bool *overflow,
                           bool head) {
    c->dense_pending = false;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n;
    const int64_t C = c->walk_chunk;
    const int64_t nw = vcfxg::af_walkers(lo, hi, C);
    const uint64_t cap_w = (uint64_t)(2 * C / std::max<int64_t>(c->hint_line, 64)) + 16;
    if (cap_w > 0xFFFF) {  // (the walk's 16-bit GT-line count): the caller's index path
        c->walk_overflowed = true;
        *overflow = true;
        return VCFXG_OK;
    }
    const uint64_t cap = (uint64_t)nw * cap_w;
    int r = ensure(c, c->wk_le, 8 * cap);
    if (!r) r = ensure(c, c->wk_alt, 4 * cap);
    if (!r) r = ensure(c, c->wk_tot, 4 * cap);
    if (!r) r = ensure(c, c->wk_rowpre, 4 * cap);
    if (!r) r = ensure(c, c->wk_status, cap);
    if (!r) r = ensure(c, c->wk_meta, vcfxg::af_meta_bytes() * cap);
    if (!r) r = ensure(c, c->wk_count, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_offs, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_gt, 4 * (size_t)nw);
    if (!r) r = ensure(c, c->wk_small, 128);
    if (!r) r = ensure(c, c->line_end, 8 * (cap + 1));
    if (!r) r = af_buffers(c, cap);
    if (!r) r = ensure(c, c->af_meta, vcfxg::af_meta_bytes() * (cap + 1));
    if (r) return r;
    const char *buf = P<char>(c->input);
    uint64_t *small = P<uint64_t>(c->wk_small);
    HIPCHK(c, hipMemsetAsync(small, 0, 16, c->stream));
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->wk_count) + nw, 0, 8, c->stream));
    prof_begin(c, "dose_walk");
    HIPCHK(c, vcfxg::launch_af_walk(buf, lo, hi, C, mode, c->hint_span, cap_w, P<uint64_t>(c->wk_le),
                                    P<int32_t>(c->wk_alt), P<int32_t>(c->wk_tot), P<uint32_t>(c->wk_rowpre),
                                    P<uint8_t>(c->wk_status), c->wk_meta.p, P<uint64_t>(c->wk_count),
                                    P<uint32_t>(c->wk_gt), reinterpret_cast<unsigned *>(small), c->stream, nullptr,
                                    nullptr, true, false, head));
    prof_end(c, "dose_walk");
    prof_begin(c, "walk_compact");
    r = exclusive_scan(c, P<uint64_t>(c->wk_count), P<uint64_t>(c->wk_offs), (size_t)nw + 1);
    if (r) return r;
    HIPCHK(c, vcfxg::launch_walk_compact(nw, cap_w, P<uint64_t>(c->wk_offs), P<uint32_t>(c->wk_gt),
                                         P<uint64_t>(c->wk_le), P<int32_t>(c->wk_alt), P<int32_t>(c->wk_tot),
                                         P<uint32_t>(c->wk_rowpre), P<uint8_t>(c->wk_status), c->wk_meta.p,
                                         P<uint64_t>(c->line_end), P<int32_t>(c->alt), P<int32_t>(c->tot),
                                         P<uint32_t>(c->rowpre), P<uint8_t>(c->status), c->af_meta.p,
                                         P<uint64_t>(c->d_nlines), P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "walk_compact");
    static thread_local uint64_t h[2];  // overflow flag, lines
    HIPCHK(c, hipMemcpyAsync(&h[0], small, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&h[1], c->d_nlines.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *overflow = (h[0] & 0xFFFFFFFFull) != 0;
    if (*overflow) {
        c->walk_overflowed = true;
        return VCFXG_OK;
    }
    c->data_start = data_start;
    c->n_lines = h[1];
    c->indexed = true;
    *L_out = h[1];
    return VCFXG_OK;
}

// VCFX_dosage_calculator over [data_start, n): the line index, the row lengths, a scan, the
// rows (one host synchronisation for the text size).  Records of >= 512 B (a GT-dense VCF): the
// walk reads each record once for its line end and (fixed-stride records) its samples and "NA"
// samples -- no index sweep, no row-length pass over the records; the other lines take the
// exact row-length pass; VCFXG_DOSE_WALK=0 keeps the index + two-pass schedule
//
// On such input the first attempt is the HEAD walk (DoseHeadOp): a GT-only record whose '\n' is
// where the previous fixed-stride record predicts it is taken as a fixed-stride row without
// "NA" and its samples are not read by the walk -- only the record heads are -- so the input is
// read about once in all (by k_dose_fmt, which checks every sample byte of those rows while it
// writes them).  A row that fails the check (an "NA", a wider sample, ...) flags the call,
// which is then redone with the sweeping walk; an input that failed once keeps the sweeping
// walk until the next load.  VCFXG_DOSE_HEAD=0 always sweeps.
static int dose_walk_index(vcfxg_ctx *c, size_t data_start, int mode, uint64_t *L_out, bool *overflow, bool head);
static int dosage_region_once(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out, bool head, bool *redo);

int vcfxg_dosage_region(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    static const bool head_ok = [] {
        const char *e = getenv("VCFXG_DOSE_HEAD");
        return !(e && e[0] == '0');
    }();
    bool redo = false;
    int r = dosage_region_once(c, data_start, mode, out, head_ok && !c->dose_head_failed, &redo);
    if (r || !redo) return r;
    c->dose_head_failed = true;
    return dosage_region_once(c, data_start, mode, out, false, &redo);
}

static int dosage_region_once(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out, bool head, bool *redo) {
    static const bool walk_ok = [] {
        const char *e = getenv("VCFXG_DOSE_WALK");
        return !(e && e[0] == '0');
    }();
    const bool walk = walk_ok && c->af_path != 3 && c->af_path != 8 && c->hint_line >= 512 && c->hint_gt_only &&
                      !c->walk_overflowed && vcfxg::af_walkers((int64_t)data_start, (int64_t)c->n, c->walk_chunk) > 0;
    uint64_t L = 0;
    int r;
    bool walked = false;
    head = head && walk;
    if (walk) {
        bool ovf = false;
        r = dose_walk_index(c, data_start, mode, &L, &ovf, head);
        if (r) return r;
        walked = !ovf;
    }
    head = head && walked;
    if (!walked) {
        r = vcfxg_index(c, data_start, &L);
        if (r) return r;
    }
    HIPCHK(c, hipSetDevice(c->device));
    r = af_buffers(c, L);
    if (!r) r = ensure(c, c->dose_meta, vcfxg::dose_meta_bytes() * (L + 1));
    if (r) return r;
    const char *buf = P<char>(c->input);
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->rowlen) + L, 0, 8, c->stream));
    prof_begin(c, "dose_len");
    if (walked)
        HIPCHK(c, vcfxg::launch_dose_from_walk(P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), L, c->af_meta.p,
                                               P<int32_t>(c->alt), P<int32_t>(c->tot), P<uint8_t>(c->status),
                                               P<uint64_t>(c->rowlen), c->dose_meta.p,
                                               P<unsigned long long>(c->counters), c->stream));
    HIPCHK(c, vcfxg::launch_dose_len(buf, (int64_t)data_start, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), L,
                                     mode, P<uint8_t>(c->status), P<uint64_t>(c->rowlen), c->dose_meta.p,
                                     P<unsigned long long>(c->counters), c->stream, walked));
    prof_end(c, "dose_len");
    prof_begin(c, "dose_rows");
    r = exclusive_scan(c, P<uint64_t>(c->rowlen), P<uint64_t>(c->rowoff), (size_t)L + 1);
    if (r) return r;
    prof_end(c, "dose_rows");
    static thread_local uint64_t tail[6];
    HIPCHK(c, hipMemcpyAsync(&tail[0], P<uint64_t>(c->rowoff) + L, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&tail[1], c->counters.p, 40, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t text = tail[0];
    r = ensure(c, c->text, text + 1);
    if (r) return r;
    // (the head walk's rows are checked by the formatting pass: a failed check flags the call)
    unsigned *bad = head ? reinterpret_cast<unsigned *>(P<uint64_t>(c->wk_small) + 4) : nullptr;
    static thread_local unsigned bad_h;
    bad_h = 0;
    if (bad) HIPCHK(c, hipMemsetAsync(bad, 0, 4, c->stream));
    prof_begin(c, "dose_fmt");
    HIPCHK(c, vcfxg::launch_dose_fmt(buf, (int64_t)data_start, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), L,
                                     P<uint8_t>(c->status), c->dose_meta.p, P<uint64_t>(c->rowoff), P<char>(c->text),
                                     ~0ull, tail[2], c->stream, bad, tail[5]));
    prof_end(c, "dose_fmt");
    if (bad) HIPCHK(c, hipMemcpyAsync(&bad_h, bad, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    if (bad_h) {  // some row the head walk took is not a fixed-stride row without "NA": redo
        *redo = true;
        c->text_bytes = 0;
        return VCFXG_OK;
    }
    c->text_bytes = text;
    if (out) {
        out->n_lines = L;
        out->rows = tail[1];
        out->data_lines = tail[1] + tail[3];
        out->warn_lines = tail[3];
        out->general_records = tail[4];
        out->text_bytes = text;
    }
    return VCFXG_OK;
}

// VCFX_allele_counter over indexed lines [l0, l1): row bytes, a scan, the rows (one host
// synchronisation for the text size)
int vcfxg_allele_counter(vcfxg_ctx *c, uint64_t l0, uint64_t l1, const vcfxg_ac_params *p, vcfxg_summary *out) {
    if (!c || !p || (p->m && (!p->sample || !p->name_off)) || p->kind < 0 || p->kind > 2 || p->m >= (1ull << 31))
        return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    if (l0 > l1 || l1 > c->n_lines) return VCFXG_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t m = p->m, n = l1 - l0, L = c->n_lines;
    // slot i reads eff[i]: the selection itself, or (seq) its running maximum
    c->ac_eff_host.resize(m + 1);
    c->ac_noff_host.assign(p->name_off, p->name_off + m + 1);
    uint32_t run = 0, mx = 0;
    for (uint64_t i = 0; i < m; i++) {
        run = p->seq ? std::max(run, p->sample[i]) : p->sample[i];
        c->ac_eff_host[i] = run;
        mx = std::max(mx, run);
    }
    const uint64_t nb = p->name_off[m] - p->name_off[0];
    if (p->name_off[0] != 0) return VCFXG_E_ARG;
    c->ac_names_host.assign(p->names ? p->names : "", (size_t)nb);
    const uint64_t scap = (uint64_t)mx + 1;
    // the selection in k_ac_fmt's LDS when it fits in 40 KiB (the sample indices, 32-bit name
    // offsets and the names); VCFXG_AC_SEL_GLOBAL=1 keeps it in global memory (test hook)
    // an identity selection (slot i reads sample i: every sample, in order) keeps no index array
    bool ident = true;
    for (uint64_t i = 0; i < m && ident; i++) ident = c->ac_eff_host[i] == i;
    const uint64_t sel_bytes = (((ident ? 0 : 4 * m) + 4 * (m + 1) + (p->name_off[m] - p->name_off[0]) + 15) / 16) * 16;
    const uint32_t sel_lds = sel_bytes <= 40960 && !getenv("VCFXG_AC_SEL_GLOBAL") ? (uint32_t)sel_bytes : 0u;
    // text rows under a selection whose names share one length L <= 11: k_ac_rows writes the
    // fixed-stride records straight from registers (vcfxg_ac.hip); VCFXG_AC_DIRECT=0 keeps every
    // record on k_ac_fmt's LDS image (A/B and test hook)
    static const bool direct_env = [] {
        const char *e = getenv("VCFXG_AC_DIRECT");
        return !(e && e[0] == '0');
    }();
    const uint64_t L0 = m ? p->name_off[1] - p->name_off[0] : 0;
    bool direct = direct_env && p->kind == 0 && m > 0 && m <= 4096 && L0 <= 11 &&
                  vcfxg::ac_rows_lds((uint32_t)m, ident ? 1 : 0) <= vcfxg::ac_rows_lds_max();
    for (uint64_t i = 0; i < m && direct; i++) direct = p->name_off[i + 1] - p->name_off[i] == L0;
    if (direct) {
        c->ac_etab_host.assign(16 * m, 0);
        for (uint64_t i = 0; i < m; i++) {
            uint8_t *e = &c->ac_etab_host[16 * i];
            std::memcpy(e + 11 - L0, c->ac_names_host.data() + p->name_off[i], (size_t)L0);
            std::memcpy(e + 11, "\t0\t0\n", 5);
        }
    }
    // grid: a wave per line up to 2048 blocks, and at most 1 GiB of per-wave sample tables
    const uint64_t waves_per_block = (uint64_t)(vcfxg::ac_threads() / 64);
    uint64_t blocks = std::min<uint64_t>((n + waves_per_block - 1) / waves_per_block, 2048);
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, (1ull << 30) / (4 * scap * waves_per_block)));
    int r = ensure(c, c->ac_eff, 4 * (m + 1));
    if (!r) r = ensure(c, c->ac_noff, 8 * (m + 1));
    if (!r) r = ensure(c, c->ac_names, nb + 1);
    if (!r) r = ensure(c, c->ac_scratch, 4 * scap * waves_per_block * blocks);
    if (!r && direct) {
        // the entries and k_ac_nib's counts for k_ac_rows (n x ceil(m / 64) x 32 B); without room
        // for them every record takes k_ac_fmt
        int rd = ensure(c, c->ac_etab, 16 * m);
        if (!rd) rd = ensure(c, c->ac_nib, n * ((m + 63) / 64) * 32);
        if (rd == VCFXG_E_NOMEM) {
            (void)hipGetLastError();  // (a failed hipMalloc leaves its error to be read once)
            c->err.clear();
            direct = false;
        } else
            r = rd;
    }
    if (!r) r = af_buffers(c, L);
    if (!r) r = ensure(c, c->af_meta, vcfxg::ac_meta_bytes() * (L + 1));
    if (r) return r;
    HIPCHK(c, hipMemcpyAsync(c->ac_eff.p, c->ac_eff_host.data(), 4 * (m + 1), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->ac_noff.p, c->ac_noff_host.data(), 8 * (m + 1), hipMemcpyHostToDevice, c->stream));
    if (nb) HIPCHK(c, hipMemcpyAsync(c->ac_names.p, c->ac_names_host.data(), nb, hipMemcpyHostToDevice, c->stream));
    if (direct)
        HIPCHK(c, hipMemcpyAsync(c->ac_etab.p, c->ac_etab_host.data(), 16 * m, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->rowlen) + n, 0, 8, c->stream));
    const char *buf = P<char>(c->input);
    prof_begin(c, "ac_len");
    HIPCHK(c, vcfxg::launch_ac_len(buf, (int64_t)c->data_start, P<uint64_t>(c->line_end), l0, l1, (unsigned)blocks,
                                   P<uint32_t>(c->ac_eff), P<uint64_t>(c->ac_noff), P<char>(c->ac_names),
                                   P<uint32_t>(c->ac_scratch), (uint32_t)m, (uint32_t)scap, p->seq, p->kind,
                                   ident ? 1 : 0, direct ? 1 : 0, direct ? P<uint32_t>(c->ac_nib) : nullptr,
                                   P<uint8_t>(c->status), P<uint64_t>(c->rowlen), c->af_meta.p,
                                   P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "ac_len");
    r = exclusive_scan(c, P<uint64_t>(c->rowlen), P<uint64_t>(c->rowoff), (size_t)n + 1);
    if (r) return r;
    static thread_local uint64_t tail[6];
    HIPCHK(c, hipMemcpyAsync(&tail[0], P<uint64_t>(c->rowoff) + n, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&tail[1], c->counters.p, 40, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t text = tail[0];
    r = ensure(c, c->text, text + 1);
    if (r) return r;
    prof_begin(c, "ac_fmt");
    if (direct) {
        const uint64_t rw = (uint64_t)(vcfxg::ac_rows_threads() / 64);
        const unsigned rb = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + rw - 1) / rw, 1024));
        HIPCHK(c, vcfxg::launch_ac_rows(buf, (int64_t)c->data_start, P<uint64_t>(c->line_end), l0, l1, rb,
                                        P<uint32_t>(c->ac_eff), (uint32_t)m, ident ? 1 : 0, c->ac_etab.p, (uint32_t)L0,
                                        P<uint32_t>(c->ac_nib), c->af_meta.p, P<uint64_t>(c->rowoff), P<char>(c->text),
                                        c->stream));
    }
    if (!direct || tail[5])  // (the records k_ac_rows does not take)
        HIPCHK(c, vcfxg::launch_ac_fmt(buf, (int64_t)c->data_start, P<uint64_t>(c->line_end), l0, l1, (unsigned)blocks,
                                       P<uint32_t>(c->ac_eff), P<uint64_t>(c->ac_noff), P<char>(c->ac_names),
                                       P<uint32_t>(c->ac_scratch), (uint32_t)m, (uint32_t)scap, p->seq, p->kind, sel_lds,
                                       ident ? 1 : 0, direct ? 1 : 0, P<uint8_t>(c->status), c->af_meta.p,
                                       P<uint64_t>(c->rowoff), P<char>(c->text), c->stream));
    prof_end(c, "ac_fmt");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->text_bytes = text;
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = n;
        out->rows = tail[1];
        out->data_lines = tail[2];
        out->warn_lines = tail[3];
        out->general_records = tail[4];
        out->text_bytes = text;
    }
    return VCFXG_OK;
}

// VCFX_haplotype_phaser over [data_start, n): index, the per-line parse into genotype rows, the
// variant compaction (one host synchronisation for the variant count), the pair pass, a scan
// and the entries (a second synchronisation)
// VCFX_haplotype_phaser.  Records of >= 512 B, GT-only (a GT-dense VCF): the line index comes
// from the dosage HEAD walk (record heads only; a GT-only record whose '\n' is where the
// previous fixed-stride record predicts it is taken unswept), and k_ph_lines' fixed-stride
// sweep, which reads every record anyway, validates the unswept records' interiors; a record it
// cannot validate flags the call, which is redone on vcfxg_index (and this input keeps the
// index).  VCFXG_PH_WALK=0: always the index.
static int phaser_once(vcfxg_ctx *c, size_t data_start, int mode, double thr, uint32_t hint, vcfxg_summary *out,
                       bool walk, bool *redo);

int vcfxg_haplotype_phaser(vcfxg_ctx *c, size_t data_start, int mode, double thr, uint32_t hint, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    static const bool walk_ok = [] {
        const char *e = getenv("VCFXG_PH_WALK");
        return !(e && e[0] == '0');
    }();
    const bool walk = walk_ok && !c->ph_head_failed && c->af_path != 3 && c->af_path != 8 && c->hint_line >= 512 &&
                      c->hint_gt_only && !c->walk_overflowed &&
                      vcfxg::af_walkers((int64_t)data_start, (int64_t)c->n, c->walk_chunk) > 0;
    bool redo = false;
    int r = phaser_once(c, data_start, mode, thr, hint, out, walk, &redo);
    if (r || !redo) return r;
    c->ph_head_failed = true;
    return phaser_once(c, data_start, mode, thr, hint, out, false, &redo);
}

static int phaser_once(vcfxg_ctx *c, size_t data_start, int mode, double thr, uint32_t hint, vcfxg_summary *out,
                       bool walk, bool *redo) {
    *redo = false;
    uint64_t L = 0;
    int r;
    bool walked = false;
    if (walk) {
        bool ovf = false;
        note_schedule(c, "ph_head_walk");
        r = dose_walk_index(c, data_start, mode, &L, &ovf, true);
        if (r) return r;
        walked = !ovf;
    }
    if (!walked) {
        note_schedule(c, "ph_index");
        r = vcfxg_index(c, data_start, &L);
        if (r) return r;
    }
    HIPCHK(c, hipSetDevice(c->device));
    unsigned *bad = walked ? reinterpret_cast<unsigned *>(P<uint64_t>(c->wk_small) + 4) : nullptr;
    const char *buf = P<char>(c->input);
    uint64_t kpad = ((uint64_t)std::max<uint32_t>(hint, 16) + 15) & ~15ull;
    static thread_local uint64_t h[2];
    for (int pass = 0;; pass++) {
        r = ensure(c, c->ph_G, L * kpad + 16);
        if (!r) r = af_buffers(c, L);
        if (!r) r = ensure(c, c->ph_isvar, 4 * (L + 1));
        if (!r) r = ensure(c, c->ph_info, vcfxg::ph_line_bytes() * (L + 1));
        if (!r) r = ensure(c, c->ph_vnum, 8 * (L + 1));
        if (!r) r = ensure(c, c->ph_vline, 8 * (L + 1));
        if (r) return r;
        HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
        HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->counters) + 4, 0, 8, c->stream));
        if (bad) HIPCHK(c, hipMemsetAsync(bad, 0, 4, c->stream));
        prof_begin(c, "ph_lines");
        HIPCHK(c, vcfxg::launch_ph_lines(buf, (int64_t)data_start, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), L,
                                         mode, (uint32_t)kpad, P<int8_t>(c->ph_G), P<uint8_t>(c->status),
                                         P<uint32_t>(c->ph_isvar), c->ph_info.p, P<unsigned long long>(c->counters),
                                         c->stream, walked ? c->af_meta.p : nullptr, bad));
        prof_end(c, "ph_lines");
        if (L) {
            r = exclusive_scan(c, P<uint32_t>(c->ph_isvar), P<uint64_t>(c->ph_vnum), (size_t)L);
            if (r) return r;
            HIPCHK(c, vcfxg::launch_ph_compact(P<uint32_t>(c->ph_isvar), P<uint64_t>(c->ph_vnum), P<uint64_t>(c->d_nlines),
                                               L, P<uint64_t>(c->ph_vline), P<uint64_t>(c->counters) + 4, c->stream));
        }
        HIPCHK(c, hipMemcpyAsync(h, P<uint64_t>(c->counters) + 3, 16, hipMemcpyDeviceToHost, c->stream));
        static thread_local unsigned bad_h;
        bad_h = 0;
        if (bad) HIPCHK(c, hipMemcpyAsync(&bad_h, bad, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (bad_h) {  // an unswept record the parse could not validate: the call again on the index
            *redo = true;
            return VCFXG_OK;
        }
        if (h[0] > kpad && pass == 0) {  // a record wider than the rows: once more with rows that fit
            kpad = (h[0] + 15) & ~15ull;
            continue;
        }
        break;
    }
    const uint64_t V = h[1];
    r = ensure(c, c->ph_flags, V + 1);
    if (!r) r = ensure(c, c->ph_r2, 8 * (V + 1));
    if (!r) r = ensure(c, c->rowlen, 8 * (V + 1));
    if (!r) r = ensure(c, c->rowoff, 8 * (V + 1));
    if (r) return r;
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->rowlen) + V, 0, 8, c->stream));
    prof_begin(c, "ph_pairs");
    HIPCHK(c, vcfxg::launch_ph_pairs(buf, P<uint64_t>(c->ph_vline), P<uint64_t>(c->counters) + 4, V, c->ph_info.p,
                                     P<int8_t>(c->ph_G), (uint32_t)kpad, thr, P<uint8_t>(c->ph_flags),
                                     P<uint64_t>(c->rowlen), P<double>(c->ph_r2), c->stream));
    prof_end(c, "ph_pairs");
    r = exclusive_scan(c, P<uint64_t>(c->rowlen), P<uint64_t>(c->rowoff), (size_t)V + 1);
    if (r) return r;
    static thread_local uint64_t text;
    HIPCHK(c, hipMemcpyAsync(&text, P<uint64_t>(c->rowoff) + V, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    r = ensure(c, c->text, text + 1);
    if (r) return r;
    prof_begin(c, "ph_fmt");
    HIPCHK(c, vcfxg::launch_ph_fmt(buf, P<uint64_t>(c->ph_vline), P<uint64_t>(c->counters) + 4, V, c->ph_info.p,
                                   P<uint64_t>(c->rowoff), P<char>(c->text), c->stream));
    prof_end(c, "ph_fmt");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->text_bytes = text;
    c->ph_nvar = V;
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = L;
        out->rows = V;
        out->text_bytes = text;
    }
    return VCFXG_OK;
}

int vcfxg_phaser_variants(vcfxg_ctx *c, uint8_t *flags, double *r2, uint64_t *offs) {
    if (!c) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    const uint64_t V = c->ph_nvar;
    if (flags && V) HIPCHK(c, hipMemcpyAsync(flags, c->ph_flags.p, V, hipMemcpyDeviceToHost, c->stream));
    if (r2 && V) HIPCHK(c, hipMemcpyAsync(r2, c->ph_r2.p, 8 * V, hipMemcpyDeviceToHost, c->stream));
    if (offs) HIPCHK(c, hipMemcpyAsync(offs, c->rowoff.p, 8 * (V + 1), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

// VCFX_missing_detector over [data_start, n): for long GT-only records the filter / query walk
// with the missing-allele reducer (one HBM pass; k_md_lines then takes the lines it left and
// the flagged lines' INFO spans), else the line index and k_md_lines on every line
static int md_region_walk(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out) {
    c->dense_pending = false;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n, C = c->walk_chunk;
    const int64_t nw = vcfxg::af_walkers(lo, hi, C);
    const uint64_t cap_w = (uint64_t)(2 * C / std::max<int64_t>(c->hint_line, 64)) + 16;
    const uint64_t cap = (uint64_t)nw * cap_w;
    const size_t mb = vcfxg::af_meta_bytes();
    int r = ensure(c, c->wk_le, 8 * cap);
    if (!r) r = ensure(c, c->wk_status, cap);
    if (!r) r = ensure(c, c->wk_meta, mb * cap);
    if (!r) r = ensure(c, c->wk_count, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->wk_offs, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->fq_small, 128);
    if (!r) r = ensure_sum_host(c);
    if (!r) r = ensure(c, c->line_end, 8 * (cap + 1));
    if (!r) r = ensure(c, c->af_meta, mb * (cap + 1));
    if (!r) r = af_buffers(c, cap);
    if (r) return r;
    const char *buf = P<char>(c->input);
    // the filter / query walk's slot and counters (zeroed by k_fq_done after the last call)
    unsigned *ovf = P<unsigned>(c->fq_small);
    unsigned long long *cnt = P<unsigned long long>(c->fq_small) + 1;
    const vcfxg::RfArgs ra{nullptr, 0, 1, nullptr, 0};
    if (c->fq_small_dirty) HIPCHK(c, hipMemsetAsync(c->fq_small.p, 0, 128, c->stream));
    c->fq_small_dirty = true;
    prof_begin(c, "md_walk");
    HIPCHK(c, vcfxg::launch_fq_walk(vcfxg::kFqMD, buf, lo, hi, C, mode == VCFXG_MODE_FILE ? 1 : 0, c->hint_span, cap_w, ra,
                                    nullptr, 0, 0, -1, -1, P<uint64_t>(c->wk_le), P<uint8_t>(c->wk_status),
                                    c->wk_meta.p, nullptr, P<uint64_t>(c->wk_count), ovf, c->stream));
    prof_end(c, "md_walk");
    prof_begin(c, "md_rest");
    r = exclusive_scan(c, P<uint64_t>(c->wk_count), P<uint64_t>(c->wk_offs), (size_t)nw + 1);
    if (r) return r;
    HIPCHK(c, vcfxg::launch_fq_compact(vcfxg::kFqMD, nw, cap_w, P<uint64_t>(c->wk_offs), P<uint64_t>(c->wk_le),
                                       P<uint8_t>(c->wk_status), c->wk_meta.p, nullptr, P<uint64_t>(c->line_end),
                                       P<uint8_t>(c->status), c->af_meta.p, nullptr, P<uint64_t>(c->d_nlines),
                                       c->stream));
    HIPCHK(c, vcfxg::launch_md_lines(buf, lo, (int64_t)c->n, P<uint64_t>(c->line_end), P<uint64_t>(c->d_nlines), cap,
                                     mode, P<uint8_t>(c->status), P<int32_t>(c->alt), P<int32_t>(c->tot),
                                     cnt, c->stream, 1));
    prof_end(c, "md_rest");
    HIPCHK(c, vcfxg::launch_fq_done(cnt, P<uint64_t>(c->d_nlines), P<uint64_t>(c->fq_small), c->sum_dev + 8, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->fq_small_dirty = false;
    uint64_t h[5] = {c->sum_host[8], c->sum_host[9], c->sum_host[10], c->sum_host[16], c->sum_host[17]};
    prof_collect(c);
    if (h[4] & 0xFFFFFFFFu) {  // a walker ran out of line slots (short lines): no walk
        c->walk_overflowed = true;
        return vcfxg_missing_region(c, data_start, mode, out);
    }
    c->data_start = data_start;
    c->n_lines = h[3];
    c->indexed = true;
    c->text_bytes = 0;
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = h[3];
        out->data_lines = h[0];
        out->rows = h[1];
        out->general_records = h[2];
    }
    return VCFXG_OK;
}

int vcfxg_missing_region(vcfxg_ctx *c, size_t data_start, int mode, vcfxg_summary *out) {
    if (!c || (mode != VCFXG_MODE_FILE && mode != VCFXG_MODE_STDIN)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    // the walk for long GT-only records (VCFXG_FQ_WALK: 1 always, -1 never), as the filter tools
    if (vcfxg::af_walkers((int64_t)data_start, (int64_t)c->n, c->walk_chunk) && c->fq_path >= 0 && !c->walk_overflowed &&
        (c->fq_path == 1 || (c->hint_line >= 512 && c->hint_gt_only)))
        return md_region_walk(c, data_start, mode, out);
    uint64_t L = 0;
    int r = vcfxg_index(c, data_start, &L);
    if (r) return r;
    HIPCHK(c, hipSetDevice(c->device));
    r = af_buffers(c, L);
    if (r) return r;
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 64, c->stream));
    prof_begin(c, "md_lines");
    HIPCHK(c, vcfxg::launch_md_lines(P<char>(c->input), (int64_t)data_start, (int64_t)c->n, P<uint64_t>(c->line_end),
                                     P<uint64_t>(c->d_nlines), L, mode, P<uint8_t>(c->status), P<int32_t>(c->alt),
                                     P<int32_t>(c->tot), P<unsigned long long>(c->counters), c->stream));
    prof_end(c, "md_lines");
    static thread_local uint64_t cnt[3];
    HIPCHK(c, hipMemcpyAsync(cnt, c->counters.p, sizeof cnt, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    if (out) {
        std::memset(out, 0, sizeof *out);
        out->n_lines = L;
        out->data_lines = cnt[0];
        out->rows = cnt[1];
        out->general_records = cnt[2];
    }
    return VCFXG_OK;
}

int vcfxg_variant_count(vcfxg_ctx *c, int strip_cr, vcfxg_summary *out) {
    if (!c) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
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

// ---------------------------------------------------------------------------------------
// LD
// ---------------------------------------------------------------------------------------
struct U16ToU64 {
    __host__ __device__ uint64_t operator()(const uint16_t &x) const { return x; }
};

// the shared tail of the LD prepare paths: M variants with ld_vars / ld_fast / ld_Gp, the
// prefix offsets ld_poff (pbytes in all) and the per-group flags ld_gflag_host in place (and
// ld_Gc when ld_gc_ready): the sparse-missing / masked planes the groups need, the prefixes
static int ld_prepare_finish(vcfxg_ctx *c, uint64_t M, int n_samples, int kpad, int kp4, int id_dot_to_pos,
                             uint64_t pbytes, bool sync_end, uint64_t *n_variants) {
    int r = VCFXG_OK;
    if (!c->ld_gc_ready) {
        for (uint64_t g = 0; g * vcfxg::kLdFastBlock < M; g++)
            if (c->ld_gflag_host[g] != 1) return VCFXG_E_STATE;  // (the walk gathers Gc for these)
    }
    r = ensure(c, c->ld_prefix, pbytes + 16);
    if (r) return r;
    // a group with a missing genotype: the valid-mask and squared-dosage planes of the
    // missing-data kernel (k_ld_mask), next to the dosage plane ld_Gp
    c->ld_vq = false;
    c->ld_sp = false;
    for (uint64_t g = 0; g * vcfxg::kLdFastBlock < M; g++) {
        c->ld_vq = c->ld_vq || c->ld_gflag_host[g] == 0;
        c->ld_sp = c->ld_sp || c->ld_gflag_host[g] == 2;
    }
    // the sparse-missing kernel's extra planes (CSR + the [sample][variant] u16 plane, about twice
    // the int8 plane) must not make an input fail that the masked kernel alone fits: when they do
    // not fit, every sparse group goes back to k_ld_mask (VCFXG_LD_SPARSE_NOMEM=1: a test hook
    // that takes this way as if the allocation had failed)
    static const bool sparse_nomem_hook = [] {
        const char *e = getenv("VCFXG_LD_SPARSE_NOMEM");
        return e && e[0] == '1';
    }();
    auto sparse_to_mask = [&]() -> int {
        (void)hipGetLastError();  // (a failed hipMalloc leaves its error to be read once)
        prof_end(c, "ld_sparse_prep");
        c->ld_sp = false;
        c->ld_vq = true;
        for (auto &f : c->ld_gflag_host)
            if (f == 2) f = 0;
        if (M)
            HIPCHK(c, hipMemcpyAsync(c->ld_gflag.p, c->ld_gflag_host.data(),
                                     (M + vcfxg::kLdFastBlock - 1) / vcfxg::kLdFastBlock, hipMemcpyHostToDevice, c->stream));
        c->err.clear();
        return VCFXG_OK;
    };
    if (c->ld_sp && sparse_nomem_hook) {
        r = sparse_to_mask();
        if (r) return r;
    }
    if (c->ld_sp) {
        // the missing samples of every variant (CSR) and the contribution plane of the
        // sparse-missing kernel (vcfxg_ld_fast.hip, kSp)
        prof_begin(c, "ld_sparse_prep");
        r = ensure(c, c->ld_moff, 8 * (M + 1));
        if (r == VCFXG_E_NOMEM) r = sparse_to_mask();
        if (r) return r;
    }
    if (c->ld_sp) {
        struct MissOf {
            int ns;
            __host__ __device__ uint64_t operator()(const vcfxg::LdVar &v) const { return (uint64_t)(ns - v.cnt); }
        };
        hipcub::TransformInputIterator<uint64_t, MissOf, const vcfxg::LdVar *> min(P<vcfxg::LdVar>(c->ld_vars),
                                                                                   MissOf{n_samples});
        size_t tmp2 = 0;
        HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, min, P<uint64_t>(c->ld_moff), (int)M + 1, c->stream));
        r = ensure(c, c->scan_tmp, tmp2);
        if (r) return r;
        // (entry M of the input is vars[M]: its cnt is written as ns below, so moff[M] = total)
        static thread_local vcfxg::LdVar pad_var;
        pad_var = vcfxg::LdVar{};
        pad_var.cnt = n_samples;
        HIPCHK(c, hipMemcpyAsync(P<vcfxg::LdVar>(c->ld_vars) + M, &pad_var, sizeof pad_var, hipMemcpyHostToDevice,
                                 c->stream));
        HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tmp2, min, P<uint64_t>(c->ld_moff), (int)M + 1,
                                                   c->stream));
        static thread_local uint64_t entries;
        HIPCHK(c, hipMemcpyAsync(&entries, P<uint64_t>(c->ld_moff) + M, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const uint64_t mp = (M + vcfxg::kLdFastBlock - 1) / vcfxg::kLdFastBlock * vcfxg::kLdFastBlock;
        r = ensure(c, c->ld_midx, 2 * entries + 16);
        if (!r) r = ensure(c, c->ld_mvar, 4 * entries + 16);
        if (!r) r = ensure(c, c->ld_midx16, 32 * (M + 1));
        if (!r) r = ensure(c, c->ld_sprec, sizeof(vcfxg::LdSpRec) * (M + 1));
        if (!r) r = ensure(c, c->ld_gt16, 2 * (size_t)n_samples * mp + 64);
        if (r == VCFXG_E_NOMEM) r = sparse_to_mask();
        if (r) return r;
    }
    if (c->ld_sp) {
        const uint64_t mp = (M + vcfxg::kLdFastBlock - 1) / vcfxg::kLdFastBlock * vcfxg::kLdFastBlock;
        HIPCHK(c, vcfxg::launch_ld_miss_fill(P<int8_t>(c->ld_Gc), M, kpad, n_samples, P<uint64_t>(c->ld_moff),
                                             P<uint16_t>(c->ld_midx), P<uint32_t>(c->ld_mvar), P<uint16_t>(c->ld_midx16),
                                             c->stream));
        HIPCHK(c, vcfxg::launch_ld_gt16(P<int8_t>(c->ld_Gc), M, kpad, n_samples, mp, P<uint16_t>(c->ld_gt16),
                                        c->stream));
        HIPCHK(c, vcfxg::launch_ld_sprec(P<vcfxg::LdVar>(c->ld_vars), M, n_samples, P<vcfxg::LdSpRec>(c->ld_sprec),
                                         c->stream));
        c->ld_mp = mp;
        prof_end(c, "ld_sparse_prep");
    }
    if (c->ld_vq) {
        r = ensure(c, c->ld_Gv, (size_t)(M + 1) * kp4 + 64);
        if (!r) r = ensure(c, c->ld_Gq, (size_t)(M + 1) * kp4 + 64);
        if (r) return r;
        prof_begin(c, "ld_pack_vq");
        HIPCHK(c, vcfxg::launch_ld_pack_vq(P<int8_t>(c->ld_Gc), M, kpad, n_samples, P<uint8_t>(c->ld_Gv),
                                           P<uint8_t>(c->ld_Gq), kp4, c->stream));
        prof_end(c, "ld_pack_vq");
    }
    HIPCHK(c, vcfxg::launch_ld_prefix(1, P<vcfxg::LdVar>(c->ld_vars), M, P<char>(c->input), id_dot_to_pos,
                                      P<uint64_t>(c->ld_poff), P<char>(c->ld_prefix), c->stream));
    if (sync_end) HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->ld_m = M;
    c->ld_kpad = kpad;
    c->ld_kp4 = kp4;
    c->ld_ns = n_samples;
    c->ld_prefix_bytes = pbytes;
    c->ld_chrom_ids = false;
    if (n_variants) *n_variants = M;
    return VCFXG_OK;
}

int vcfxg_ld_prepare(vcfxg_ctx *c, int n_samples, int id_dot_to_pos, const char *rchrom, size_t rlen, int has_region,
                     int rstart, int rend, int parse_mode, uint64_t *n_variants) {
    if (!c || n_samples < 0 || (has_region && !rchrom && rlen)) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t L = c->n_lines;
    const int kpad = n_samples > 0 ? ((n_samples + 63) / 64) * 64 : 64;  // MFMA k-steps of 32 B
    int r = ensure(c, c->ld_G, (size_t)L * kpad + 64);
    if (!r) r = ensure(c, c->ld_lines, sizeof(vcfxg::LdLine) * (L + 1));
    if (!r) r = ensure(c, c->ld_vidx, 8 * (L + 1));
    if (!r) r = ensure(c, c->ld_valid, 4 * (L + 1));
    if (!r) r = ensure(c, c->query, rlen + 1);
    if (r) return r;
    c->query_host.assign(rchrom ? rchrom : "", rlen);
    if (rlen) {
        c->query_dev_p = nullptr;
        HIPCHK(c, hipMemcpyAsync(c->query.p, c->query_host.data(), rlen, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipMemsetAsync(c->ld_G.p, 0xFF, (size_t)L * kpad + 64, c->stream));
    vcfxg::LdParseArgs a{n_samples, kpad, has_region, rstart, rend, (int64_t)rlen, P<char>(c->query), parse_mode};
    prof_begin(c, "ld_parse");
    HIPCHK(c, vcfxg::launch_ld_parse(P<char>(c->input), (int64_t)c->data_start, P<uint64_t>(c->line_end),
                                     P<uint64_t>(c->d_nlines), L, a, P<int8_t>(c->ld_G), P<vcfxg::LdLine>(c->ld_lines),
                                     c->stream));
    prof_end(c, "ld_parse");
    // compact order: exclusive scan of the valid flags (first member of LdLine)
    struct ValidOf {
        __host__ __device__ uint64_t operator()(const vcfxg::LdLine &x) const { return x.valid; }
    };
    hipcub::TransformInputIterator<uint64_t, ValidOf, const vcfxg::LdLine *> vin(P<vcfxg::LdLine>(c->ld_lines),
                                                                                 ValidOf());
    size_t tmp = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, vin, P<uint64_t>(c->ld_vidx), (int)L, c->stream));
    r = ensure(c, c->scan_tmp, tmp);
    if (r) return r;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tmp, vin, P<uint64_t>(c->ld_vidx), (int)L, c->stream));
    static thread_local uint64_t last[2];
    static thread_local vcfxg::LdLine lastline;
    if (L) {
        HIPCHK(c, hipMemcpyAsync(&last[0], P<uint64_t>(c->ld_vidx) + L - 1, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(&lastline, P<vcfxg::LdLine>(c->ld_lines) + L - 1, sizeof lastline,
                                 hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t M = L ? last[0] + lastline.valid : 0;
    r = ensure(c, c->ld_Gc, (size_t)(M + 1) * kpad + 64);
    if (!r) r = ensure(c, c->ld_vars, sizeof(vcfxg::LdVar) * (M + 1));
    if (!r) r = ensure(c, c->ld_fast, sizeof(vcfxg::LdFast) * (M + 1));
    const int kp4 = vcfxg::ld_kp4(n_samples);
    if (!r) r = ensure(c, c->ld_Gp, (size_t)(M + 1) * kp4 + 64);
    if (!r) r = ensure(c, c->ld_gflag, M / vcfxg::kLdFastBlock + 2);
    if (!r) r = ensure(c, c->ld_plen, 8 * (M + 2));
    if (!r) r = ensure(c, c->ld_poff, 8 * (M + 2));
    if (r) return r;
    prof_begin(c, "ld_compact");
    HIPCHK(c, vcfxg::launch_ld_compact(P<vcfxg::LdLine>(c->ld_lines), P<uint64_t>(c->ld_vidx), P<uint64_t>(c->d_nlines),
                                       L, kpad, n_samples, P<int8_t>(c->ld_G), P<int8_t>(c->ld_Gc),
                                       P<vcfxg::LdVar>(c->ld_vars), P<vcfxg::LdFast>(c->ld_fast), c->stream));
    HIPCHK(c, vcfxg::launch_ld_pack4(P<int8_t>(c->ld_Gc), M, kpad, n_samples, P<uint8_t>(c->ld_Gp), kp4, c->stream));
    prof_end(c, "ld_compact");
    // VCFXG_LD_SPARSE=0: no sparse-missing groups (their tiles take k_ld_mask)
    static const bool sparse_env = [] {
        const char *e = getenv("VCFXG_LD_SPARSE");
        return !(e && e[0] == '0');
    }();
    const int sparse = sparse_env && n_samples > 0 && n_samples <= 16383 ? 1 : 0;  // (Sxy as u16 in the epilogue)
    HIPCHK(c, vcfxg::launch_ld_groups(P<vcfxg::LdVar>(c->ld_vars), M, n_samples, sparse, P<uint8_t>(c->ld_gflag),
                                      c->stream));
    c->ld_gflag_host.assign(M / vcfxg::kLdFastBlock + 1, 0);
    if (M)
        HIPCHK(c, hipMemcpyAsync(c->ld_gflag_host.data(), c->ld_gflag.p, (M + vcfxg::kLdFastBlock - 1) / vcfxg::kLdFastBlock,
                                 hipMemcpyDeviceToHost, c->stream));
    // per-variant "chrom\tpos\tid" prefixes
    HIPCHK(c, vcfxg::launch_ld_prefix(0, P<vcfxg::LdVar>(c->ld_vars), M, P<char>(c->input), id_dot_to_pos,
                                      P<uint64_t>(c->ld_plen), nullptr, c->stream));
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->ld_plen) + M, 0, 8, c->stream));
    r = exclusive_scan(c, P<uint64_t>(c->ld_plen), P<uint64_t>(c->ld_poff), (size_t)M + 1);
    if (r) return r;
    static thread_local uint64_t pbytes;
    HIPCHK(c, hipMemcpyAsync(&pbytes, P<uint64_t>(c->ld_poff) + M, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->ld_gc_ready = true;
    return ld_prepare_finish(c, M, n_samples, kpad, kp4, id_dot_to_pos, pbytes, true, n_variants);
}

// vcfxg_index(data_start) + vcfxg_ld_prepare in one call, with the same variants, rows, sums and
// prefixes.  The default for records averaging >= 512 B with n_samples <= 4096: the LD walk
// (vcfxg_ld.hip k_ld_walk: one HBM pass over the records, no line index), then one compaction
// that writes the variant records, the FP4 rows and the prefix lengths, and ONE host
// synchronisation for the variant count, the prefix bytes and the group flags.  The int8 rows in
// variant order (ld_Gc) are gathered only when some variant misses a call (the sparse-missing and
// masked kernels read them).  A walker over its line capacity, or an input the walk does not
// take, runs vcfxg_index + vcfxg_ld_prepare (VCFXG_LD_WALK=0: always).  The context is not
// indexed afterwards (vcfxg_line_ends and the per-line calls need vcfxg_index).
int vcfxg_ld_prepare_region(vcfxg_ctx *c, size_t data_start, int n_samples, int id_dot_to_pos, const char *rchrom,
                            size_t rlen, int has_region, int rstart, int rend, int parse_mode, uint64_t *n_variants) {
    if (!c || n_samples < 0 || (has_region && !rchrom && rlen)) return VCFXG_E_ARG;
    if (!c->loaded) return VCFXG_E_STATE;
    if (data_start > c->n) data_start = c->n;
    c->dense_pending = false;  // a new index / regions replace the pending ones
    HIPCHK(c, hipSetDevice(c->device));
    static const bool walk_env = [] {
        const char *e = getenv("VCFXG_LD_WALK");
        return !(e && e[0] == '0');
    }();
    const int64_t lo = (int64_t)data_start, hi = (int64_t)c->n;
    // the walkers' chunk: the record walks' (128 KiB for ~10 KB records), halved while the input
    // would give fewer than about 2 rounds of walkers over the chip (a 1 GB LD shard: 64 KiB;
    // each walker's last round otherwise runs with the chip half empty); VCFXG_LD_WALK_CHUNK
    // overrides
    static const int64_t ld_chunk_env = getenv("VCFXG_LD_WALK_CHUNK") ? atol(getenv("VCFXG_LD_WALK_CHUNK")) : 0;
    int64_t C = c->walk_chunk;
    if (ld_chunk_env >= 4096) C = ld_chunk_env;
    else
        while (C > 32768 && (hi - lo) / C < 2 * 20 * (int64_t)std::max(c->n_cu, 1)) C /= 2;
    const int64_t nw = hi > lo ? (hi - lo + C - 1) / C : 0;
    const uint64_t cap_w = (uint64_t)(2 * C / std::max<int64_t>(c->hint_line, 64)) + 16;
    const bool walk = walk_env && nw > 0 && n_samples > 0 && n_samples <= 4096 && c->hint_line >= 512 &&
                      !c->walk_overflowed && cap_w <= 0xFFFF;
    auto indexed_path = [&]() -> int {
        note_schedule(c, "ld_index");
        int r = vcfxg_index(c, data_start, nullptr);
        return r ? r : vcfxg_ld_prepare(c, n_samples, id_dot_to_pos, rchrom, rlen, has_region, rstart, rend, parse_mode,
                                        n_variants);
    };
    if (!walk) return indexed_path();
    const uint64_t cap = (uint64_t)nw * cap_w;
    const int kpad = ((n_samples + 63) / 64) * 64;
    const int kp4 = vcfxg::ld_kp4(n_samples);
    int r = ensure(c, c->ld_G, (size_t)cap * kpad + 64);
    if (!r) r = ensure(c, c->ld_lines, sizeof(vcfxg::LdLine) * (cap + 1));
    if (!r) r = ensure(c, c->ld_wcnt, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->ld_wval, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->ld_vbase, 8 * (size_t)(nw + 1));
    if (!r) r = ensure(c, c->ld_small, 64);
    if (!r) r = ensure(c, c->ld_pend, 8 * (cap + 1));
    if (!r) r = ensure(c, c->ld_vars, sizeof(vcfxg::LdVar) * (cap + 1));
    if (!r) r = ensure(c, c->ld_fast, sizeof(vcfxg::LdFast) * (cap + 1));
    if (!r) r = ensure(c, c->ld_Gp, (size_t)(cap + 1) * kp4 + 64);
    if (!r) r = ensure(c, c->ld_gflag, cap / vcfxg::kLdFastBlock + 2);
    if (!r) r = ensure(c, c->ld_plen, 8 * (cap + 2));
    if (!r) r = ensure(c, c->ld_poff, 8 * (cap + 2));
    if (!r) r = ensure(c, c->query, rlen + 1);
    if (r) return r;
    if (rlen) {
        c->query_host.assign(rchrom, rlen);
        c->query_dev_p = nullptr;
        HIPCHK(c, hipMemcpyAsync(c->query.p, c->query_host.data(), rlen, hipMemcpyHostToDevice, c->stream));
    }
    const char *buf = P<char>(c->input);
    // small: [0] walk overflow (u32) | flags (u32: bit 0 = an incomplete variant), [1] M,
    // [2] pending lines
    uint64_t *small = P<uint64_t>(c->ld_small);
    unsigned *ovf = reinterpret_cast<unsigned *>(small), *flags = ovf + 1;
    HIPCHK(c, hipMemsetAsync(small, 0, 24, c->stream));
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->ld_wval) + nw, 0, 8, c->stream));
    HIPCHK(c, hipMemsetAsync(c->ld_plen.p, 0, 8 * (cap + 1), c->stream));
    vcfxg::LdParseArgs a{n_samples, kpad, has_region, rstart, rend, (int64_t)rlen, P<char>(c->query), parse_mode};
    prof_begin(c, "ld_walk");
    HIPCHK(c, vcfxg::launch_ld_walk(buf, lo, hi, C, c->hint_span, cap_w, a, P<int8_t>(c->ld_G),
                                    P<vcfxg::LdLine>(c->ld_lines), P<uint64_t>(c->ld_wcnt), P<uint64_t>(c->ld_wval),
                                    ovf, reinterpret_cast<unsigned long long *>(small + 2), P<uint64_t>(c->ld_pend),
                                    c->stream));
    prof_end(c, "ld_walk");
    prof_begin(c, "ld_compact");
    r = exclusive_scan(c, P<uint64_t>(c->ld_wval), P<uint64_t>(c->ld_vbase), (size_t)nw + 1);
    if (r) return r;
    HIPCHK(c, vcfxg::launch_ld_wcompact(nw, cap_w, P<uint64_t>(c->ld_wcnt), P<uint64_t>(c->ld_vbase),
                                        P<vcfxg::LdLine>(c->ld_lines), n_samples, buf, id_dot_to_pos,
                                        P<vcfxg::LdVar>(c->ld_vars), P<vcfxg::LdFast>(c->ld_fast),
                                        P<uint64_t>(c->ld_plen), flags, small + 1, c->stream));
    prof_end(c, "ld_compact");
    static const bool sparse_env = [] {
        const char *e = getenv("VCFXG_LD_SPARSE");
        return !(e && e[0] == '0');
    }();
    const int sparse = sparse_env && n_samples <= 16383 ? 1 : 0;
    HIPCHK(c, vcfxg::launch_ld_groups(P<vcfxg::LdVar>(c->ld_vars), cap, n_samples, sparse, P<uint8_t>(c->ld_gflag),
                                      c->stream, small + 1));
    r = exclusive_scan(c, P<uint64_t>(c->ld_plen), P<uint64_t>(c->ld_poff), (size_t)cap + 1);
    if (r) return r;
    // one synchronisation: overflow, flags, M, the prefix bytes (plen is 0 past M) and the
    // group flags (computed for every group below cap; the first ceil(M / 256) are M's)
    static thread_local uint64_t sm[3];
    const uint64_t ng = (cap + vcfxg::kLdFastBlock - 1) / vcfxg::kLdFastBlock;
    c->ld_gflag_host.assign(ng + 1, 0);
    HIPCHK(c, hipMemcpyAsync(sm, small, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(sm + 2, P<uint64_t>(c->ld_poff) + cap, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->ld_gflag_host.data(), c->ld_gflag.p, ng, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((uint32_t)sm[0]) {  // a walker ran out of line slots (short lines): the index path
        prof_collect(c);
        c->walk_overflowed = true;
        return indexed_path();
    }
    note_schedule(c, "ld_walk");
    const uint64_t M = sm[1], pbytes = sm[2];
    prof_begin(c, "ld_pack");  // the FP4 rows, from the walk's slots
    HIPCHK(c, vcfxg::launch_ld_pack4(P<int8_t>(c->ld_G), M, kpad, n_samples, P<uint8_t>(c->ld_Gp), kp4, c->stream,
                                     P<vcfxg::LdVar>(c->ld_vars)));
    prof_end(c, "ld_pack");
    c->ld_gflag_host.resize(M / vcfxg::kLdFastBlock + 1);
    for (uint64_t g = (M + vcfxg::kLdFastBlock - 1) / vcfxg::kLdFastBlock; g < c->ld_gflag_host.size(); g++)
        c->ld_gflag_host[g] = 0;  // (past M: as the indexed path leaves them)
    c->ld_gc_ready = false;
    if ((sm[0] >> 32) & 1u) {  // some variant misses a call: its group's kernels read ld_Gc
        r = ensure(c, c->ld_Gc, (size_t)(M + 1) * kpad + 64);
        if (r) return r;
        prof_begin(c, "ld_gather");
        HIPCHK(c, vcfxg::launch_ld_gather(P<vcfxg::LdVar>(c->ld_vars), M, P<int8_t>(c->ld_G), kpad,
                                          P<int8_t>(c->ld_Gc), c->stream));
        prof_end(c, "ld_gather");
        c->ld_gc_ready = true;
    }
    c->indexed = false;  // (no line index: vcfxg_index before any per-line call)
    return ld_prepare_finish(c, M, n_samples, kpad, kp4, id_dot_to_pos, pbytes, false, n_variants);
}

// exact chrom equality ids (for max_dist): strings are the first field of each prefix
static int ld_chrom_ids(vcfxg_ctx *c) {
    if (c->ld_chrom_ids) return VCFXG_OK;
    const uint64_t M = c->ld_m;
    std::vector<uint64_t> poff(M + 1);
    std::string pre(c->ld_prefix_bytes, '\0');
    HIPCHK(c, hipMemcpyAsync(poff.data(), c->ld_poff.p, 8 * (M + 1), hipMemcpyDeviceToHost, c->stream));
    if (!pre.empty())
        HIPCHK(c, hipMemcpyAsync(&pre[0], c->ld_prefix.p, pre.size(), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::map<std::string, uint32_t> ids;
    std::vector<uint32_t> id(M + 1);
    for (uint64_t v = 0; v < M; v++) {
        size_t a = poff[v], tab = pre.find('\t', a);
        auto ins = ids.emplace(pre.substr(a, tab - a), (uint32_t)ids.size());
        id[v] = ins.first->second;
    }
    int r = ensure(c, c->ld_cid, 4 * (M + 1));
    if (r) return r;
    c->ld_cid_host.swap(id);
    HIPCHK(c, hipMemcpyAsync(c->ld_cid.p, c->ld_cid_host.data(), 4 * M, hipMemcpyHostToDevice, c->stream));
    c->ld_chrom_ids = true;
    return VCFXG_OK;
}

int vcfxg_ld_stream_chunk(vcfxg_ctx *c, uint64_t j0, uint64_t j1, uint64_t window, double threshold, int max_dist,
                          uint64_t *n_pairs, uint64_t *text_bytes) {
    if (!c) return VCFXG_E_ARG;
    const uint64_t M = c->ld_m;
    if (j1 > M) j1 = M;
    if (window > M) window = M;  // a wider window holds the same pairs (and stays int64-safe)
    if (j0 >= j1 || M < 2) {
        c->text_bytes = 0;
        if (n_pairs) *n_pairs = 0;
        if (text_bytes) *text_bytes = 0;
        return VCFXG_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t BM = vcfxg::kLdBlock;
    if (max_dist > 0) {
        int r = ld_chrom_ids(c);
        if (r) return r;
    }
    // block lists.  Count-table columns are 64-blocks: row block J pairs with column blocks
    // I0(J) = (J*64 - window)/64 .. J.  Pairs of 256-groups that are all complete go to the
    // 256x256 X.X^T kernel (k_ld_fast); every other 64-block to the general kernel.
    const uint64_t FB = vcfxg::kLdFastBlock;
    auto ifirst = [&](uint64_t J) { const uint64_t jr0 = J * BM; return jr0 > window ? (jr0 - window) / BM : 0; };
    const std::vector<uint8_t> &gf = c->ld_gflag_host;
    constexpr uint64_t kSub = vcfxg::kLdFastBlock / BM;  // 64-blocks per fast group
    // a 64-block whose 256-group the fast or the sparse-missing kernel covers (with another such)
    auto gcomp = [&](uint64_t b64) { const uint8_t g = gf[b64 / kSub]; return g == 1 || (g == 2 && c->ld_sp); };
    static const bool use_mask = [] {
        const char *e = getenv("VCFXG_LD_MASK");
        return !(e && e[0] == '0');
    }();
    // the block lists are a pure function of (j0, j1, window, M, the kernel choice, the
    // per-group complete flags): a call with the same ones reuses the last lists and their
    // device copy (building 77 K tile pairs and copying them cost ~0.13 ms of host time per call)
    const bool mask_on = use_mask && c->ld_vq;
    const bool sp_on = c->ld_sp;
    const uint64_t pkey[5] = {j0, j1, window, M, (mask_on ? 1u : 0u) | (sp_on ? 2u : 0u)};
    const bool hit = c->ld_plan_dev != nullptr && c->ld_plan_dev == c->ld_blocks.p &&
                     std::equal(pkey, pkey + 5, c->ld_plan_key) && c->ld_plan_gf == gf;
    std::vector<uint32_t> blocks;
    uint64_t nb = 1;
    uint32_t nfast = 0, nmask = 0, nbl = 0, nsp = 0;
    for (uint64_t J = j0 / BM; J * BM < j1; J++) nb = std::max<uint64_t>(nb, J - ifirst(J) + 1);
    nb = (nb + 7) & ~(uint64_t)7;  // (k_ld_rowscan reads a row's counts 8 slots per 16 B load)
    if (hit) {
        nfast = c->ld_plan_n[0];
        nmask = c->ld_plan_n[1];
        nbl = c->ld_plan_n[2];
        nsp = c->ld_plan_n[3];
    } else {
        // fast list first, in kSuper x kSuper super-tiles (row blocks J x column blocks I): the
        // kernel maps contiguous list ranges to one XCD, so the blocks an XCD runs at once share
        // 2*kSuper operand tiles through its L2 instead of streaming distinct ones
        static const uint64_t kSuper = [] {
            const char *e = getenv("VCFXG_LD_SUPER");
            const long v = e ? atol(e) : 0;
            return (uint64_t)(v > 0 ? v : 4);
        }();
        const uint64_t Jb = j0 / FB, Je = (j1 + FB - 1) / FB;
        // pass 0: both groups complete (k_ld_fast); pass 1: both complete or sparse-missing, not
        // both complete (the sparse-missing form, kSp)
        for (int pass = 0; pass < (sp_on ? 2 : 1); pass++) {
            auto take = [&](uint64_t I, uint64_t J) {
                return pass == 0 ? gf[I] == 1 && gf[J] == 1 : gf[I] && gf[J] && (gf[I] == 2 || gf[J] == 2);
            };
            for (uint64_t J0 = Jb; J0 < Je; J0 += kSuper) {
                const uint64_t J1 = std::min(Je, J0 + kSuper);
                const uint64_t Ilo = ifirst(kSub * J0) / kSub;
                for (uint64_t I0 = Ilo; I0 < J1; I0 += kSuper)
                    for (uint64_t J = J0; J < J1; J++) {
                        if (!gf[J]) continue;
                        const uint64_t Imin = std::max(I0, ifirst(kSub * J) / kSub), Imax = std::min(I0 + kSuper, J + 1);
                        for (uint64_t I = Imin; I < Imax; I++)
                            if (take(I, J)) {
                                blocks.push_back((uint32_t)I);
                                blocks.push_back((uint32_t)J);
                            }
                    }
            }
            if (pass == 0) nfast = (uint32_t)(blocks.size() / 2);
            else nsp = (uint32_t)(blocks.size() / 2) - nfast;
        }
        // the missing-data tiles (k_ld_mask, default): every 128 x 128 tile pair in the window
        // whose 256-groups are not both complete (those are k_ld_fast's); VCFXG_LD_MASK=0 keeps the
        // previous int8 kernel (k_ld_block) over every 64-block pair with an incomplete side

        if (use_mask && c->ld_vq) {
            constexpr uint64_t TM = vcfxg::kLdMaskTile, kPerG = vcfxg::kLdFastBlock / vcfxg::kLdMaskTile;
            for (uint64_t J2 = j0 / TM; J2 * TM < j1; J2++) {
                const uint64_t I2lo = ifirst(J2 * (TM / BM)) / (TM / BM);  // the first 64-row's window start
                const uint8_t gj = gf[J2 / kPerG];
                for (uint64_t I2 = I2lo; I2 <= J2; I2++) {
                    const uint8_t gi = gf[I2 / kPerG];
                    if (gi == 1 && gj == 1) continue;           // a complete group pair: k_ld_fast
                    if (sp_on && gi && gj) continue;            // complete / sparse: the kSp kernel
                    blocks.push_back((uint32_t)I2);
                    blocks.push_back((uint32_t)J2);
                }
            }
            nmask = (uint32_t)(blocks.size() / 2) - nfast - nsp;
        } else {
            // for a complete row block J only the incomplete column blocks, found in the sorted list
            // of them (no scan over the whole window triangle on the host)
            const uint64_t Jlast = (j1 + BM - 1) / BM;
            std::vector<uint32_t> inc;
            for (uint64_t b = ifirst(j0 / BM); b < Jlast; b++)
                if (!gcomp(b)) inc.push_back((uint32_t)b);
            for (uint64_t J = j0 / BM; J * BM < j1; J++) {
                const uint64_t I0 = ifirst(J);
                if (!gcomp(J)) {
                    for (uint64_t I = I0; I <= J; I++) {
                        blocks.push_back((uint32_t)I);
                        blocks.push_back((uint32_t)J);
                    }
                    continue;
                }
                for (auto it = std::lower_bound(inc.begin(), inc.end(), (uint32_t)I0); it != inc.end() && *it <= J; ++it) {
                    blocks.push_back(*it);
                    blocks.push_back((uint32_t)J);
                }
            }
            nbl = (uint32_t)(blocks.size() / 2) - nfast - nsp;
        }
    }
    const uint64_t rows = j1 - j0;
    int r = hit ? VCFXG_OK : ensure(c, c->ld_blocks, 4 * blocks.size() + 8);
    if (!r) r = ensure(c, c->ld_cnt, 2 * rows * nb + 16);
    if (!r) r = ensure(c, c->ld_off, 4 * (rows * nb + 1));  // u32 offsets inside each row
    if (!r) r = ensure(c, c->ld_rowoff, 16 * (rows + 1));      // row totals, then row starts
    if (r) return r;
    if (!hit) {
        c->ld_blocks_host.swap(blocks);
        HIPCHK(c, hipMemcpyAsync(c->ld_blocks.p, c->ld_blocks_host.data(), 4 * c->ld_blocks_host.size(),
                                 hipMemcpyHostToDevice, c->stream));
        std::copy(pkey, pkey + 5, c->ld_plan_key);
        c->ld_plan_gf = gf;
        c->ld_plan_n[0] = nfast;
        c->ld_plan_n[1] = nmask;
        c->ld_plan_n[2] = nbl;
        c->ld_plan_n[3] = nsp;
        c->ld_plan_dev = c->ld_blocks.p;
    }
    // (no clearing of ld_cnt: the count kernels write every window slot the row scan reads)
    vcfxg::LdWindowArgs a{M, c->ld_kpad, c->ld_ns, window, threshold, max_dist, j0, j1, nb, 0.0, 0};
    // prefilter margin: |fp64 r^2 - exact r^2| of the reference's sequence is < ~1.2e-14 * n
    // (vx >= (n-1)/n^2 for a polymorphic complete variant); delta covers it 100-fold
    a.tm = threshold - (1e-6 + 1e-10 * (double)c->ld_ns);
    a.all_pass = a.tm <= 0.0;
    a.kp4 = c->ld_kp4;
    const uint32_t *cid = max_dist > 0 ? P<uint32_t>(c->ld_cid) : nullptr;
    const uint32_t *fbl = P<uint32_t>(c->ld_blocks), *sbl = fbl + 2 * (size_t)nfast,
                   *gbl = sbl + 2 * (size_t)nsp;
    vcfxg::LdSparse spa;
    if (nsp) {
        spa.vars = P<vcfxg::LdVar>(c->ld_vars);
        spa.gt16 = P<uint16_t>(c->ld_gt16);
        spa.mp = c->ld_mp;
        spa.moff = P<uint64_t>(c->ld_moff);
        spa.midx = P<uint16_t>(c->ld_midx);
        spa.mvar = P<uint32_t>(c->ld_mvar);
        spa.midx16 = P<uint16_t>(c->ld_midx16);
        spa.rec = P<vcfxg::LdSpRec>(c->ld_sprec);
        const double big = 4.0 * (double)c->ld_ns * (double)c->ld_ns;  // (k_ld_mask's bound)
        spa.pe = (float)(big * std::ldexp(1.0, -23) + 1.0);
    }
    // staging for the pairs the count pass finds (capacity: what the last chunk needed, at
    // least 4 M pairs; a larger chunk overflows once and the emit pass recomputes)
    vcfxg::LdStage stg;
    {
        const uint64_t qcap = 16ull * (nfast + nsp) + 16;
        const uint64_t tcap = c->ld_stage_cap_fixed ? c->ld_stage_cap_fixed : std::max<uint64_t>(c->ld_temp_cap, 4ull << 20);
        int r0 = ensure(c, c->ld_temp, sizeof(vcfxg::LdPair) * tcap);
        if (!r0) r0 = ensure(c, c->ld_quarters, sizeof(vcfxg::LdQuarter) * qcap);
        if (!r0) r0 = ensure(c, c->ld_stage_ctr, 64);
        if (r0) return r0;
        HIPCHK(c, hipMemsetAsync(c->ld_stage_ctr.p, 0, 64, c->stream));
        // (the register count path, n <= 23170, is the one that stages)
        stg.temp = c->ld_ns <= 23170 ? P<vcfxg::LdPair>(c->ld_temp) : nullptr;
        stg.cap = tcap;
        stg.quarters = P<vcfxg::LdQuarter>(c->ld_quarters);
        stg.qcap = qcap;
        stg.ctr = P<unsigned long long>(c->ld_stage_ctr);
        stg.overflow = reinterpret_cast<unsigned *>(P<unsigned long long>(c->ld_stage_ctr) + 2);
    }
    prof_begin(c, "ld_count");
    HIPCHK(c, vcfxg::launch_ld_fast(1, P<uint8_t>(c->ld_Gp), P<vcfxg::LdFast>(c->ld_fast), cid, a, fbl, nfast,
                                    P<uint16_t>(c->ld_cnt), vcfxg::LdOffsets{}, nullptr, stg, c->stream));
    prof_end(c, "ld_count");
    prof_begin(c, "ld_count_sparse");
    HIPCHK(c, vcfxg::launch_ld_sparse(1, P<uint8_t>(c->ld_Gp), spa, cid, a, sbl, nsp, P<uint16_t>(c->ld_cnt),
                                      vcfxg::LdOffsets{}, nullptr, stg, c->stream));
    prof_end(c, "ld_count_sparse");
    prof_begin(c, "ld_count_gen");
    HIPCHK(c, vcfxg::launch_ld_block(1, P<int8_t>(c->ld_Gc), P<vcfxg::LdVar>(c->ld_vars), cid, a, gbl, nbl,
                                     P<uint16_t>(c->ld_cnt), vcfxg::LdOffsets{}, nullptr, c->stream));
    prof_end(c, "ld_count_gen");
    prof_begin(c, "ld_count_mask");
    HIPCHK(c, vcfxg::launch_ld_mask(1, P<uint8_t>(c->ld_Gp), P<uint8_t>(c->ld_Gv), P<uint8_t>(c->ld_Gq),
                                    P<vcfxg::LdVar>(c->ld_vars), cid, a, gbl, nmask, P<uint16_t>(c->ld_cnt),
                                    vcfxg::LdOffsets{}, nullptr, c->stream));
    prof_end(c, "ld_count_mask");
    // ordered offsets: per-row scan of the count table (u32 inside a row), then the rows
    uint64_t *rowtot = P<uint64_t>(c->ld_rowoff), *rowbase = rowtot + (rows + 1);
    HIPCHK(c, vcfxg::launch_ld_rowscan(P<uint16_t>(c->ld_cnt), rows, nb, j0, window, P<uint32_t>(c->ld_off), rowtot,
                                       c->stream));
    HIPCHK(c, hipMemsetAsync(rowtot + rows, 0, 8, c->stream));
    r = exclusive_scan(c, rowtot, rowbase, (size_t)rows + 1);
    if (r) return r;
    vcfxg::LdOffsets offs;
    offs.row = rowbase;
    offs.in_row = P<uint32_t>(c->ld_off);
    static thread_local uint64_t tot, sctr[3];
    HIPCHK(c, hipMemcpyAsync(&tot, rowbase + rows, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(sctr, c->ld_stage_ctr.p, 24, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (getenv("VCFXG_LD_DEBUG")) {  // (with a VCFXG_LD_EXPT & 256 build: the sparse kernel's half counts)
        uint64_t dbg[3] = {0, 0, 0};
        (void)hipMemcpy(dbg, P<unsigned long long>(c->ld_stage_ctr) + 4, 24, hipMemcpyDeviceToHost);
        fprintf(stderr, "ld_sparse: halves %llu, with tables %llu, prefilter candidates %llu\n",
                (unsigned long long)dbg[0], (unsigned long long)dbg[1], (unsigned long long)dbg[2]);
    }
    const uint64_t np = tot;
    const bool staged = stg.temp && (sctr[2] & 0xFFFFFFFFull) == 0;  // staged, no overflow
    c->ld_temp_cap = std::max<uint64_t>(c->ld_temp_cap, sctr[0] + sctr[0] / 4);
    r = ensure(c, c->ld_pairs, sizeof(vcfxg::LdPair) * (np + 1));
    if (!r) r = ensure(c, c->rowlen, 8 * (np + 1));
    if (!r) r = ensure(c, c->rowoff, 8 * (np + 1));
    if (r) return r;
    prof_begin(c, "ld_emit");
    if (staged)
        HIPCHK(c, vcfxg::launch_ld_scatter(P<vcfxg::LdQuarter>(c->ld_quarters), P<unsigned long long>(c->ld_stage_ctr),
                                           sctr[1], a, P<uint16_t>(c->ld_cnt), offs,
                                           P<vcfxg::LdPair>(c->ld_temp), P<vcfxg::LdPair>(c->ld_pairs), c->stream));
    else {
        HIPCHK(c, vcfxg::launch_ld_fast(2, P<uint8_t>(c->ld_Gp), P<vcfxg::LdFast>(c->ld_fast), cid, a, fbl, nfast,
                                        P<uint16_t>(c->ld_cnt), offs, P<vcfxg::LdPair>(c->ld_pairs),
                                        vcfxg::LdStage{}, c->stream));
        HIPCHK(c, vcfxg::launch_ld_sparse(2, P<uint8_t>(c->ld_Gp), spa, cid, a, sbl, nsp, P<uint16_t>(c->ld_cnt), offs,
                                          P<vcfxg::LdPair>(c->ld_pairs), vcfxg::LdStage{}, c->stream));
    }
    prof_end(c, "ld_emit");
    prof_begin(c, "ld_emit_gen");
    HIPCHK(c, vcfxg::launch_ld_block(2, P<int8_t>(c->ld_Gc), P<vcfxg::LdVar>(c->ld_vars), cid, a, gbl, nbl,
                                     P<uint16_t>(c->ld_cnt), offs, P<vcfxg::LdPair>(c->ld_pairs),
                                     c->stream));
    prof_end(c, "ld_emit_gen");
    prof_begin(c, "ld_emit_mask");
    HIPCHK(c, vcfxg::launch_ld_mask(2, P<uint8_t>(c->ld_Gp), P<uint8_t>(c->ld_Gv), P<uint8_t>(c->ld_Gq),
                                    P<vcfxg::LdVar>(c->ld_vars), cid, a, gbl, nmask, P<uint16_t>(c->ld_cnt), offs,
                                    P<vcfxg::LdPair>(c->ld_pairs), c->stream));
    prof_end(c, "ld_emit_mask");
    HIPCHK(c, vcfxg::launch_ld_pairtext(0, P<vcfxg::LdPair>(c->ld_pairs), np, P<uint64_t>(c->ld_poff), nullptr,
                                        P<uint64_t>(c->rowlen), nullptr, c->stream));
    HIPCHK(c, hipMemsetAsync(P<uint64_t>(c->rowlen) + np, 0, 8, c->stream));
    r = exclusive_scan(c, P<uint64_t>(c->rowlen), P<uint64_t>(c->rowoff), (size_t)np + 1);
    if (r) return r;
    static thread_local uint64_t tb;
    HIPCHK(c, hipMemcpyAsync(&tb, P<uint64_t>(c->rowoff) + np, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    r = ensure(c, c->text, tb + 16);
    if (r) return r;
    prof_begin(c, "ld_text");
    HIPCHK(c, vcfxg::launch_ld_pairtext(1, P<vcfxg::LdPair>(c->ld_pairs), np, P<uint64_t>(c->ld_poff),
                                        P<char>(c->ld_prefix), P<uint64_t>(c->rowoff), P<char>(c->text), c->stream));
    prof_end(c, "ld_text");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->text_bytes = tb;
    c->ld_np = np;
    if (n_pairs) *n_pairs = np;
    if (text_bytes) *text_bytes = tb;
    return VCFXG_OK;
}

int vcfxg_ld_fetch_pairs(vcfxg_ctx *c, uint64_t first, uint64_t count, uint32_t *vi, uint32_t *vj, double *r2) {
    if (!c || first > c->ld_np || count > c->ld_np - first) return VCFXG_E_ARG;
    if (!count) return VCFXG_OK;
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<vcfxg::LdPair> h(count);
    HIPCHK(c, hipMemcpyAsync(h.data(), P<vcfxg::LdPair>(c->ld_pairs) + first, sizeof(vcfxg::LdPair) * count,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (uint64_t k = 0; k < count; ++k) {
        if (vi) vi[k] = h[k].i;
        if (vj) vj[k] = h[k].j;
        if (r2) r2[k] = h[k].r2;
    }
    return VCFXG_OK;
}

int vcfxg_ld_prefixes(vcfxg_ctx *c, char *text, size_t cap, uint64_t *offsets) {
    if (!c) return VCFXG_E_ARG;
    if (cap < c->ld_prefix_bytes) return VCFXG_E_CAP;
    if (c->ld_prefix_bytes && text)
        HIPCHK(c, hipMemcpyAsync(text, c->ld_prefix.p, c->ld_prefix_bytes, hipMemcpyDeviceToHost, c->stream));
    if (offsets)
        HIPCHK(c, hipMemcpyAsync(offsets, c->ld_poff.p, 8 * (c->ld_m + 1), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

int vcfxg_ld_matrix(vcfxg_ctx *c, int gate, int printf4, uint64_t *cell_bytes) {
    if (!c) return VCFXG_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t M = c->ld_m, BM = vcfxg::kLdBlock;
    std::vector<uint32_t> blocks;
    for (uint64_t J = 0; J * BM < M; J++)
        for (uint64_t I = 0; I <= J; I++) {
            blocks.push_back((uint32_t)I);
            blocks.push_back((uint32_t)J);
        }
    const uint64_t cells = 7ull * M * M;
    int r = ensure(c, c->ld_blocks, 4 * blocks.size() + 8);
    if (!r) r = ensure(c, c->text, cells + 16);
    if (r) return r;
    c->ld_blocks_host.swap(blocks);
    c->ld_plan_dev = nullptr;  // (the streaming lists' device copy is overwritten)
    HIPCHK(c, hipMemcpyAsync(c->ld_blocks.p, c->ld_blocks_host.data(), 4 * c->ld_blocks_host.size(),
                             hipMemcpyHostToDevice, c->stream));
    prof_begin(c, "ld_matrix");
    HIPCHK(c, vcfxg::launch_ld_matrix(P<int8_t>(c->ld_Gc), P<vcfxg::LdVar>(c->ld_vars), M, c->ld_kpad, c->ld_ns, gate,
                                      printf4, P<uint32_t>(c->ld_blocks), (uint32_t)(c->ld_blocks_host.size() / 2),
                                      P<char>(c->text), c->stream));
    prof_end(c, "ld_matrix");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->text_bytes = cells;
    if (cell_bytes) *cell_bytes = cells;
    return VCFXG_OK;
}

int vcfxg_selftest_mfma_i8(vcfxg_ctx *c, int *mismatches) {
    if (!c || !mismatches) return VCFXG_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<int8_t> A(32 * 32), B(32 * 32);
    for (int i = 0; i < 32 * 32; i++) {
        A[i] = (int8_t)((i * 7 + 3) % 5 - 2);
        B[i] = (int8_t)((i * 11 + 1) % 7 - 3);
    }
    int r = ensure(c, c->scan_tmp, 8192);
    if (r) return r;
    char *d = P<char>(c->scan_tmp);
    HIPCHK(c, hipMemcpyAsync(d, A.data(), 1024, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d + 1024, B.data(), 1024, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, vcfxg::launch_mfma_i8_selftest((int8_t *)d, (int8_t *)(d + 1024), (int *)(d + 2048), c->stream));
    std::vector<int> C(32 * 32);
    HIPCHK(c, hipMemcpyAsync(C.data(), d + 2048, 4096, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int bad = 0;
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            int s = 0;
            for (int k = 0; k < 32; k++) s += A[i * 32 + k] * B[j * 32 + k];
            bad += s != C[i * 32 + j];
        }
    *mismatches = bad;
    return VCFXG_OK;
}

int vcfxg_selftest_mfma_fp4(vcfxg_ctx *c, int *mismatches) {
    if (!c || !mismatches) return VCFXG_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    // dosages 0..2 in a 32x64 A and an asymmetric 32x64 B, packed e2m1 two per byte
    std::vector<int> A(32 * 64), B(32 * 64);
    for (int i = 0; i < 32 * 64; i++) {
        A[i] = (i * 7 + 3) % 3;
        B[i] = (i * 11 + i / 64 + 1) % 3;
    }
    std::vector<uint8_t> Ap(1024), Bp(1024);
    for (int i = 0; i < 1024; i++) {
        Ap[i] = (uint8_t)((2 * A[2 * i]) | ((2 * A[2 * i + 1]) << 4));
        Bp[i] = (uint8_t)((2 * B[2 * i]) | ((2 * B[2 * i + 1]) << 4));
    }
    int r = ensure(c, c->scan_tmp, 8192);
    if (r) return r;
    char *d = P<char>(c->scan_tmp);
    HIPCHK(c, hipMemcpyAsync(d, Ap.data(), 1024, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d + 1024, Bp.data(), 1024, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, vcfxg::launch_mfma_f4_selftest((uint8_t *)d, (uint8_t *)(d + 1024), (float *)(d + 2048), c->stream));
    std::vector<float> C(32 * 32);
    HIPCHK(c, hipMemcpyAsync(C.data(), d + 2048, 4096, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int bad = 0;
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            int sum = 0;
            for (int k = 0; k < 64; k++) sum += A[i * 64 + k] * B[j * 64 + k];
            bad += (float)sum != C[i * 32 + j];
        }
    *mismatches = bad;
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

int vcfxg_shard_cuts(const char *data, size_t n, size_t lo, int world, uint64_t *cuts) {
    if ((!data && n) || world < 1 || !cuts || lo > n) return VCFXG_E_ARG;
    cuts[0] = lo;
    for (int i = 1; i < world; i++) {
        size_t p = lo + (size_t)((unsigned __int128)(n - lo) * (unsigned)i / (unsigned)world);
        if (p < cuts[i - 1]) p = cuts[i - 1];
        if (p > lo && p < n && data[p - 1] != '\n') {
            const void *nl = memchr(data + p, '\n', n - p);
            p = nl ? (size_t)((const char *)nl - data) + 1 : n;
        }
        cuts[i] = p < n ? p : n;
    }
    cuts[world] = n;
    return VCFXG_OK;
}

// ---- rank cliques: the count all-reduce of the in-process multi-GPU drop-in ------------------
// RCCL comes from librccl at run time (dlopen: a single-GPU process never loads it).  rccl.h is
// included for its declarations only: the function pointer types and the enum values below are
// checked against it at compile time (no link dependency).
namespace {
typedef decltype(&ncclCommInitAll) nccl_init_all_f;
typedef decltype(&ncclAllReduce) nccl_allreduce_f;
typedef decltype(&ncclCommDestroy) nccl_destroy_f;
static_assert(ncclUint64 == 5 && ncclSum == 0 && ncclSuccess == 0, "rccl.h enum values");
constexpr size_t kCommSlots = 64;  // u64 values per all-reduce
}  // namespace

struct vcfxg_comm {
    int n = 0;
    std::vector<vcfxg_ctx *> ctx;
    // RCCL
    void *lib = nullptr;
    nccl_allreduce_f allreduce = nullptr;
    nccl_destroy_f destroy = nullptr;
    std::vector<ncclComm_t> comms;
    std::vector<uint64_t *> dbuf;  // per rank: kCommSlots u64 on its device
    // host side: every all-reduce is first a host reduction + vote of all ranks (the RCCL result
    // is checked against it, and no rank enters the collective unless every rank staged its values)
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0, failed = 0;
    bool result_failed = false;
    std::vector<uint64_t> acc, result;
    uint64_t rccl_calls = 0, rccl_mismatch = 0;
};

int vcfxg_comm_init(vcfxg_ctx *const *ctxs, int n, vcfxg_comm **out) {
    if (!ctxs || n < 1 || !out) return VCFXG_E_ARG;
    vcfxg_comm *c = new vcfxg_comm;
    c->n = n;
    c->ctx.assign(ctxs, ctxs + n);
    std::vector<int> dev(n);
    bool distinct = n > 1;
    for (int r = 0; r < n; r++) {
        if (!ctxs[r]) {
            delete c;
            return VCFXG_E_ARG;
        }
        dev[r] = ctxs[r]->device;
        for (int q = 0; q < r; q++) distinct = distinct && dev[q] != dev[r];
    }
    // RCCL over n distinct devices; VCFX_RCCL=1 also forms a one-rank clique (a one-GPU box runs
    // the whole RCCL path: init, the collective on the rank's stream, destroy); VCFX_RCCL=0 never.
    // RCCL cannot put two ranks on one device, so ranks sharing one reduce on the host.
    const char *e = getenv("VCFX_RCCL");
    const bool want = (distinct && !(e && e[0] == '0')) || (n == 1 && e && e[0] == '1');
    if (want) {
        c->lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!c->lib) c->lib = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        nccl_init_all_f init = c->lib ? (nccl_init_all_f)dlsym(c->lib, "ncclCommInitAll") : nullptr;
        c->allreduce = c->lib ? (nccl_allreduce_f)dlsym(c->lib, "ncclAllReduce") : nullptr;
        c->destroy = c->lib ? (nccl_destroy_f)dlsym(c->lib, "ncclCommDestroy") : nullptr;
        c->comms.assign(n, nullptr);
        if (!init || !c->allreduce || !c->destroy || init(c->comms.data(), n, dev.data()) != ncclSuccess) {
            if (c->lib) dlclose(c->lib);
            c->lib = nullptr;
            c->allreduce = nullptr;
            c->comms.clear();
            ctxs[0]->err = "vcfxg_comm_init: RCCL clique over " + std::to_string(n) + " devices failed";
            delete c;
            return VCFXG_E_HIP;
        }
        c->dbuf.assign(n, nullptr);
        for (int r = 0; r < n; r++) {
            if (hipSetDevice(dev[r]) != hipSuccess || hipMalloc((void **)&c->dbuf[r], kCommSlots * 8) != hipSuccess) {
                ctxs[r]->err = "vcfxg_comm_init: no device buffer for the all-reduce";
                vcfxg_comm_destroy(c);
                return VCFXG_E_HIP;
            }
        }
    }
    c->acc.assign(kCommSlots, 0);
    c->result.assign(kCommSlots, 0);
    *out = c;
    return VCFXG_OK;
}

int vcfxg_comm_uses_rccl(const vcfxg_comm *c) { return c && c->allreduce ? 1 : 0; }

const char *vcfxg_last_schedule(const vcfxg_ctx *c) { return c ? c->last_schedule : ""; }
uint64_t vcfxg_bgzf_handed_over(const vcfxg_ctx *c) { return c ? c->bgz_handed : 0; }

int vcfxg_comm_rccl_stats(vcfxg_comm *c, uint64_t *calls, uint64_t *mismatches) {
    if (!c) return VCFXG_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (calls) *calls = c->rccl_calls;
    if (mismatches) *mismatches = c->rccl_mismatch;
    return VCFXG_OK;
}

int vcfxg_comm_allreduce_u64(vcfxg_comm *c, int rank, uint64_t *vals, size_t count) {
    if (!c || rank < 0 || rank >= c->n || (!vals && count) || count > kCommSlots) return VCFXG_E_ARG;
    vcfxg_ctx *x = c->ctx[rank];
    // 1. stage the values on the rank's device (RCCL); a rank whose device call fails votes "no"
    bool ok = true;
    if (c->allreduce) {
        ok = hipSetDevice(x->device) == hipSuccess &&
             hipMemcpyAsync(c->dbuf[rank], vals, 8 * count, hipMemcpyHostToDevice, x->stream) == hipSuccess &&
             hipStreamSynchronize(x->stream) == hipSuccess;
        if (!ok) x->err = "vcfxg_comm_allreduce_u64: staging the values on the device failed";
    }
    // 2. host reduction + vote: the last rank to arrive publishes the sums of this generation
    std::vector<uint64_t> host(count);
    bool any_failed;
    {
        std::unique_lock<std::mutex> lk(c->mu);
        const uint64_t g = c->gen;
        for (size_t k = 0; k < count; k++) c->acc[k] += vals[k];
        if (!ok) c->failed++;
        if (++c->arrived == c->n) {
            c->result = c->acc;
            c->result_failed = c->failed != 0;
            std::fill(c->acc.begin(), c->acc.end(), 0);
            c->arrived = c->failed = 0;
            c->gen++;
            c->cv.notify_all();
        } else {
            c->cv.wait(lk, [&] { return c->gen != g; });
        }
        std::copy(c->result.begin(), c->result.begin() + (long)count, host.begin());
        any_failed = c->result_failed;
    }
    if (!c->allreduce) {
        std::copy(host.begin(), host.end(), vals);
        return VCFXG_OK;
    }
    if (any_failed) {  // no rank enters the collective; the host sums stand, the failure is reported
        std::copy(host.begin(), host.end(), vals);
        if (ok) x->err = "vcfxg_comm_allreduce_u64: another rank failed to stage its values";
        return VCFXG_E_HIP;
    }
    // 3. RCCL over the devices (xGMI), on the rank's own stream; checked against the host sums
    std::vector<uint64_t> dv(count);
    if (c->allreduce(c->dbuf[rank], c->dbuf[rank], count, ncclUint64, ncclSum, c->comms[rank], x->stream) !=
        ncclSuccess) {
        x->err = "ncclAllReduce failed";
        std::copy(host.begin(), host.end(), vals);
        return VCFXG_E_HIP;
    }
    if (hipMemcpyAsync(dv.data(), c->dbuf[rank], 8 * count, hipMemcpyDeviceToHost, x->stream) != hipSuccess ||
        hipStreamSynchronize(x->stream) != hipSuccess) {
        x->err = "vcfxg_comm_allreduce_u64: reading the RCCL sums back failed";
        std::copy(host.begin(), host.end(), vals);
        return VCFXG_E_HIP;
    }
    const bool same = dv == host;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->rccl_calls++;
        if (!same) c->rccl_mismatch++;
    }
    std::copy(host.begin(), host.end(), vals);
    if (!same) {
        x->err = "vcfxg_comm_allreduce_u64: the RCCL sums differ from the host reduction";
        return VCFXG_E_HIP;
    }
    return VCFXG_OK;
}

void vcfxg_comm_destroy(vcfxg_comm *c) {
    if (!c) return;
    for (size_t r = 0; r < c->comms.size(); r++)
        if (c->comms[r] && c->destroy) c->destroy(c->comms[r]);
    for (size_t r = 0; r < c->dbuf.size(); r++)
        if (c->dbuf[r]) {
            (void)hipSetDevice(c->ctx[r]->device);
            (void)hipFree(c->dbuf[r]);
        }
    // (librccl stays loaded: its teardown threads may still be unwinding)
    delete c;
}

int vcfxg_fetch_text_range(vcfxg_ctx *c, uint64_t offset, size_t n, void *host) {
    if (!c || (!host && n)) return VCFXG_E_ARG;
    if (offset > c->text_bytes || n > c->text_bytes - offset) return VCFXG_E_ARG;
    if (!n) return VCFXG_OK;
    HIPCHK(c, hipMemcpyAsync(host, P<char>(c->text) + offset, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

int vcfxg_fetch_lines(vcfxg_ctx *c, uint64_t first, uint64_t count, int32_t *alt, int32_t *total, uint8_t *status) {
    if (!c) return VCFXG_E_ARG;
    if (!c->indexed) return VCFXG_E_STATE;
    DENSE(c);
    if (first + count > c->n_lines) return VCFXG_E_ARG;
    if (!count) return VCFXG_OK;
    if (alt) HIPCHK(c, hipMemcpyAsync(alt, P<int32_t>(c->alt) + first, 4 * count, hipMemcpyDeviceToHost, c->stream));
    if (total) HIPCHK(c, hipMemcpyAsync(total, P<int32_t>(c->tot) + first, 4 * count, hipMemcpyDeviceToHost, c->stream));
    if (status) HIPCHK(c, hipMemcpyAsync(status, P<uint8_t>(c->status) + first, count, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VCFXG_OK;
}

}  // extern "C"
