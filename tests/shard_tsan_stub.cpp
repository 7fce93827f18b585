// shard_tsan_stub.cpp -- test infrastructure: a host-only stand-in for libvcfx_gpu so the
// in-process multi-GPU runner (vcfx_amd/csrc/tools/tool_shard_main.cpp) can be built and run
// under ThreadSanitizer on a machine without a GPU (`make sanitize`, tests/test_sanitize.py).
//
// Built together with the REAL host sources -- tool_shard_main.cpp (rank threads, clique, the
// ordered output writer), tool_allele_freq_calc.cpp (its getopt phase under the getopt lock, the
// thread-local ShardRank overrides, shard_records_begin, the count reduction) and hostio.cpp /
// gz.cpp (file views, ingest).  Only the vcfxg_* entry points those sources call are replaced:
//   - a "device" is a host byte buffer; vcfxg_allele_freq_region writes, for every data line of
//     the region, "CHROM..ALT\t<tabs in the line>\n" (a deterministic function of the line, so a
//     sharded run must equal the single-context run byte for byte: the runner is under test,
//     not the AF arithmetic, which the GPU tests pin against the reference);
//   - vcfxg_shard_cuts restates the cut rule of vcfxg_api.hip (VCFX_allele_counter.cpp:889-901);
//   - the rank clique is the host reduction (last rank to arrive publishes the sums);
//   - VCFX_STUB_DEVICES sets the device count (default 2), VCFX_STUB_FAIL_RANK=r makes the
//     context of device r fail to open (a rank that stops before its records).
// Built with -DVCFX_STUB_DISCARD (build/bin/vcfx_pipe_ceiling, tools/microbench/pipe_ceiling.cpp)
// the ingest keeps nothing: the drop-in's own stdin reader with the device stage stubbed, the
// pipe ceiling bench.py's e2e leg quotes.
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

#include "tools.h"
#include "vcfx_gpu.h"

struct vcfxg_ctx {
    int device = 0;
    std::string input, text, err;
    bool ingesting = false;
};

extern "C" {

int vcfxg_device_count(int *n) {
    const char *e = getenv("VCFX_STUB_DEVICES");
    *n = e ? atoi(e) : 2;
    return VCFXG_OK;
}

int vcfxg_open(int device, vcfxg_ctx **out) {
    const char *f = getenv("VCFX_STUB_FAIL_RANK");
    if (f && atoi(f) == device) return VCFXG_E_NODEV;
    *out = new vcfxg_ctx;
    (*out)->device = device;
    return VCFXG_OK;
}

void vcfxg_close(vcfxg_ctx *c) { delete c; }

const char *vcfxg_last_error(const vcfxg_ctx *c) { return c ? c->err.c_str() : "no context"; }

int vcfxg_ingest_begin(vcfxg_ctx *c, size_t size_hint) {
    c->input.clear();
#ifndef VCFX_STUB_DISCARD
    c->input.reserve(size_hint);
#else
    (void)size_hint;
#endif
    c->ingesting = true;
    return VCFXG_OK;
}

int vcfxg_ingest(vcfxg_ctx *c, const char *host, size_t n, int is_final_chunk) {
    if (!c->ingesting) return VCFXG_E_STATE;
#ifndef VCFX_STUB_DISCARD
    c->input.append(host, n);
#else
    (void)host, (void)n;
#endif
    if (is_final_chunk) c->ingesting = false;
    return VCFXG_OK;
}

int vcfxg_ingest_wait(vcfxg_ctx *, size_t) { return VCFXG_OK; }
// (no device inflate in the stand-in: the runner's gzip inputs are unsharded anyway)
int vcfxg_ingest_bgzf(vcfxg_ctx *, const void *, size_t, const vcfxg_bgzf_member *, size_t, const char *, size_t,
                      uint64_t *) {
    return VCFXG_E_STATE;
}
int vcfxg_bgzf_stage(vcfxg_ctx *, const void *, size_t, size_t, size_t) { return VCFXG_E_STATE; }
int vcfxg_bgzf_inflate(vcfxg_ctx *, const vcfxg_bgzf_member *, size_t) { return VCFXG_E_STATE; }

int vcfxg_load_host(vcfxg_ctx *c, const char *host, size_t n) {
    vcfxg_ingest_begin(c, n);
    return vcfxg_ingest(c, host, n, 1);
}

int vcfxg_host_alloc(vcfxg_ctx *, size_t bytes, void **out) {
    *out = malloc(bytes);
    return *out ? VCFXG_OK : VCFXG_E_NOMEM;
}

void vcfxg_host_free(vcfxg_ctx *, void *p) { free(p); }

int vcfxg_allele_freq_region(vcfxg_ctx *c, size_t data_start, int, vcfxg_summary *out) {
    memset(out, 0, sizeof *out);
    c->text.clear();
    const std::string &s = c->input;
    size_t p = data_start;
    while (p < s.size()) {
        size_t e = s.find('\n', p);
        if (e == std::string::npos) e = s.size();
        if (e > p && s[p] != '#') {
            out->data_lines++;
            size_t tabs = 0, t5 = std::string::npos;
            for (size_t k = p; k < e; k++)
                if (s[k] == '\t' && ++tabs == 5) t5 = k;
            if (tabs < 8) {
                out->warn_lines++;
            } else {
                out->rows++;
                c->text.append(s, p, t5 - p);
                c->text += "\t" + std::to_string(tabs) + "\n";
            }
        }
        p = e + 1;
    }
    out->n_lines = out->data_lines;
    out->text_bytes = c->text.size();
    return VCFXG_OK;
}

int vcfxg_fetch_text(vcfxg_ctx *c, char *host, size_t cap) {
    if (cap < c->text.size()) return VCFXG_E_CAP;
    memcpy(host, c->text.data(), c->text.size());
    return VCFXG_OK;
}

int vcfxg_fetch_text_range(vcfxg_ctx *c, uint64_t offset, size_t n, void *host) {
    if (offset > c->text.size() || n > c->text.size() - offset) return VCFXG_E_ARG;
    memcpy(host, c->text.data() + offset, n);
    return VCFXG_OK;
}

int vcfxg_shard_cuts(const char *data, size_t n, size_t lo, int world, uint64_t *cuts) {
    if (world < 1 || lo > n) return VCFXG_E_ARG;
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

struct vcfxg_comm {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0;
    std::vector<uint64_t> acc = std::vector<uint64_t>(64, 0), result = std::vector<uint64_t>(64, 0);
};

int vcfxg_comm_init(vcfxg_ctx *const *ctxs, int n, vcfxg_comm **out) {
    if (!ctxs || n < 1) return VCFXG_E_ARG;
    *out = new vcfxg_comm;
    (*out)->n = n;
    return VCFXG_OK;
}

int vcfxg_comm_allreduce_u64(vcfxg_comm *c, int rank, uint64_t *vals, size_t count) {
    if (!c || rank < 0 || rank >= c->n || count > 64) return VCFXG_E_ARG;
    std::unique_lock<std::mutex> lk(c->mu);
    const uint64_t g = c->gen;
    for (size_t k = 0; k < count; k++) c->acc[k] += vals[k];
    if (++c->arrived == c->n) {
        c->result = c->acc;
        std::fill(c->acc.begin(), c->acc.end(), 0);
        c->arrived = 0;
        c->gen++;
        c->cv.notify_all();
    } else {
        c->cv.wait(lk, [&] { return c->gen != g; });
    }
    for (size_t k = 0; k < count; k++) vals[k] = c->result[k];
    return VCFXG_OK;
}

void vcfxg_comm_destroy(vcfxg_comm *c) { delete c; }

}  // extern "C"

// the dispatch of tool_dispatch.cpp for the one tool linked in
namespace vcfxh {
std::recursive_mutex &getopt_mutex() {
    static std::recursive_mutex m;
    return m;
}
}  // namespace vcfxh

#ifndef VCFX_STUB_DISCARD  // (the pipe ceiling has its own main and no tool)
extern "C" int vcfx_tool_main(const char *tool, int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    const char *t = strrchr(tool, '/');
    t = t ? t + 1 : tool;
    if (!strcmp(t, "VCFX_allele_freq_calc")) return vcfx_tool_allele_freq_calc(argc, argv, in_fd, out_fd, err_fd);
    return -100;
}

// shard_tsan_stub TOOL ARGS...  (VCFX_NGPU=N: the in-process multi-GPU runner)
int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const char *e = getenv("VCFX_NGPU");
    const int ngpu = e ? atoi(e) : 1;
    if (ngpu > 1) return vcfx_tool_main_sharded(argv[1], argc - 1, argv + 1, 0, 1, 2, ngpu);
    return vcfx_tool_main(argv[1], argc - 1, argv + 1, 0, 1, 2);
}
#endif
