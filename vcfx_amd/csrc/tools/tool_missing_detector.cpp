// VCFX_missing_detector drop-in (a per-sample GT predicate on the record
// path): the reference CLI (VCFX_missing_detector.cpp:943-997) on top of vcfxg_missing_region.
// The GPU tests every record's samples; the host writes the records in order, straight from
// the input bytes, splicing "MISSING_GENOTYPES=1" into the INFO field of the flagged ones.
#include <getopt.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "emit.h"
#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

// displayHelp :916-938
const char *kHelp =
    "VCFX_missing_detector v2.0 - Extreme-performance missing genotype detector\n\n"
    "Usage:\n"
    "  VCFX_missing_detector [OPTIONS] [input.vcf]\n"
    "  VCFX_missing_detector [OPTIONS] < input.vcf > flagged.vcf\n\n"
    "Options:\n"
    "  -i, --input FILE   Input VCF file (uses memory-mapping for best performance)\n"
    "  -t, --threads N    Number of threads (default: auto)\n"
    "  -q, --quiet        Suppress informational messages\n"
    "  -h, --help         Display this help message and exit\n"
    "  -v, --version      Show program version and exit\n\n"
    "Description:\n"
    "  Detects variants with missing sample genotypes and flags them\n"
    "  with 'MISSING_GENOTYPES=1' in the INFO field.\n\n"
    "Performance:\n"
    "  - Memory-mapped I/O: Use -i flag for extreme speed\n"
    "  - SIMD-accelerated '.' character search (AVX2/SSE2/NEON)\n"
    "  - Multi-threaded chunk processing\n"
    "  - Zero-copy output for lines without missing genotypes\n\n"
    "Example:\n"
    "  VCFX_missing_detector -i input.vcf > flagged.vcf\n"
    "  VCFX_missing_detector < input.vcf > flagged.vcf\n";

const char kTag[] = "MISSING_GENOTYPES=1";
const char kSemiTag[] = ";MISSING_GENOTYPES=1";

// the end of the leading '#' lines within the host bytes (both modes copy them; the file
// pre-scan starts after them)
size_t leading_headers(const Input &in) {
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;
    size_t ds = 0;
    while (p < end && *p == '#') {
        const char *q = p;
        if (!next_line(q, end, ls, le) || le == end) break;  // (an unterminated line: the device's)
        p = q;
        ds = (size_t)(p - in.p);
    }
    return ds;
}

// the file path's closing lines (processMmapZeroCopy :575-589): the pre-scan's fast path
// (no '.' in any sample column) reports its line count, the per-line pass its flagged share
std::string md_summary(bool fast, uint64_t lines, uint64_t data_lines, uint64_t flagged) {
    if (fast)
        return "Fast path: No '.' in sample columns (scan complete)\nProcessed " + std::to_string(lines) +
               " variants, 0 with missing genotypes (0%)\n";
    const double pct = data_lines ? 100.0 * (double)flagged / (double)data_lines : 0.0;
    char b[160];
    snprintf(b, sizeof b, "Processed %llu variants, %llu with missing genotypes (%g%%)\n",
             (unsigned long long)data_lines, (unsigned long long)flagged, pct);
    return b;
}

// file: processMmapZeroCopy :450-589; stdin: detectMissingGenotypes :860-911.  Returns false
// on a device error (already reported).
bool run_md(const Input &in, bool file, const char *path, bool quiet, int out_fd, Out &err) {
    if (file && !quiet) {
        char b[64];
        snprintf(b, sizeof b, " (%zu MB)\n", reported_size(in) / (1024 * 1024));
        err.put(std::string("Processing ") + path + b);
        err.flush();
    }
    shard_records_begin(err);
    LineEmitter em(in.p, in.host_n, out_fd);
    const size_t ds = leading_headers(in);
    // the leading '#' lines: copied (file) / each followed by '\n' (stdin: getline); a multi-GPU
    // rank > 0 leaves them to rank 0
    if (file) {
        if (!view_skip_header()) em.bytes(in.p, in.p + ds);
    } else {
        const char *p = in.p, *end = in.p + ds, *ls, *le;
        while (next_line(p, end, ls, le)) em.line(ls, le);
    }
    vcfxg_summary s{};
    uint64_t nl = 0;
    vcfxg_ctx *g = nullptr;
    if (ds < in.n) {
        g = gpu(err.fd);
        if (!g) return false;
        if (!load_input(g, in, err.fd) ||
            !gpu_ok(g, vcfxg_missing_region(g, ds, file ? VCFXG_MODE_FILE : VCFXG_MODE_STDIN, &s), "missing_region",
                    err.fd))
            return false;
        nl = s.n_lines;
    }
    // a multi-GPU rank: the summary over every rank (the fast path's message only when no rank
    // saw a '.'; a rank's own fast path writes the same bytes as its per-line pass in file mode)
    // (the input's last byte: a shard view's tail, the host bytes, or -- a device-only input, the
    // records of a pipe or of BGZF inflated on the device -- one byte fetched from the device)
    char lastb = 0;
    if (in.n == 0) {
    } else if (in.tail) lastb = in.tail[in.n - in.host_n - 1];
    else if (in.host_n == in.n) lastb = in.p[in.n - 1];
    else if (!gpu_ok(g, vcfxg_input_fetch(g, in.n - 1, 1, &lastb), "input_fetch", err.fd)) return false;
    const bool last_nl = lastb == '\n';
    const uint64_t lines = nl - (nl && !last_nl ? 1 : 0);
    if (file && t_shard) {
        t_shard->cnt[0] = lines;
        t_shard->cnt[1] = s.data_lines;
        t_shard->cnt[2] = s.rows;
        t_shard->cnt[3] = s.general_records;
        if (!quiet && t_shard->rank == 0)
            t_shard->summary = [](const uint64_t *c) { return md_summary(c[3] == 0, c[0], c[1], c[2]); };
    }
    if (file && s.general_records == 0) {
        // the pre-scan saw no '.' in any sample column: the input as it is
        em.bytes(in.p + ds, in.p + in.host_n);
        em.finish();
        if (in.tail) write_all(out_fd, in.tail, in.n - in.host_n);
        else if (in.host_n < in.n) {  // a device-only input: read back window by window
            LineSource src(in, g, em);
            for (uint64_t a = in.host_n; a < in.n;) {
                const uint64_t b = std::min<uint64_t>(in.n, a + window_bytes() - 1);
                const char *q = src.at(a, b);
                if (!q) break;
                em.bytes(q, q + (b - a));
                a = b;
            }
            em.finish();
            if (!src.ok) return gpu_ok(g, VCFXG_E_HIP, "input_fetch", err.fd);
        }
        if (!quiet && !t_shard) err.put(md_summary(true, lines, 0, 0));
        return true;
    }
    if (nl) {
        std::vector<uint64_t> ends(nl);
        std::vector<uint8_t> st(nl);
        std::vector<int32_t> is(nl), ie(nl);
        if (!gpu_ok(g, vcfxg_line_ends(g, 0, nl, ends.data()), "line_ends", err.fd) ||
            !gpu_ok(g, vcfxg_fetch_lines(g, 0, nl, is.data(), ie.data(), st.data()), "fetch_lines", err.fd))
            return false;
        LineSource src(in, g, em);
        uint64_t prev = ds;
        for (uint64_t i = 0; i < nl; i++) {
            const uint8_t v = st[i];
            const char *a = src.at(prev, ends[i]);
            if (!a) break;
            const char *b = a + (ends[i] - prev);
            if (v == VCFXG_LINE_MISSING) {
                const char *ae = (file && b > a && b[-1] == '\r') ? b - 1 : b;
                const char *i0 = a + is[i], *i1 = a + ie[i];
                em.bytes(a, i0);
                if (i1 == i0 || (i1 - i0 == 1 && *i0 == '.')) em.raw(kTag, sizeof kTag - 1);
                else {
                    em.bytes(i0, i1);
                    if (i1[-1] == ';') em.raw(kTag, sizeof kTag - 1);
                    else em.raw(kSemiTag, sizeof kSemiTag - 1);
                }
                em.bytes(i1, ae);
                em.raw("\n", 1);
            } else if (file) em.bytes(a, ends[i] < in.n ? b + 1 : b);  // the line's bytes as they are
            else if (b == a) em.raw("\n", 1);
            else em.line(a, b);
            prev = ends[i] + 1;
        }
        if (!src.ok) {
            em.finish();
            return gpu_ok(g, VCFXG_E_HIP, "input_fetch", err.fd);
        }
    }
    em.finish();
    if (file && !quiet && !t_shard) err.put(md_summary(false, lines, s.data_lines, s.rows));
    return true;
}

}  // namespace

extern "C" int vcfx_tool_missing_detector(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    Out out(out_fd), err(err_fd);
    // run :943-997 (no vcfx::handle_common_flags: -h / -v go through getopt)
    const char *input = nullptr;
    bool quiet = false;
    static struct option lo[] = {{"input", required_argument, nullptr, 'i'},
                                 {"threads", required_argument, nullptr, 't'},
                                 {"quiet", no_argument, nullptr, 'q'},
                                 {"help", no_argument, nullptr, 'h'},
                                 {"version", no_argument, nullptr, 'v'},
                                 {nullptr, 0, nullptr, 0}};
    GetoptStderr gs(err);
    optind = 0;
    int opt, rc = -1;
    while (rc < 0 && (opt = getopt_long(argc, argv, "i:t:qhv", lo, nullptr)) != -1) {
        switch (opt) {
            case 'i': input = optarg; break;
            case 't': break;  // the reference's scan threads: no effect on the output
            case 'q': quiet = true; break;
            case 'h': out.put(kHelp); rc = 0; break;
            case 'v': out.put("VCFX_missing_detector v2.0\n"); rc = 0; break;
            default: out.put(kHelp); rc = 1; break;
        }
    }
    gs.done();
    if (rc >= 0) return rc;
    if (!input && gs.next < argc) input = argv[gs.next];
    Input in;
    in.gzip_ok = true;  // .vcf.gz / BGZF input is inflated (VCFX_GZIP=0: off)
    in.bgzf_device = true;  // BGZF members inflated on the device (the records stay there)
    if (input) {
        phase("start");
        if (!in.open_file(input)) {
            err.put(std::string("Error: Cannot open file: ") + input + "\n");
            return 1;
        }
        if (!in.decompress(err.fd)) return 1;
        out.flush();
        return run_md(in, true, input, quiet, out_fd, err) ? 0 : 1;
    }
    phase("start");
    in.read_fd(in_fd, /*host_copy=*/false);  // records are read back from the device
    if (!in.decompress(err.fd)) return 1;
    phase("stdin read");
    out.flush();
    return run_md(in, false, nullptr, quiet, out_fd, err) ? 0 : 1;
}
