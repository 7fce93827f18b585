// VCFX_ld_calculator drop-in: the reference CLI (VCFXLDCalculator::run,
// VCFX_ld_calculator.cpp:1084-1209, main :1219-1225) on top of the vcfxg LD engine.
// Streaming mode (default): every window pair's r^2 is computed on the GPU (int8 MFMA
// sums, exact fp64 epilogue) and the kept lines are formatted on the device in the
// reference's order; the host writes them chunk by chunk.  Matrix mode: tool_ld_matrix.cpp.
#include <errno.h>
#include <getopt.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "emit.h"
#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace vcfxh {
const char *kLdHelp =
    "VCFX_ld_calculator: Calculate pairwise LD (r^2) for variants in a VCF region.\n"
    "Version 2.0 - Extreme-performance with mmap, SIMD, and multi-threading.\n\n"
    "Usage:\n"
    "  VCFX_ld_calculator [options] < input.vcf\n"
    "  VCFX_ld_calculator [options] -i input.vcf\n\n"
    "Options:\n"
    "  -i, --input FILE          Input VCF file (uses memory-mapping for best performance)\n"
    "  -r, --region <chr:s-e>    Only compute LD for variants in [start, end] on 'chr'\n"
    "  -w, --window <N>          Window size in variants (default: 1000)\n"
    "  -d, --max-distance <BP>   Max base-pair distance between pairs (0=unlimited)\n"
    "  -t, --threshold <R2>      Only output pairs with r\xc2\xb2 >= threshold (default: 0.0)\n"
    "  -n, --threads <N>         Number of threads (default: auto)\n"
    "  -m, --matrix              Use matrix mode (MxM output) instead of streaming\n"
    "                            WARNING: O(M\xc2\xb2) time - avoid for >10K variants\n"
    "  -q, --quiet               Suppress informational messages\n"
    "  -h, --help                Show this help message\n"
    "  -v, --version             Show program version\n\n"
    "Modes:\n"
    "  Default (streaming): Outputs LD pairs incrementally using a sliding window.\n"
    "                       Memory: O(window * samples) - constant for any file size.\n"
    "                       Time: O(M * window) - linear in variant count.\n"
    "  Matrix mode:         Produces an MxM matrix of all pairwise r\xc2\xb2 values.\n"
    "                       Memory: O(M * samples) where M is number of variants.\n"
    "                       Time: O(M\xc2\xb2) - avoid for >10K variants!\n\n"
    "Performance:\n"
    "  - Memory-mapped I/O: Use -i flag for extreme speed\n"
    "  - SIMD-accelerated r\xc2\xb2 computation (NEON/AVX2/SSE2)\n"
    "  - Multi-threaded matrix computation\n"
    "  - Distance-based pruning with --max-distance\n\n"
    "Example:\n"
    "  # Fast streaming mode with file input\n"
    "  VCFX_ld_calculator -i input.vcf -w 500 -t 0.2 > ld_pairs.txt\n\n"
    "  # Streaming with distance limit (biology: LD decays with distance)\n"
    "  VCFX_ld_calculator -i input.vcf --max-distance 500000 > ld_pairs.txt\n\n"
    "  # Matrix mode (small regions only)\n"
    "  VCFX_ld_calculator -i input.vcf -m -r chr1:10000-20000 > ld_matrix.txt\n";

// std::stoi: strtol semantics (leading space, sign, partial parse) + int range
bool cxx_stoi(const char *s, long *out) {
    errno = 0;
    char *e;
    long v = strtol(s, &e, 10);
    if (e == s || errno == ERANGE || v < -2147483648L || v > 2147483647L) return false;
    *out = v;
    return true;
}

int ld_samples(const char *ls, const char *le) {  // numSamples from the #CHROM line
    int t = 0;
    for (const char *p = ls; p < le; p++) t += *p == '\t';
    return t >= 9 ? t - 8 : 0;
}
}  // namespace vcfxh

namespace {

struct LdOpts {
    bool matrix = false, quiet = false;
    int shard_rank = 0, shard_world = 1;  // --shard r/N (multi-GPU extension, vcfx_amd/shard.py)
    size_t window = 1000;
    double thr = 0.0;
    int maxd = 0;
    std::string region, input;
};

// parseRegion :448-463
bool parse_region(const std::string &r, std::string &chrom, int &s, int &e) {
    size_t c = r.find(':');
    if (c == std::string::npos) return false;
    size_t d = r.find('-', c + 1);
    if (d == std::string::npos) return false;
    long a, b;
    if (!cxx_stoi(r.substr(c + 1, d - c - 1).c_str(), &a) || !cxx_stoi(r.substr(d + 1).c_str(), &b)) return false;
    if (a > b) return false;
    chrom = r.substr(0, c);
    s = (int)a;
    e = (int)b;
    return true;
}

// computeLDStreamingMmap (:511-648) / computeLDStreaming (:864-987)
bool run_stream(const Input &in, bool mmap_mode, const LdOpts &o, const std::string &rchrom, bool has_region, int rs,
                int re, int out_fd, Out &err) {
    static const char kHead[] = "#VAR1_CHROM\tVAR1_POS\tVAR1_ID\tVAR2_CHROM\tVAR2_POS\tVAR2_ID\tR2\n";
    if (o.shard_rank == 0) write_all(out_fd, kHead, sizeof kHead - 1);
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;  // (device BGZF: the head on the host)
    bool found = false;
    int ns = 0;
    size_t data_start = in.n;
    while (next_line(p, end, ls, le)) {
        if (le == ls) continue;
        if (*ls == '#') {
            if (is_chrom_line(ls, (size_t)(le - ls))) {
                found = true;
                ns = ld_samples(ls, le);
                data_start = (size_t)(p - in.p);
                break;
            }
            continue;
        }
        if (mmap_mode) {
            if (!o.quiet) err.put("Error: data line before #CHROM\n");
        } else err.put("Error: encountered data line before #CHROM.\n");
        return true;
    }
    if (!found || data_start >= in.n) return true;
    vcfxg_ctx *g = gpu(err.fd);
    if (!g) return false;
    uint64_t nl = 0, M = 0;
    (void)nl;
    if (!load_input(g, in, err.fd) ||
        !gpu_ok(g, vcfxg_ld_prepare_region(g, data_start, ns, 1, rchrom.data(), rchrom.size(), has_region ? 1 : 0, rs,
                                           re, 0, &M),
                "ld_prepare", err.fd))
        return false;
    const uint64_t W = std::min<uint64_t>(o.window, M ? M : 1);
    // this shard's rows: equal shares of the window pairs (row j pairs with min(j, W) rows)
    uint64_t jb = 0, je = M;
    if (o.shard_world > 1) {
        auto cum = [&](uint64_t j) -> uint64_t {  // sum over rows k < j of min(k, W)
            return j <= W ? j * (j - 1) / 2 : W * (W + 1) / 2 + (j - W - 1) * W;
        };
        auto cut = [&](int r) -> uint64_t {
            if (r <= 0) return 0;
            if (r >= o.shard_world) return M;
            const long double target = (long double)cum(M) * r / o.shard_world;
            uint64_t lo = 0, hi = M;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                if ((long double)cum(mid) < target) lo = mid + 1;
                else hi = mid;
            }
            return std::min<uint64_t>(M, (lo + 255) / 256 * 256);
        };
        jb = cut(o.shard_rank);
        je = cut(o.shard_rank + 1);
    }
    // chunk rows so that a chunk holds at most ~16M candidate pairs
    uint64_t R = (16ull << 20) / std::max<uint64_t>(W, 1);
    R = std::max<uint64_t>(256, (R / 256) * 256);  // whole 256-variant fast blocks
    std::string text;
    for (uint64_t j0 = jb; j0 < je; j0 += R) {
        uint64_t np = 0, tb = 0;
        if (!gpu_ok(g, vcfxg_ld_stream_chunk(g, j0, std::min(j0 + R, je), W, o.thr, mmap_mode ? o.maxd : 0, &np, &tb),
                    "ld_stream_chunk", err.fd))
            return false;
        if (!tb) continue;
        text.resize(tb);
        if (!gpu_ok(g, vcfxg_fetch_text(g, &text[0], tb), "fetch", err.fd)) return false;
        write_all(out_fd, text.data(), tb);
    }
    return true;
}

}  // namespace

namespace vcfxh {
bool run_ld_matrix(const Input &in, bool mmap_mode, bool quiet, const std::string &rchrom, bool has_region, int rs,
                   int re, int out_fd, Out &err);
}

extern "C" int vcfx_tool_ld_calculator(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    Out out(out_fd), err(err_fd);
    if (flag_present(argc, argv, "--help", "-h")) {  // show_help -> run(--help) -> displayHelp
        out.put(kLdHelp);
        return 0;
    }
    if (flag_present(argc, argv, "--version", "-v")) {
        out.put("VCFX_ld_calculator version " VCFX_VERSION_STR "\n");
        return 0;
    }
    static struct option lo[] = {{"help", no_argument, 0, 'h'},       {"version", no_argument, 0, 'v'},
                                 {"input", required_argument, 0, 'i'},  {"region", required_argument, 0, 'r'},
                                 {"streaming", no_argument, 0, 's'},  {"matrix", no_argument, 0, 'm'},
                                 {"window", required_argument, 0, 'w'}, {"threshold", required_argument, 0, 't'},
                                 {"threads", required_argument, 0, 'n'}, {"max-distance", required_argument, 0, 'd'},
                                 {"quiet", no_argument, 0, 'q'},       {"shard", required_argument, 0, 'S'},
                                 {0, 0, 0, 0}};
    LdOpts o;
    bool show = false;
    GetoptStderr gs(err);
    optind = 0;
    for (;;) {
        int c = getopt_long(argc, argv, "hvi:r:smw:t:n:d:q", lo, nullptr);
        if (c == -1) break;
        switch (c) {
        case 'h': show = true; break;
        case 'v': gs.done(); out.put("VCFX_ld_calculator v2.0\n"); return 0;
        case 'i': o.input = optarg; break;
        case 'r': o.region = optarg; break;
        case 's': o.matrix = false; break;
        case 'm': o.matrix = true; break;
        case 'w': {
            errno = 0;
            char *e;
            unsigned long v = strtoul(optarg, &e, 10);  // std::stoul
            if (e == optarg || errno == ERANGE) {
                gs.done();
                err.put(std::string("Error: Invalid window size '") + optarg + "'\n");
                return 1;
            }
            o.window = v == 0 ? 1 : v;
            break;
        }
        case 't': {
            errno = 0;
            char *e;
            double v = strtod(optarg, &e);  // std::stod
            if (e == optarg || errno == ERANGE) {
                gs.done();
                err.put(std::string("Error: Invalid threshold '") + optarg + "'\n");
                return 1;
            }
            if (v < 0.0) v = 0.0;
            if (v > 1.0) v = 1.0;
            o.thr = v;
            break;
        }
        case 'n': {
            long v;
            if (!cxx_stoi(optarg, &v)) {
                gs.done();
                err.put(std::string("Error: Invalid thread count '") + optarg + "'\n");
                return 1;
            }
            break;
        }
        case 'd': {
            long v;
            if (!cxx_stoi(optarg, &v)) {
                gs.done();
                err.put(std::string("Error: Invalid max-distance '") + optarg + "'\n");
                return 1;
            }
            o.maxd = v < 0 ? 0 : (int)v;
            break;
        }
        case 'q': o.quiet = true; break;
        case 'S':  // --shard r/N: rows of shard r of N (streaming); other shards print nothing else
            if (sscanf(optarg, "%d/%d", &o.shard_rank, &o.shard_world) != 2 || o.shard_world < 1 ||
                o.shard_rank < 0 || o.shard_rank >= o.shard_world) {
                gs.done();
                err.put(std::string("Error: Invalid shard '") + optarg + "'\n");
                return 1;
            }
            break;
        default: show = true;
        }
    }
    gs.done();
    if (gs.next < argc && o.input.empty()) o.input = argv[gs.next];
    if (show) {
        out.put(kLdHelp);
        return 0;
    }
    std::string rchrom;
    int rs = 0, re = 0;
    bool has_region = false;
    if (!o.region.empty()) {
        if (!parse_region(o.region, rchrom, rs, re)) {
            err.put("Error parsing region '" + o.region + "'. Use e.g. chr1:10000-20000\n");
            return 1;
        }
        has_region = !rchrom.empty();
    }
    out.flush();
    Input in;
    in.gzip_ok = true;  // .vcf.gz / BGZF input is inflated (VCFX_GZIP=0: off)
    // BGZF members inflated on the device (the records stay there) in streaming mode; matrix mode
    // reads the records' text on the host
    in.bgzf_device = !o.matrix;
    if (!o.input.empty()) {
        if (!in.open_file(o.input.c_str()) || in.n == 0) {
            err.put("Error: cannot open file '" + o.input + "'\n");
            return 1;
        }
        if (!in.decompress(err.fd)) return 1;
        shard_records_begin(err);  // (a multi-GPU rank > 0 drops its stderr before this)
        if (o.matrix && o.shard_rank > 0) return 0;  // matrix mode is not sharded: rank 0 writes it
        bool ok = o.matrix ? run_ld_matrix(in, true, o.quiet, rchrom, has_region, rs, re, out_fd, err)
                           : run_stream(in, true, o, rchrom, has_region, rs, re, out_fd, err);
        return ok ? 0 : 1;
    }
    in.read_fd(in_fd);
    if (!in.decompress(err.fd)) return 1;
    if (o.matrix && o.shard_rank > 0) return 0;
    bool ok = o.matrix ? run_ld_matrix(in, false, o.quiet, rchrom, has_region, rs, re, out_fd, err)
                       : run_stream(in, false, o, rchrom, has_region, rs, re, out_fd, err);
    return ok ? 0 : 1;
}
