// VCFX_variant_counter drop-in: the reference CLI (VCFXVariantCounter::run,
// VCFX_variant_counter.cpp:116-180, main :399-405) on top of vcfxg_variant_count.
// gzip on stdin is inflated on the host with the reference's own chunk loop (first gzip
// member only, lines of a failed inflate call dropped: countVariantsGzip :223-290); the
// per-line column check runs on the GPU.
#include <getopt.h>
#include <string.h>
#include <zlib.h>

#include <string>
#include <vector>

#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

const char *kHelp =
    "VCFX_variant_counter: Counts the total number of valid variants in a VCF.\n\n"
    "Usage:\n"
    "  VCFX_variant_counter [options] [input.vcf]\n"
    "  VCFX_variant_counter [options] < input.vcf\n\n"
    "Options:\n"
    "  -h, --help        Show this help.\n"
    "  -s, --strict      Fail on any data line with <8 columns.\n\n"
    "Description:\n"
    "  Reads a VCF from file argument or stdin. For each data line,\n"
    "  we check if it has >=8 columns; if it does, we count it; if fewer columns:\n"
    "   * if --strict => we exit with error,\n"
    "   * otherwise => we skip with a warning.\n"
    "  When a file is provided directly, uses memory-mapped I/O for faster processing.\n"
    "  Finally, we print 'Total Variants: X'.\n\n"
    "Example:\n"
    "  VCFX_variant_counter input.vcf          # Fast memory-mapped mode\n"
    "  VCFX_variant_counter < input.vcf        # Stdin mode\n"
    "  VCFX_variant_counter --strict input.vcf\n";

// returns the count, or -1 (error already printed)
long count_lines(const char *p, size_t n, bool strip_cr, bool strict, Out &err) {
    if (n == 0) return 0;
    vcfxg_ctx *g = gpu(err.fd);
    if (!g) return -1;
    uint64_t nl = 0;
    vcfxg_summary s;
    if (!gpu_ok(g, vcfxg_load_host(g, p, n), "load", err.fd) || !gpu_ok(g, vcfxg_index(g, 0, &nl), "index", err.fd) ||
        !gpu_ok(g, vcfxg_variant_count(g, strip_cr ? 1 : 0, &s), "variant_count", err.fd))
        return -1;
    if (s.warn_lines) {
        std::vector<uint8_t> st(nl);
        if (!gpu_ok(g, vcfxg_fetch_lines(g, 0, nl, nullptr, nullptr, st.data()), "fetch_lines", err.fd)) return -1;
        for (uint64_t i = 0; i < nl; i++) {
            if (st[i] != VCFXG_LINE_WARN) continue;
            if (strict) {
                err.put("Error: line " + std::to_string(i + 1) + " has <8 columns.\n");
                return -1;
            }
            err.put("Warning: skipping line " + std::to_string(i + 1) + " with <8 columns.\n");
        }
    }
    return (long)s.rows;
}

// countVariantsGzip's decode: bytes whose lines the reference processes, and whether the
// stream failed (then only complete lines count and the error follows their warnings)
bool gunzip_like_reference(const char *in_p, size_t in_n, std::string &out, bool &failed) {
    const size_t CHUNK = 65536;
    z_stream st;
    memset(&st, 0, sizeof st);
    failed = false;
    if (inflateInit2(&st, 15 + 32) != Z_OK) return false;
    std::vector<char> ob(CHUNK);
    size_t ip = 0;
    int ret = Z_OK;
    do {
        size_t take = std::min(CHUNK, in_n - ip);
        st.avail_in = (uInt)take;
        st.next_in = (Bytef *)(in_p + ip);
        ip += take;
        if (take == 0) break;
        do {
            st.avail_out = (uInt)CHUNK;
            st.next_out = (Bytef *)ob.data();
            ret = inflate(&st, Z_NO_FLUSH);
            if (ret == Z_STREAM_ERROR || ret == Z_NEED_DICT || ret == Z_DATA_ERROR || ret == Z_MEM_ERROR) {
                failed = true;
                inflateEnd(&st);
                return true;
            }
            out.append(ob.data(), CHUNK - st.avail_out);
        } while (st.avail_out == 0);
    } while (ret != Z_STREAM_END);
    inflateEnd(&st);
    return true;
}

}  // namespace

extern "C" int vcfx_tool_variant_counter(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    Out out(out_fd), err(err_fd);
    if (flag_present(argc, argv, "--help", "-h")) {
        out.put(kHelp);
        return 0;
    }
    if (flag_present(argc, argv, "--version", "-v")) {
        out.put("VCFX_variant_counter version " VCFX_VERSION_STR "\n");
        return 0;
    }
    bool show = false, strict = false;
    static struct option lo[] = {{"help", no_argument, 0, 'h'}, {"strict", no_argument, 0, 's'}, {0, 0, 0, 0}};
    GetoptStderr gs(err);
    optind = 0;
    for (;;) {
        int c = getopt_long(argc, argv, "hs", lo, nullptr);
        if (c == -1) break;
        if (c == 'h') show = true;
        else if (c == 's') strict = true;
        else show = true;
    }
    gs.done();
    if (show) {
        out.put(kHelp);
        return 0;
    }
    long total;
    Input in;
    if (gs.next < argc) {
        if (!in.open_file(argv[gs.next])) {
            err.put(std::string("Error: cannot open file: ") + argv[gs.next] + "\n");
            return 1;
        }
        total = count_lines(in.p, in.n, true, strict, err);
    } else {
        in.read_fd(in_fd);
        if (in.n >= 2 && (unsigned char)in.p[0] == 0x1f && (unsigned char)in.p[1] == 0x8b) {
            std::string dec;
            bool failed = false;
            if (!gunzip_like_reference(in.p, in.n, dec, failed)) {
                err.put("Error: inflateInit2 failed.\n");
                return 1;
            }
            if (failed) {
                size_t keep = dec.rfind('\n');  // only complete lines were processed
                dec.resize(keep == std::string::npos ? 0 : keep + 1);
            }
            total = count_lines(dec.data(), dec.size(), false, strict, err);
            if (failed && total >= 0) {
                err.put("Error: decompression failed.\n");
                total = -1;
            }
        } else {
            total = count_lines(in.p, in.n, false, strict, err);
        }
    }
    if (total < 0) return 1;
    out.put("Total Variants: " + std::to_string(total) + "\n");
    return 0;
}
