// VCFX_hwe_tester drop-in (a per-sample GT reducer on the record path):
// the reference CLI (VCFX_hwe_tester.cpp:414-449, 614-641, 688-694) on top of
// vcfxg_hwe_region.  The host skips the leading '#' lines (performHWE_Mmap :466-472); the
// device counts every record's genotype classes, applies the row rules and writes the rows.
// The host only rewrites the rows whose 6 p-value digits the device's exp() could not settle
// (vcfxg_hwe_rechecks; practically none), from the same counts with the host libm's exp.
#include <getopt.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

// displayHelp :394-412
const char *kHelp =
    "VCFX_hwe_tester: Perform Hardy-Weinberg Equilibrium (HWE) tests on a biallelic VCF.\n\n"
    "Usage:\n"
    "  VCFX_hwe_tester [options] [input.vcf]\n"
    "  VCFX_hwe_tester [options] < input.vcf\n\n"
    "Options:\n"
    "  -i, --input FILE   Input VCF file (uses memory-mapping for best performance)\n"
    "  -q, --quiet        Suppress informational messages\n"
    "  -h, --help         Show this help.\n\n"
    "Description:\n"
    "  Reads each variant line, ignoring multi-allelic calls. For biallelic lines,\n"
    "  collects genotypes as 0/0, 0/1, 1/1, then uses chi-square test with Yates'\n"
    "  continuity correction to produce a p-value for HWE.\n\n"
    "Performance:\n"
    "  Uses memory-mapped I/O and SIMD for ~20x speedup over stdin mode.\n\n"
    "Example:\n"
    "  VCFX_hwe_tester -i input.vcf > results.txt\n"
    "  VCFX_hwe_tester < input.vcf > results.txt\n";

// calculateHWE_chisq (:290-315) and chi2_pvalue_1df (:278-287) with the host libm, for the
// rows the device lists
double host_pvalue(int hom_ref, int het, int hom_alt) {
    const int n = hom_ref + het + hom_alt;
    if (n < 1) return 1.0;
    const double p = (2.0 * hom_ref + het) / (2.0 * n), q = 1.0 - p;
    if (p <= 0.0 || p >= 1.0) return 1.0;
    const double ex[3] = {n * p * p, n * 2.0 * p * q, n * q * q};
    const double ob[3] = {(double)hom_ref, (double)het, (double)hom_alt};
    double chi2 = 0.0;
    for (int k = 0; k < 3; k++) {
        double y = 0.0;
        if (ex[k] > 0.0) {
            double d = fabs(ob[k] - ex[k]) - 0.5;
            if (d < 0.0) d = 0.0;
            y = (d * d) / ex[k];
        }
        chi2 = k == 0 ? y : chi2 + y;
    }
    if (chi2 <= 0.0) return 1.0;
    if (chi2 > 700.0) return 0.0;
    const double x = sqrt(chi2 * 0.5);
    const double t = 1.0 / (1.0 + 0.3275911 * x);
    const double y = t * (0.254829592 + t * (-0.284496736 + t * (1.421413741 + t * (-1.453152027 + t * 1.061405429))));
    return y * exp(-x * x);
}

// the 8 bytes of a p-value (0 <= v < 10): appendDouble (:236-268) in file mode, setprecision(6)
// in stdin mode
void host_digits(double v, int mode, char *o) {
    char b[32];
    if (mode == VCFXG_MODE_FILE) {
        const long long ip = (long long)v;
        double fr = v - ip;
        b[0] = (char)('0' + ip);
        b[1] = '.';
        for (int k = 0; k < 6; k++) {
            fr *= 10.0;
            const int d = (int)fr;
            b[2 + k] = (char)('0' + d);
            fr -= d;
        }
    } else {
        snprintf(b, sizeof b, "%.6f", v);
    }
    memcpy(o, b, 8);
}

// performHWE_Mmap (:455-559) / performHWE_Stdin (:565-608); false on a device error
bool run_hwe(const Input &in, int mode, Out &out, Out &err) {
    if (mode == VCFXG_MODE_FILE && in.n == 0) return true;  // an empty file: no output at all
    if (!view_skip_header()) out.put("CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n");
    // the leading '#' lines (the device skips any later '#' line the same way)
    size_t ds = 0;
    while (ds < in.host_n && in.p[ds] == '#') {
        const char *nl = (const char *)memchr(in.p + ds, '\n', in.host_n - ds);
        if (!nl) {
            ds = in.host_n;
            break;
        }
        ds = (size_t)(nl - in.p) + 1;
    }
    phase("header skip");
    if (ds >= in.n) return true;
    vcfxg_ctx *g = gpu(err.fd);
    if (!g) return false;
    if (!load_input(g, in, err.fd)) return false;
    phase("input resident in HBM");
    vcfxg_summary s;
    if (!gpu_ok(g, vcfxg_hwe_region(g, ds, mode, &s), "hwe_region", err.fd)) return false;
    phase("hwe_region");
    std::string text(s.text_bytes, '\0');
    if (!gpu_ok(g, vcfxg_fetch_text(g, &text[0], text.size()), "fetch", err.fd)) return false;
    uint64_t nrc = 0;
    if (!gpu_ok(g, vcfxg_hwe_rechecks(g, nullptr, 0, &nrc), "hwe_rechecks", err.fd)) return false;
    if (nrc) {
        std::vector<vcfxg_hwe_recheck> rc(nrc);
        if (!gpu_ok(g, vcfxg_hwe_rechecks(g, rc.data(), nrc, &nrc), "hwe_rechecks", err.fd)) return false;
        for (const vcfxg_hwe_recheck &e : rc)
            host_digits(host_pvalue(e.hom_ref, e.het, e.hom_alt), mode, &text[e.text_offset]);
    }
    phase("rows fetched");
    out.put(text);
    return true;
}

}  // namespace

extern "C" int vcfx_tool_hwe_tester(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    Out out(out_fd), err(err_fd);
    // vcfx::handle_common_flags (vcfx_core.h:57-62)
    if (flag_present(argc, argv, "--help", "-h")) {
        out.put(kHelp);
        return 0;
    }
    if (flag_present(argc, argv, "--version", "-v")) {
        out.put("VCFX_hwe_tester version " VCFX_VERSION_STR "\n");
        return 0;
    }
    // parseArgs :414-449
    const char *input = nullptr;
    bool quiet = false, help = false;
    static struct option lo[] = {{"help", no_argument, nullptr, 'h'},
                                 {"input", required_argument, nullptr, 'i'},
                                 {"quiet", no_argument, nullptr, 'q'},
                                 {nullptr, 0, nullptr, 0}};
    GetoptStderr gs(err);
    optind = 0;
    int opt;
    while ((opt = getopt_long(argc, argv, "hi:q", lo, nullptr)) != -1) {
        if (opt == 'i') input = optarg;
        else if (opt == 'q') quiet = true;
        else help = true;
    }
    gs.done();
    if (!input && gs.next < argc) input = argv[gs.next];
    if (help) {
        out.put(kHelp);
        return 0;
    }
    Input in;
    in.gzip_ok = true;  // .vcf.gz / BGZF input is inflated (VCFX_GZIP=0: off)
    in.bgzf_device = true;  // BGZF members inflated on the device (the records stay there)
    if (input) {
        phase("start");
        if (!in.open_file(input)) {
            err.put(std::string("Error: Cannot open file: ") + input + "\n");
            return 1;
        }
        if (!quiet) err.put(std::string("Processing ") + input + " (" + std::to_string(reported_size(in)) + " bytes)...\n");
        err.flush();
        if (!in.decompress(err.fd)) return 1;
        shard_records_begin(err);
        return run_hwe(in, VCFXG_MODE_FILE, out, err) ? 0 : 1;
    }
    phase("start");
    in.read_fd(in_fd, /*host_copy=*/false);  // only the leading '#' lines are needed on the host
    if (!in.decompress(err.fd)) return 1;
    phase("stdin read");
    return run_hwe(in, VCFXG_MODE_STDIN, out, err) ? 0 : 1;
}
