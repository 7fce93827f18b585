// VCFX_dosage_calculator drop-in (a per-sample GT map on the record path):
// the reference CLI (VCFX_dosage_calculator.cpp:52-102, 614-620) on top of
// vcfxg_dosage_region.  The host runs the '#CHROM' gate over the header prefix (a data line
// before it is the reference's error); every record after it is parsed and formatted on the
// GPU, one dosage per sample.
#include <getopt.h>
#include <string.h>

#include <string>

#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

// displayHelp :24-47
const char *kHelp =
    "VCFX_dosage_calculator: Calculate genotype dosage for each variant in a VCF file.\n\n"
    "Usage:\n"
    "  VCFX_dosage_calculator [options] [input.vcf]\n"
    "  VCFX_dosage_calculator [options] < input.vcf > dosage_output.txt\n\n"
    "Options:\n"
    "  -i, --input FILE  Input VCF file (uses mmap for best performance)\n"
    "  -q, --quiet       Suppress warning messages\n"
    "  -h, --help        Display this help message and exit\n\n"
    "Description:\n"
    "  For each variant in the input VCF, the tool computes the dosage for each sample\n"
    "  based on the genotype (GT) field. Dosage is defined as the number of alternate\n"
    "  alleles (i.e. each allele > 0 counts as 1). Thus:\n"
    "    0/0  => dosage 0\n"
    "    0/1  => dosage 1\n"
    "    1/1  => dosage 2\n"
    "    1/2  => dosage 2  (each alternate, regardless of numeric value, counts as 1)\n\n"
    "Performance:\n"
    "  When using -i/--input, the tool uses memory-mapped I/O for\n"
    "  ~10-15x faster processing of large files.\n\n"
    "Example:\n"
    "  VCFX_dosage_calculator -i input.vcf > dosage_output.txt\n"
    "  VCFX_dosage_calculator < input.vcf > dosage_output.txt\n";

const char *kHeader = "CHROM\tPOS\tID\tREF\tALT\tDosages\n";
const char *kNoHeader = "Error: VCF header (#CHROM) not found before variant records.\n";
const char *kWarn = "Warning: Skipping VCF line with fewer than 10 fields.\n";

// processFileMmap :375-588 (mode file: '\r' stripped, the warning obeys -q, the header error
// exits 1) / calculateDosage :209-360 (stdin: lines as getline gives them, the warning always,
// the header error exits 0).  Either error path writes nothing on stdout.  Returns the exit
// code, or -1 on a device error (already reported).
int run_dose(const Input &in, int mode, bool quiet, Out &out, Out &err) {
    if (mode == VCFXG_MODE_FILE && in.n == 0) return 0;  // an empty file: no output at all
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;
    size_t data_start = in.n;
    bool found = false;
    while (next_line(p, end, ls, le)) {
        const char *ae = le;
        if (mode == VCFXG_MODE_FILE && ae > ls && ae[-1] == '\r') --ae;
        if (ae == ls) continue;
        if (*ls == '#') {
            if (is_chrom_line(ls, (size_t)(ae - ls))) {
                data_start = (size_t)(p - in.p);
                found = true;
                break;
            }
            continue;
        }
        err.put(kNoHeader);  // a data line before '#CHROM'
        return mode == VCFXG_MODE_FILE ? 1 : 0;
    }
    if (!view_skip_header()) out.put(kHeader);
    if (!found || data_start >= in.n) return 0;
    vcfxg_ctx *g = gpu(err.fd);
    if (!g) return -1;
    if (!load_input(g, in, err.fd)) return -1;
    phase("input resident in HBM");
    vcfxg_summary s;
    if (!gpu_ok(g, vcfxg_dosage_region(g, data_start, mode, &s), "dosage_region", err.fd)) return -1;
    phase("dosage_region");
    std::string text(s.text_bytes, '\0');
    if (!gpu_ok(g, vcfxg_fetch_text(g, &text[0], text.size()), "fetch", err.fd)) return -1;
    phase("rows fetched");
    out.put(text);
    if (mode == VCFXG_MODE_STDIN || !quiet)
        for (uint64_t k = 0; k < s.warn_lines; k++) err.put(kWarn);
    return 0;
}

}  // namespace

extern "C" int vcfx_tool_dosage_calculator(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    Out out(out_fd), err(err_fd);
    // vcfx::handle_common_flags (vcfx_core.h:57-62)
    if (flag_present(argc, argv, "--help", "-h")) {
        out.put(kHelp);
        return 0;
    }
    if (flag_present(argc, argv, "--version", "-v")) {
        out.put("VCFX_dosage_calculator version " VCFX_VERSION_STR "\n");
        return 0;
    }
    // run :52-102
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
    int rc;
    if (input) {
        phase("start");
        if (!in.open_file(input)) {
            err.put(std::string("Error: cannot open file '") + input + "'\n");
            return 1;
        }
        if (!in.decompress(err.fd)) return 1;
        shard_records_begin(err);  // (a multi-GPU rank > 0 drops its stderr before this)
        rc = run_dose(in, VCFXG_MODE_FILE, quiet, out, err);
    } else {
        phase("start");
        in.read_fd(in_fd, /*host_copy=*/false);  // only the header is needed on the host
        if (!in.decompress(err.fd)) return 1;
        phase("stdin read");
        rc = run_dose(in, VCFXG_MODE_STDIN, quiet, out, err);
    }
    return rc < 0 ? 1 : rc;
}
