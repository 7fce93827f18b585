// VCFX_allele_counter drop-in (a per-sample GT reducer with a row per
// (record, sample)): the reference CLI (VCFX_allele_counter.cpp:352-395 parseArguments, main
// :1473-1536) on top of vcfxg_allele_counter.  The host reads the header (sample names, the
// selection), the GPU counts and formats every row, and the host streams the text out
// (through zlib for -z, one deflate stream as the reference's GzipWriter writes).
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

// printHelp :400-426
const char *kHelp =
    "VCFX_allele_counter - Count reference and alternate alleles per sample\n\n"
    "Usage: VCFX_allele_counter [OPTIONS] [FILE]\n\n"
    "Options:\n"
    "  -i, --input FILE      Input VCF file (uses mmap for best performance)\n"
    "  -t, --threads N       Number of threads (default: auto-detect CPU cores)\n"
    "  -s, --samples STR     Space-separated list of sample names to include\n"
    "  -l, --limit-samples N Limit to first N samples (useful for large cohorts)\n"
    "  -a, --aggregate       Output per-variant aggregates instead of per-sample\n"
    "  -z, --gzip            Compress output with gzip (~10x smaller)\n"
    "  -b, --binary          Output binary format (compact, for machine consumption)\n"
    "  -q, --quiet           Suppress informational messages\n"
    "  -h, --help            Display this help message\n"
    "  -v, --version         Display version information\n\n"
    "Examples:\n"
    "  VCFX_allele_counter -i input.vcf > counts.tsv              # Default per-sample\n"
    "  VCFX_allele_counter -a -i input.vcf > aggregate.tsv        # Per-variant aggregates\n"
    "  VCFX_allele_counter -z -i input.vcf > counts.tsv.gz        # Gzip compressed\n"
    "  VCFX_allele_counter -l 100 -i input.vcf > counts.tsv       # First 100 samples\n"
    "  VCFX_allele_counter -b -i input.vcf > counts.bin           # Binary format\n"
    "  VCFX_allele_counter -t 8 -i input.vcf > counts.tsv         # 8 threads\n\n"
    "Output formats:\n"
    "  Default:    CHROM  POS  ID  REF  ALT  Sample  Ref_Count  Alt_Count\n"
    "  Aggregate:  CHROM  POS  ID  REF  ALT  Total_Ref  Total_Alt  Sample_Count\n"
    "  Binary:     Compact binary with header (use -b flag)\n";

const char kTextHdr[] = "CHROM\tPOS\tID\tREF\tALT\tSample\tRef_Count\tAlt_Count\n";
const char kAggHdr[] = "CHROM\tPOS\tID\tREF\tALT\tTotal_Ref\tTotal_Alt\tSample_Count\n";

enum { kText = 0, kAgg = 1, kBin = 2 };

struct Args {
    std::vector<std::string> samples;
    const char *input = nullptr;
    int threads = 0, limit = 0, kind = kText;
    bool gzip = false, quiet = false;
};

// where the output goes: the fd as it is, or one gzip stream (gzdopen(dup(fd), "wb6"))
struct Sink {
    int fd;
    bool gz;
    z_stream z{};
    std::vector<unsigned char> zb;
    Sink(int f, bool g) : fd(f), gz(g) {
        if (gz) {
            deflateInit2(&z, 6, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY);
            zb.resize(1 << 20);
        }
    }
    void put(const char *p, size_t n, bool last = false) {
        if (!gz) {
            write_all(fd, p, n);
            return;
        }
        do {  // (zpipe.c's loop: deflate consumes all input while it has output space)
            const size_t k = std::min<size_t>(n, 1u << 30);
            z.next_in = (Bytef *)p;
            z.avail_in = (uInt)k;
            p += k;
            n -= k;
            const int flush = last && n == 0 ? Z_FINISH : Z_NO_FLUSH;
            int r;
            do {
                z.next_out = zb.data();
                z.avail_out = (uInt)zb.size();
                r = deflate(&z, flush);
                write_all(fd, (const char *)zb.data(), zb.size() - z.avail_out);
            } while (z.avail_out == 0 || (flush == Z_FINISH && r != Z_STREAM_END));
        } while (n > 0);
    }
    void finish() {
        if (!gz) return;
        put("", 0, true);
        deflateEnd(&z);
        gz = false;
    }
};

// the device text [0, n) to the sink through a pinned window
bool emit_text(vcfxg_ctx *g, uint64_t n, Sink &sink, int err_fd) {
    if (!n) return true;
    const size_t win = (size_t)std::min<uint64_t>(n, 256ull << 20);
    char *h = nullptr;
    if (!gpu_ok(g, vcfxg_host_alloc(g, win, (void **)&h), "host_alloc", err_fd)) return false;
    bool ok = true;
    for (uint64_t o = 0; o < n && ok; o += win) {
        const size_t k = (size_t)std::min<uint64_t>(win, n - o);
        ok = gpu_ok(g, vcfxg_fetch_text_range(g, o, k, h), "fetch_text", err_fd);
        if (ok) sink.put(h, k);
    }
    vcfxg_host_free(g, h);
    return ok;
}

// the "#CHROM" line's sample names (fields after the 9th tab), appended
void chrom_names(const char *ls, const char *le, std::vector<std::string> &names) {
    const char *p = ls;
    for (int i = 0; i < 9 && p < le; i++) {
        const char *t = (const char *)memchr(p, '\t', (size_t)(le - p));
        p = t ? t + 1 : le;
    }
    while (p < le) {
        const char *t = (const char *)memchr(p, '\t', (size_t)(le - p));
        const char *e = t ? t : le;
        names.emplace_back(p, (size_t)(e - p));
        p = t ? t + 1 : le;
    }
}

// sampleMap lookups (:843-855): the last of duplicated names wins; false after the error line
bool select(const std::vector<std::string> &names, const Args &A, std::vector<uint32_t> &idx, Out &err) {
    idx.clear();
    if (A.samples.empty()) {
        for (size_t i = 0; i < names.size(); i++) idx.push_back((uint32_t)i);
        return true;
    }
    for (const auto &s : A.samples) {
        long hit = -1;
        for (size_t i = 0; i < names.size(); i++)
            if (names[i] == s) hit = (long)i;
        if (hit < 0) {
            err.put("Error: Sample '" + s + "' not found\n");
            return false;
        }
        idx.push_back((uint32_t)hit);
    }
    return true;
}

struct Slots {
    std::vector<uint32_t> idx;
    std::string names;
    std::vector<uint64_t> off{0};
    void add(const std::string &s) {
        names += s;
        off.push_back(names.size());
    }
};

// the rows of lines [l0, l1) of the indexed region to the sink
bool count_rows(vcfxg_ctx *g, uint64_t l0, uint64_t l1, const Slots &S, size_t m, int seq, int kind, Sink &sink,
                int err_fd, vcfxg_summary *sum = nullptr) {
    vcfxg_ac_params p{S.idx.data(), (uint64_t)m, S.names.data(), S.off.data(), seq, kind};
    vcfxg_summary s;
    if (!gpu_ok(g, vcfxg_allele_counter(g, l0, l1, &p, &s), "allele_counter", err_fd)) return false;
    phase("allele_counter");
    if (sum) *sum = s;
    if (!emit_text(g, s.text_bytes, sink, err_fd)) return false;
    phase("rows written");
    return true;
}

// the file paths' header scan (:802-839 / :1284-1307): '#' lines up to the first other line
// (an empty one included), names from every "#CHROM" line; returns the data start (n: none)
size_t file_header(const Input &in, std::vector<std::string> &names) {
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;
    while (p < end) {
        const char *q = p;
        next_line(q, end, ls, le);
        if (*ls != '#') return (size_t)(ls - in.p);
        if (is_chrom_line(ls, (size_t)(le - ls))) chrom_names(ls, le, names);
        p = q;
    }
    // a shard view (VCFX_INPUT_VIEW / a multi-GPU rank) or a device-only input (BGZF inflated on
    // the device): its records follow the header part
    return (in.tail || in.host_n < in.n) && p >= end ? in.host_n : in.n;
}

int hw_threads() {
    long k = sysconf(_SC_NPROCESSORS_ONLN);
    return k > 0 ? (int)k : 0;
}

// countAllelesMmapMT :786-950 (seq 0) / countAllelesUnified :1266-1468 (seq 1)
int run_file(const Args &A, int out_fd, Out &err) {
    Input in;
    in.gzip_ok = true;  // .vcf.gz / BGZF input is inflated (VCFX_GZIP=0: off)
    in.bgzf_device = true;  // BGZF members inflated on the device (the records stay there)
    phase("start");
    if (!in.open_file(A.input)) {
        err.put(std::string("Error: Cannot open file: ") + A.input + "\n");
        return 1;
    }
    if (!in.decompress(err.fd)) return 1;
    if (in.n == 0) {
        err.put("Error: Empty file\n");
        return 1;
    }
    const bool unified = A.kind != kText || A.gzip || A.limit > 0;
    std::vector<std::string> names;
    const size_t ds = file_header(in, names);
    if (names.empty()) {
        err.put("Error: No samples found in VCF\n");
        return 1;
    }
    if (!unified && ds >= in.n) {
        err.put("Error: No data lines found\n");
        return 1;
    }
    Slots S;
    if (!select(names, A, S.idx, err)) return 1;
    size_t m = S.idx.size();
    if (unified && A.limit > 0 && m > (size_t)A.limit) {
        m = (size_t)A.limit;
        if (!A.quiet) err.put("Info: Limiting to first " + std::to_string(A.limit) + " samples\n");
    }
    for (size_t i = 0; i < m; i++) S.add(names[S.idx[i]]);
    if (!unified && !A.quiet) {
        int nt = A.threads;
        if (nt <= 0) {
            nt = hw_threads();
            if (nt <= 0) nt = 4;
        }
        const size_t dsz = reported_size(in) - ds;  // (a multi-GPU rank: the whole file's data)
        if (dsz < 10u * 1024 * 1024) nt = 1;
        else if (dsz < 100u * 1024 * 1024 && nt > 4) nt = 4;
        err.put("Info: Using " + std::to_string(nt) + " threads\n");
    }
    err.flush();
    shard_records_begin(err);
    Sink sink(out_fd, A.gzip);
    if (view_skip_header()) {  // a multi-GPU rank > 0: rank 0 writes the header
    } else if (A.kind == kText) sink.put(kTextHdr, sizeof kTextHdr - 1);
    else if (A.kind == kAgg) sink.put(kAggHdr, sizeof kAggHdr - 1);
    else {  // BinaryHeader :327-332: "VCAC", version 1, sample count, 8 reserved bytes
        unsigned char h[20] = {'V', 'C', 'A', 'C', 1, 0, 0, 0};
        const uint32_t ns = (uint32_t)m;
        memcpy(h + 8, &ns, 4);
        sink.put((const char *)h, sizeof h);
    }
    bool ok = true;
    if (ds < in.n) {
        vcfxg_ctx *g = gpu(err.fd);
        uint64_t L = 0;
        ok = g && load_input(g, in, err.fd) && gpu_ok(g, vcfxg_index(g, ds, &L), "index", err.fd) &&
             count_rows(g, 0, L, S, m, unified ? 1 : 0, A.kind, sink, err.fd);
    }
    sink.finish();
    return ok ? 0 : 1;
}

// countAllelesStream :1122-1260: every "#CHROM" line appends its names and the selection made
// over all names so far; the slot names are the first m of a list that grows by the whole
// selection each time (kept as the reference builds it); text rows, seq semantics
int run_stream(const Args &A, int in_fd, int out_fd, Out &err) {
    Input in;
    in.gzip_ok = true;
    in.bgzf_device = true;
    phase("start");
    in.read_fd(in_fd, /*host_copy=*/false);  // the header on the host; records on the device
    if (!in.decompress(err.fd)) return 1;
    phase("stdin read");
    std::vector<std::string> names, suf;
    Slots S;
    bool found = false;
    size_t ds = in.n;
    auto rechrom = [&](const char *ls, const char *le) {
        chrom_names(ls, le, names);
        std::vector<uint32_t> add;
        if (!select(names, A, add, err)) return false;
        S.idx.insert(S.idx.end(), add.begin(), add.end());
        for (uint32_t i : S.idx) suf.push_back(names[i]);
        found = true;
        return true;
    };
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;
    while (p < end) {
        const char *q = p;
        next_line(q, end, ls, le);
        if (le == end && q == end && (size_t)(end - in.p) < in.n) break;  // a line cut by the host part
        if (le == ls) {
            p = q;
            continue;
        }
        if (*ls == '#') {
            if (is_chrom_line(ls, (size_t)(le - ls)) && !rechrom(ls, le)) return 1;
            p = q;
            continue;
        }
        if (!found) {
            err.put("Error: No #CHROM header found before data\n");
            return 1;
        }
        break;
    }
    ds = (size_t)(p - in.p);
    Sink sink(out_fd, false);
    if (ds >= in.n) {  // no data lines: the column header alone
        sink.put(kTextHdr, sizeof kTextHdr - 1);
        return found ? 0 : 1;
    }
    vcfxg_ctx *g = gpu(err.fd);
    uint64_t L = 0;
    if (!g || !load_input(g, in, err.fd) || !gpu_ok(g, vcfxg_index(g, ds, &L), "index", err.fd)) return 1;
    // the rows of [l0, l1) with the current selection (the device text of the last call)
    auto segment = [&](uint64_t l0, uint64_t l1, vcfxg_summary &s) {
        Slots cur;
        cur.idx = S.idx;
        for (size_t i = 0; i < S.idx.size(); i++) cur.add(suf[i]);
        vcfxg_ac_params prm{cur.idx.data(), (uint64_t)cur.idx.size(), cur.names.data(), cur.off.data(), 1, kText};
        return gpu_ok(g, vcfxg_allele_counter(g, l0, l1, &prm, &s), "allele_counter", err.fd);
    };
    vcfxg_summary s;
    if (!found) return 1;  // (a data line before '#CHROM' was reported above)
    if (!segment(0, L, s)) return 1;
    if (s.warn_lines == 0) {  // one selection for every record
        sink.put(kTextHdr, sizeof kTextHdr - 1);
        return emit_text(g, s.text_bytes, sink, err.fd) ? 0 : 1;
    }
    // '#CHROM' lines among the records: the rows between them with the selection at that point
    std::vector<uint8_t> st(L);
    std::vector<uint64_t> ends(L);
    if (!gpu_ok(g, vcfxg_fetch_lines(g, 0, L, nullptr, nullptr, st.data()), "fetch_lines", err.fd) ||
        !gpu_ok(g, vcfxg_line_ends(g, 0, L, ends.data()), "line_ends", err.fd))
        return 1;
    std::string pend(kTextHdr);  // (written at the end, as the reference's buffer)
    uint64_t l0 = 0;
    for (uint64_t k = 0; k <= L; k++) {
        if (k < L && st[k] != 4) continue;
        if (k > l0) {
            if (!segment(l0, k, s)) return 1;
            const size_t at = pend.size();
            pend.resize(at + s.text_bytes);
            if (s.text_bytes && !gpu_ok(g, vcfxg_fetch_text(g, &pend[at], s.text_bytes), "fetch", err.fd)) return 1;
        }
        if (k == L) break;
        const uint64_t a = k ? ends[k - 1] + 1 : ds, b = ends[k];
        std::string line(b - a, '\0');
        if (b > a && !gpu_ok(g, vcfxg_input_fetch(g, a, b - a, &line[0]), "input_fetch", err.fd)) return 1;
        if (!rechrom(line.data(), line.data() + line.size())) return 1;
        l0 = k + 1;
    }
    sink.put(pend.data(), pend.size());
    return 0;
}

}  // namespace

extern "C" int vcfx_tool_allele_counter(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    Out out(out_fd), err(err_fd);
    Args A;
    for (int i = 1; i < argc; i++) {  // parseArguments :352-395
        const std::string a = argv[i];
        if ((a == "--samples" || a == "-s") && i + 1 < argc) {
            const std::string s = argv[++i];
            size_t st = 0, e;
            while ((e = s.find(' ', st)) != std::string::npos) {
                if (e > st) A.samples.push_back(s.substr(st, e - st));
                st = e + 1;
            }
            if (st < s.size()) A.samples.push_back(s.substr(st));
            for (auto &x : A.samples) {  // (every sample so far, as the reference trims)
                const size_t f = x.find_first_not_of(" \t\n\r"), l = x.find_last_not_of(" \t\n\r");
                if (f != std::string::npos) x = x.substr(f, l - f + 1);
            }
        } else if (a == "--input" || a == "-i") {
            if (i + 1 < argc) A.input = argv[++i];
        } else if (a == "--threads" || a == "-t") {
            if (i + 1 < argc) A.threads = atoi(argv[++i]);
        } else if (a == "--limit-samples" || a == "-l") {
            if (i + 1 < argc) A.limit = atoi(argv[++i]);
        } else if (a == "--gzip" || a == "-z") A.gzip = true;
        else if (a == "--aggregate" || a == "-a") A.kind = kAgg;
        else if (a == "--binary" || a == "-b") A.kind = kBin;
        else if (a == "--quiet" || a == "-q") A.quiet = true;
        else if (a == "--help" || a == "-h") {
            out.put(kHelp);
            return 0;
        } else if (argv[i][0] != '-' && !A.input) A.input = argv[i];
    }
    for (int i = 1; i < argc; i++)
        if (!strcmp(argv[i], "--version") || !strcmp(argv[i], "-v")) {
            out.put("VCFX_allele_counter 2.0 (multi-threaded)\n");
            return 0;
        }
    if (!A.quiet) {
        if (!A.samples.empty()) {
            std::string s = "Info: Counting alleles for samples:";
            for (const auto &x : A.samples) s += " " + x;
            err.put(s + "\n");
        } else if (A.limit > 0) err.put("Info: Counting alleles for first " + std::to_string(A.limit) + " samples\n");
        else err.put("Info: Counting alleles for ALL samples\n");
        if (A.kind == kAgg) err.put("Info: Output mode: aggregate (per-variant summaries)\n");
        else if (A.kind == kBin) err.put("Info: Output mode: binary\n");
        if (A.gzip) err.put("Info: Output compression: gzip\n");
    }
    out.flush();
    if (A.input) {
        if (!A.quiet) err.put(std::string("Info: Using mmap mode for file: ") + A.input + "\n");
        return run_file(A, out_fd, err);
    }
    if (!A.quiet) err.put("Info: Using stdin streaming mode (single-threaded)\n");
    err.flush();
    return run_stream(A, in_fd, out_fd, err);
}
