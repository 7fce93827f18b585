// VCFX_haplotype_phaser drop-in (LD reuse in block phasing): the reference
// CLI (VCFX_haplotype_phaser.cpp:478-569 run, :1336-1342 main) on top of
// vcfxg_haplotype_phaser.  The GPU parses every record into genotype codes, computes r / r^2 of
// each variant with the one before it and takes the block rule's decision; the host runs the
// header gate, writes the '#' lines and warnings in line order and assembles the block lines
// (default mode: groupVariants :1275-1322; streaming: the window of CircularVariantBuffer
// :153-203, restated over variant numbers) from the decisions and the device-formatted entries.
#include <errno.h>
#include <getopt.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "emit.h"
#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

// displayHelp :571-601
const char *kHelp =
    "VCFX_haplotype_phaser: Group variants into blocks by naive LD threshold.\n\n"
    "Usage:\n"
    "  VCFX_haplotype_phaser [options] [input.vcf]\n"
    "  VCFX_haplotype_phaser [options] < input.vcf\n\n"
    "Options:\n"
    "  -h, --help               Show this help message\n"
    "  -l, --ld-threshold <val> r^2 threshold [0..1], default 0.8\n"
    "  -s, --streaming          Enable streaming mode with sliding window.\n"
    "                           Uses O(window * samples) memory instead of O(variants * samples).\n"
    "  -w, --window <N>         Window size for streaming mode (default: 1000)\n"
    "  -i, --input FILE         Input VCF file (uses fast memory-mapped I/O)\n"
    "  -q, --quiet              Suppress warning messages\n\n"
    "Performance:\n"
    "  File input (-i) uses memory-mapped I/O for 20-50x faster processing.\n"
    "  Features include:\n"
    "  - SIMD-optimized line scanning (AVX2/SSE2)\n"
    "  - Zero-copy string parsing with string_view\n"
    "  - 1MB output buffering\n"
    "  - Circular buffer for O(1) streaming operations\n"
    "  - FORMAT field caching\n"
    "  - SIMD-optimized LD calculation\n\n"
    "Modes:\n"
    "  Default mode:   Loads all variants into memory, outputs blocks at end.\n"
    "  Streaming mode: Uses sliding window, outputs blocks incrementally.\n"
    "                  Enables processing of arbitrarily large files.\n\n"
    "Examples:\n"
    "  VCFX_haplotype_phaser -i input.vcf              # Fast (mmap)\n"
    "  VCFX_haplotype_phaser input.vcf                 # Fast (mmap)\n"
    "  VCFX_haplotype_phaser < input.vcf               # Slower (stdin)\n"
    "  VCFX_haplotype_phaser --streaming -w 500 -i large.vcf\n";

enum : uint8_t { kVar = 1, kFew = 3, kHead = 4, kPos = 7, kNoGt = 8 };

struct Phaser {
    bool file, streaming, quiet;
    double thr;
    size_t win;
    Out &out, &err;
    // the variants' entries (device text) and per-variant flags
    std::string text;
    std::vector<uint64_t> off;
    std::vector<uint8_t> flags;
    int blockno = 0;
    bool marker = false;
    // streaming: CircularVariantBuffer over variant numbers
    std::vector<uint64_t> ring;
    size_t head = 0, cnt = 0;

    void entry(uint64_t v) { out.put(text.data() + off[v], (size_t)(off[v + 1] - off[v])); }
    void block(size_t k) {  // "Block N: " + the first k buffered variants
        out.put("Block " + std::to_string(++blockno) + ": ");
        for (size_t j = 0; j < k; j++) {
            entry(ring[(head + j) % ring.size()]);
            if (j + 1 < k) out.put(", ", 2);
        }
        out.putc('\n');
    }
    void push(uint64_t v) {
        ring[(head + cnt) % ring.size()] = v;
        if (cnt < ring.size()) cnt++;
        else head = (head + 1) % ring.size();
    }
    // streaming: variant v arrives (the previous one is the buffer's back whenever it is not empty)
    void stream_var(uint64_t v) {
        if (cnt == 0) {
            push(v);
            return;
        }
        if (!(flags[v] & 2)) {  // CHROM changed
            block(cnt);
            head = cnt = 0;
            push(v);
            return;
        }
        if (flags[v] & 1) {
            push(v);
            if (cnt > win) {
                const size_t ev = cnt - win;
                block(ev);
                for (size_t j = 0; j < ev && cnt; j++) {
                    head = (head + 1) % ring.size();
                    cnt--;
                }
            }
        } else {
            block(cnt);
            head = cnt = 0;
            push(v);
        }
    }
    void warn(uint8_t st) {
        if (quiet) return;
        if (st == kFew) err.put("Warning: skipping line with <10 fields\n");
        else if (st == kPos) err.put("Warning: invalid pos => skip\n");
        else if (st == kNoGt && !streaming) err.put(file ? "Warning: no GT field found\n" : "Warning: no GT field\n");
    }
    void header_line(const char *ls, const char *le) {
        out.put(ls, (size_t)(le - ls));
        out.putc('\n');
    }
};

// '\r' stripped; an empty line: true when the mode skips it
inline bool bare_line(bool file, const char *ls, const char *&le) {
    if (!file && le == ls) return true;  // getline: skipped before the strip
    if (le > ls && le[-1] == '\r') --le;
    return file && le == ls;
}

// sample count of the '#CHROM' line (fields after the 9th)
uint32_t chrom_samples(const char *ls, const char *le) {
    uint32_t tabs = 0;
    for (const char *p = ls; p < le; p++) tabs += *p == '\t';
    return tabs >= 9 ? tabs - 8 : 0;
}

bool run_ph(const Input &in, Phaser &P) {
    if (P.file && in.n == 0) return true;
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;
    size_t ds = in.n;
    uint32_t ns = 0;
    bool found = false;
    // the lines up to '#CHROM' (host bytes)
    while (next_line(p, end, ls, le)) {
        if (bare_line(P.file, ls, le)) continue;
        if (le > ls && *ls == '#') {
            P.header_line(ls, le);
            if (is_chrom_line(ls, (size_t)(le - ls))) {
                found = true;
                ns = chrom_samples(ls, le);
                ds = (size_t)(p - in.p);
                break;
            }
            continue;
        }
        if (P.file) {
            if (!P.quiet) P.err.put("Warning: VCF data line before #CHROM\n");
            continue;
        }
        if (!P.quiet) P.err.put("Error: no #CHROM line found.\n");
        return true;
    }
    uint64_t V = 0, nl = 0;
    std::vector<uint8_t> st;
    std::vector<uint64_t> ends;
    vcfxg_ctx *g = nullptr;
    if (found && ds < in.n) {
        g = gpu(P.err.fd);
        if (!g) return false;
        vcfxg_summary s;
        if (!load_input(g, in, P.err.fd) ||
            !gpu_ok(g, vcfxg_haplotype_phaser(g, ds, P.file ? VCFXG_MODE_FILE : VCFXG_MODE_STDIN, P.thr, ns, &s),
                    "haplotype_phaser", P.err.fd))
            return false;
        phase("haplotype_phaser");
        V = s.rows;
        nl = s.n_lines;
        st.resize(nl);
        ends.resize(nl);
        P.text.resize(s.text_bytes);
        P.off.resize(V + 1);
        P.flags.resize(V + 1);
        if (!gpu_ok(g, vcfxg_fetch_lines(g, 0, nl, nullptr, nullptr, st.data()), "fetch_lines", P.err.fd) ||
            !gpu_ok(g, vcfxg_line_ends(g, 0, nl, ends.data()), "line_ends", P.err.fd) ||
            !gpu_ok(g, vcfxg_phaser_variants(g, P.flags.data(), nullptr, P.off.data()), "phaser_variants", P.err.fd) ||
            (s.text_bytes && !gpu_ok(g, vcfxg_fetch_text(g, &P.text[0], s.text_bytes), "fetch_text", P.err.fd)))
            return false;
    }
    // the record lines in order: '#' lines written, warnings, (streaming) the blocks as they close
    if (P.streaming) P.ring.assign(P.win + 1 ? P.win + 1 : 1, 0);
    uint64_t v = 0;
    if (nl) {
        // pass-through lines are read from the input (a device-only stdin through a window)
        LineEmitter dummy(in.p, in.host_n, -1);
        LineSource src(in, g, dummy);
        uint64_t prev = ds;
        for (uint64_t i = 0; i < nl; i++) {
            const uint8_t s = st[i];
            if (s == kHead) {
                const char *a = src.at(prev, ends[i]);
                if (!a) break;
                const char *b = a + (ends[i] - prev);
                if (b > a && b[-1] == '\r') --b;
                P.header_line(a, b);
            } else if (s != 0) {
                if (P.streaming && !P.marker) {
                    P.out.put("#HAPLOTYPE_BLOCKS_START (streaming)\n");
                    P.marker = true;
                }
                if (s == kVar) {
                    if (P.streaming) P.stream_var(v);
                    v++;
                } else P.warn(s);
            }
            prev = ends[i] + 1;
        }
        if (!src.ok) return gpu_ok(g, VCFXG_E_HIP, "input_fetch", P.err.fd);
    }
    if (P.streaming) {
        if (P.cnt) P.block(P.cnt);
        if (P.marker) P.out.put("#HAPLOTYPE_BLOCKS_END\n");
        return true;
    }
    if (V == 0) {
        if (!P.quiet) P.err.put("Error: no variant data found.\n");
        return true;
    }
    P.out.put("#HAPLOTYPE_BLOCKS_START\n");
    for (uint64_t k = 0; k < V; k++) {
        if (k == 0 || (P.flags[k] & 3) != 3) {  // a new block: CHROM changed or the pair failed
            if (k) P.out.putc('\n');
            P.out.put("Block " + std::to_string(++P.blockno) + ": ");
        } else P.out.put(", ", 2);
        P.entry(k);
    }
    P.out.put("\n#HAPLOTYPE_BLOCKS_END\n");
    return true;
}

// std::stod / std::stoul: false when nothing converts or the value is out of range
bool stod_ok(const char *s, double &v) {
    char *e;
    errno = 0;
    v = strtod(s, &e);
    return e != s && errno != ERANGE;
}
bool stoul_ok(const char *s, unsigned long &v) {
    char *e;
    errno = 0;
    v = strtoul(s, &e, 10);
    return e != s && errno != ERANGE;
}

}  // namespace

extern "C" int vcfx_tool_haplotype_phaser(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    Out out(out_fd), err(err_fd);
    // vcfx::handle_common_flags (vcfx_core.h:57-62)
    if (flag_present(argc, argv, "--help", "-h")) {
        out.put(kHelp);
        return 0;
    }
    if (flag_present(argc, argv, "--version", "-v")) {
        out.put("VCFX_haplotype_phaser version " VCFX_VERSION_STR "\n");
        return 0;
    }
    double thr = 0.8;
    unsigned long win = 1000;
    bool streaming = false, quiet = false, help = false;
    std::string input;
    static struct option lo[] = {{"help", no_argument, nullptr, 'h'},      {"ld-threshold", required_argument, nullptr, 'l'},
                                 {"streaming", no_argument, nullptr, 's'}, {"window", required_argument, nullptr, 'w'},
                                 {"input", required_argument, nullptr, 'i'}, {"quiet", no_argument, nullptr, 'q'},
                                 {nullptr, 0, nullptr, 0}};
    GetoptStderr gs(err);
    optind = 0;
    int opt;
    while ((opt = getopt_long(argc, argv, "hl:sw:i:q", lo, nullptr)) != -1) {
        switch (opt) {
            case 'h': help = true; break;
            case 'l':
                if (!stod_ok(optarg, thr)) {
                    gs.done();
                    err.put("Error: invalid LD threshold.\n");
                    out.put(kHelp);
                    return 1;
                }
                break;
            case 's': streaming = true; break;
            case 'w':
                if (!stoul_ok(optarg, win)) {
                    gs.done();
                    err.put("Error: invalid window size.\n");
                    out.put(kHelp);
                    return 1;
                }
                break;
            case 'i': input = optarg; break;
            case 'q': quiet = true; break;
            default: help = true;
        }
    }
    gs.done();
    if (input.empty() && gs.next < argc) input = argv[gs.next];
    if (help) {
        out.put(kHelp);
        return 0;
    }
    if (thr < 0.0 || thr > 1.0) {
        err.put("Error: invalid LD threshold\n");
        out.put(kHelp);
        return 1;
    }
    if (streaming && win + 1 == 0) {  // the reference's window buffer of size 0 faults (SIGFPE)
        err.put("Error: invalid window size.\n");
        return 1;
    }
    Phaser P{false, streaming, quiet, thr, (size_t)win, out, err};
    Input in;
    in.gzip_ok = true;  // .vcf.gz / BGZF input is inflated (VCFX_GZIP=0: off)
    in.bgzf_device = true;  // BGZF members inflated on the device (the records stay there)
    phase("start");
    if (!input.empty() && input != "-") {
        if (!in.open_file(input.c_str())) {
            err.put("Error: Cannot open file: " + input + "\n");
            return 0;
        }
        if (!in.decompress(err.fd)) return 1;
        P.file = true;
    } else {
        in.read_fd(in_fd, /*host_copy=*/false);  // the header on the host; records on the device
        if (!in.decompress(err.fd)) return 1;
        phase("stdin read");
    }
    return run_ph(in, P) ? 0 : 1;
}
