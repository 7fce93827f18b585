// tool_pipe.cpp -- `vcfx_pipe 'VCFX_record_filter ... | VCFX_genotype_query ... | VCFX_allele_freq_calc'`:
// the reference's documented use -- drop-ins chained stdin -> stdout (README.md:60-66; the
// `vcfx` wrapper only execvp's each tool, src/vcfx_wrapper/vcfx.cpp:177-187) -- in ONE process
// with ONE device context, output byte-identical to the shell pipeline.
//
// Two schedules:
//   fused   the input goes to HBM once; each filter stage (VCFX_record_filter, VCFX_genotype_query,
//           VCFX_nonref_filter) is one walk over the whole device input giving its per-record
//           keep decision (the stage's own rules, in its mode: the first stage's file / stdin
//           mode, stdin mode after it); the decisions are AND-ed, since a filter's output stream
//           is its input's header followed by the records it keeps, byte for byte.  The last
//           stage is VCFX_allele_freq_calc (stdin mode: one walk over every record, the rows of
//           the kept records gathered in order) or a filter (the header and the kept records,
//           read back from the device input).  The reference's per-stage work
//           (VCFX_record_filter.cpp:498-549, VCFX_genotype_query.cpp:527-617,
//           VCFX_nonref_filter.cpp:553-636, VCFX_allele_freq_calc.cpp:477-557) is the same
//           per-record function either way.
//   chain   every other chain, and any input the fused schedule does not cover: each stage runs
//           in-process (vcfx_tool_main on the shared context) with its stdin the previous
//           stage's stdout held in a memory file.
// The fused schedule is taken only where it provably equals the chain: the header lines up to
// '#CHROM' are non-empty '#' lines, the records hold no '\r', every record is one each filter
// keeps or drops (no warnings, no '#' or empty lines among them), at least one record survives
// (genotype_query holds the header until its first record), every survivor is an AF row, and
// the options are the plain ones (anything else -- abbreviated long options, unknown flags,
// gzip input -- takes the chain, whose tools parse it themselves).  stderr: the stages' in
// stage order; the exit code is the last stage's (the shell's default; VCFX_PIPEFAIL=1: the
// last non-zero).
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "emit.h"
#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

using Argv = std::vector<std::string>;

// shell words and '|' separators of a chain string (single / double quotes, backslash escapes)
bool split_chain(const std::string &s, std::vector<Argv> &stages, std::string &why) {
    stages.assign(1, Argv{});
    std::string w;
    bool inw = false;
    char q = 0;
    for (size_t i = 0; i < s.size(); i++) {
        const char c = s[i];
        if (q == '\'') {
            if (c == '\'') q = 0;
            else w += c;
            continue;
        }
        if (q == '"') {
            if (c == '"') q = 0;
            else if (c == '\\' && i + 1 < s.size() && strchr("\"\\$`", s[i + 1])) w += s[++i];
            else w += c;
            continue;
        }
        if (c == '\'' || c == '"') {
            q = c;
            inw = true;
        } else if (c == '\\' && i + 1 < s.size()) {
            w += s[++i];
            inw = true;
        } else if (c == ' ' || c == '\t' || c == '\n') {
            if (inw) stages.back().push_back(w);
            w.clear();
            inw = false;
        } else if (c == '|') {
            if (inw) stages.back().push_back(w);
            w.clear();
            inw = false;
            stages.push_back(Argv{});
        } else {
            w += c;
            inw = true;
        }
    }
    if (q) {
        why = "unterminated quote";
        return false;
    }
    if (inw) stages.back().push_back(w);
    for (auto &st : stages)
        if (st.empty()) {
            why = "empty stage";
            return false;
        }
    return true;
}

std::string base(const std::string &t) {
    const size_t k = t.rfind('/');
    return k == std::string::npos ? t : t.substr(k + 1);
}

// ---- the in-process chain -------------------------------------------------------------------
int run_stage(const Argv &a, int in_fd, int out_fd, int err_fd) {
    std::vector<std::string> own(a);
    std::vector<char *> av;
    for (auto &x : own) av.push_back(&x[0]);
    av.push_back(nullptr);
    return vcfx_tool_main(own[0].c_str(), (int)own.size(), av.data(), in_fd, out_fd, err_fd);
}

int mem_file() {
    int fd = memfd_create("vcfx_pipe_stage", MFD_CLOEXEC);
    if (fd < 0) {
        char t[] = "/tmp/vcfx_pipeXXXXXX";
        fd = mkstemp(t);
        if (fd >= 0) unlink(t);
    }
    return fd;
}

int run_chain(const std::vector<Argv> &stages, int in_fd, int out_fd, int err_fd) {
    const char *pf = getenv("VCFX_PIPEFAIL");
    const bool pipefail = pf && pf[0] == '1';
    int cur = in_fd, rc = 0, failed = 0;
    for (size_t k = 0; k < stages.size(); k++) {
        const bool last = k + 1 == stages.size();
        const int out = last ? out_fd : mem_file();
        if (out < 0) {
            write_str(err_fd, "Error: vcfx_pipe: no memory file for a stage's output\n");
            return 1;
        }
        rc = run_stage(stages[k], cur, out, err_fd);
        if (rc == -100) {
            write_str(err_fd, "Error: vcfx_pipe: unknown tool '" + stages[k][0] + "'\n");
            rc = 127;
        }
        if (rc) failed = rc;
        if (k > 0) ::close(cur);
        if (!last) {
            lseek(out, 0, SEEK_SET);
            cur = out;
        }
    }
    return pipefail && failed ? failed : rc;
}

// ---- the fused schedule ---------------------------------------------------------------------
enum Kind { kRF, kGQ, kNR, kAF };
struct Stage {
    Kind k;
    std::vector<Criterion> crit;
    bool and_logic = true;
    std::string query;
    bool strict = false;
};

// value of option `o` at argv[i]: "-x V", "-xV", "--long V", "--long=V"; advances i
bool opt_val(const Argv &a, size_t &i, const char *s, const char *l, std::string &v) {
    const std::string &x = a[i];
    const size_t ls = strlen(l);
    if (x == s || x == l) {
        if (i + 1 >= a.size()) return false;
        v = a[++i];
        return true;
    }
    if (x.size() > 2 && x.compare(0, 2, s) == 0 && x[1] != '-') {
        v = x.substr(2);
        return true;
    }
    if (x.size() > ls && x.compare(0, ls, l) == 0 && x[ls] == '=') {
        v = x.substr(ls + 1);
        return true;
    }
    return false;
}

// the plain option forms of the supported stages; false: the chain schedule parses it
bool plan_stage(const Argv &a, bool first, bool last, Stage &st, std::string &input) {
    const std::string t = base(a[0]);
    if (t == "VCFX_record_filter") st.k = kRF;
    else if (t == "VCFX_genotype_query") st.k = kGQ;
    else if (t == "VCFX_nonref_filter") st.k = kNR;
    else if (t == "VCFX_allele_freq_calc") st.k = kAF;
    else return false;
    if (st.k == kAF && (first || !last)) return false;
    std::string crit, logic = "and", in, v;
    bool have_in = false;
    for (size_t i = 1; i < a.size(); i++) {
        const std::string &x = a[i];
        if (first && st.k != kAF && opt_val(a, i, "-i", "--input", v)) {
            if (have_in) return false;
            in = v;
            have_in = true;
        } else if (st.k == kRF && opt_val(a, i, "-f", "--filter", v)) {
            crit = v;
        } else if (st.k == kRF && opt_val(a, i, "-l", "--logic", v)) {
            logic = v;
        } else if (st.k == kGQ && opt_val(a, i, "-g", "--genotype-query", v)) {
            st.query = v;
        } else if (st.k == kGQ && x == "--strict") {
            st.strict = true;
        } else if ((st.k == kRF || st.k == kGQ || st.k == kAF) && (x == "-q" || x == "--quiet")) {
        } else if (first && st.k != kAF && !x.empty() && x[0] != '-' && !have_in) {
            in = x;
            have_in = true;
        } else {
            return false;
        }
    }
    if (have_in && (in.empty() || in == "-")) return false;
    if (st.k == kRF) {
        if (crit.empty() || (logic != "and" && logic != "or")) return false;
        Out sink(-1);  // (a criteria error is the chain's to report)
        if (!compile_filter(crit, st.crit, sink)) return false;
        sink.buf.clear();
        st.and_logic = logic == "and";
    }
    if (st.k == kGQ && st.query.empty()) return false;
    if (first) input = in;
    return true;
}

enum { kFusedNo = -1, kFusedFallbackStdin = -2 };

// -1: not taken (nothing consumed); -2: not taken after stdin was consumed (*replay holds the
// input as a memory file); >= 0: the exit code
int run_fused(const std::vector<Stage> &P, const std::string &path, int in_fd, int out_fd, int err_fd, int *replay) {
    const bool file = !path.empty();
    const int n_filters = P.back().k == kAF ? (int)P.size() - 1 : (int)P.size();
    Input in;
    if (file) {
        struct stat st;
        if (stat(path.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) return kFusedNo;
        if (!in.open_file_device(path.c_str())) return kFusedNo;
    } else {
        in.read_fd(in_fd, /*host_copy=*/false);
    }
    phase("pipe: input");
    vcfxg_ctx *g = nullptr;
    auto give_up = [&]() -> int {
        if (file) return kFusedNo;  // the chain re-reads the file
        // stdin was consumed: its bytes (host part, then the device part) become the chain's stdin
        const int fd = mem_file();
        if (fd < 0) return 1;
        write_all(fd, in.p, in.host_n);
        if (in.host_n < in.n) {
            vcfxg_ctx *c = g ? g : gpu(err_fd);
            if (!c || (!g && !load_input(c, in, err_fd))) return 1;
            std::vector<char> w((size_t)64 << 20);
            for (uint64_t o = in.host_n; o < in.n; o += w.size()) {
                const size_t k = (size_t)std::min<uint64_t>(w.size(), in.n - o);
                if (!gpu_ok(c, vcfxg_input_fetch(c, o, k, w.data()), "input_fetch", err_fd)) return 1;
                write_all(fd, w.data(), k);
            }
        }
        lseek(fd, 0, SEEK_SET);
        *replay = fd;
        return kFusedFallbackStdin;
    };
    if (in.read_errno || (in.n >= 2 && (unsigned char)in.p[0] == 0x1f && (unsigned char)in.p[1] == 0x8b))
        return give_up();  // read errors and gzip input: the tools' own handling
    // the header: non-empty '#' lines without '\r' through '#CHROM'
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;
    size_t ds = in.n;
    while (next_line(p, end, ls, le)) {
        if (le == ls || *ls != '#' || le[-1] == '\r') return give_up();
        if (is_chrom_line(ls, (size_t)(le - ls))) {
            ds = (size_t)(p - in.p);
            break;
        }
    }
    if (ds >= in.n) return give_up();
    g = gpu_quiet();
    if (!g) return give_up();
    if (!load_input(g, in, err_fd)) return 1;
    uint64_t cr = 0;
    if (!gpu_ok(g, vcfxg_count_byte(g, ds, '\r', &cr), "count_byte", err_fd)) return 1;
    if (cr) return give_up();
    phase("pipe: input resident, checked");
    uint64_t nl = 0;
    std::vector<uint8_t> keep, st;
    std::vector<uint64_t> ends;
    for (int k = 0; k < n_filters; k++) {
        const Stage &S = P[(size_t)k];
        const int mode = (k == 0 && file) ? VCFXG_MODE_FILE : VCFXG_MODE_STDIN;
        vcfxg_summary s;
        int rc;
        if (S.k == kRF) {
            std::vector<vcfxg_criterion> abi = to_abi(S.crit);
            rc = vcfxg_record_filter_region(g, ds, abi.data(), (int)abi.size(), S.and_logic ? 1 : 0, &s);
        } else if (S.k == kGQ) {
            rc = vcfxg_genotype_query_region(g, ds, S.query.data(), S.query.size(), S.strict ? 1 : 0, 0, &s);
        } else {
            rc = vcfxg_nonref_filter_region(g, ds, mode, &s);
        }
        if (!gpu_ok(g, rc, "pipe stage", err_fd)) return 1;
        if (k == 0) {
            nl = s.n_lines;
            keep.assign(nl, 1);
            st.resize(nl);
            ends.resize(nl);
            if (!gpu_ok(g, vcfxg_line_ends(g, 0, nl, ends.data()), "line_ends", err_fd)) return 1;
        } else if (s.n_lines != nl) {
            return give_up();
        }
        if (!gpu_ok(g, vcfxg_fetch_lines(g, 0, nl, nullptr, nullptr, st.data()), "fetch_lines", err_fd)) return 1;
        for (uint64_t i = 0; i < nl; i++) {
            if (!keep[i]) continue;  // what a stage does with a record it never sees does not matter
            if (st[i] == VCFXG_LINE_ROW) continue;
            if (st[i] != VCFXG_LINE_DROP) return give_up();
            keep[i] = 0;
        }
        phase("pipe: filter stage");
    }
    uint64_t kept = 0;
    for (uint64_t i = 0; i < nl; i++) kept += keep[i];
    if (!kept) return give_up();
    if (P.back().k == kAF) {
        vcfxg_summary s;
        if (!gpu_ok(g, vcfxg_allele_freq_region(g, ds, VCFXG_MODE_STDIN, &s), "allele_freq", err_fd)) return 1;
        if (s.n_lines != nl) return give_up();
        if (!gpu_ok(g, vcfxg_fetch_lines(g, 0, nl, nullptr, nullptr, st.data()), "fetch_lines", err_fd)) return 1;
        for (uint64_t i = 0; i < nl; i++)
            if (keep[i] && st[i] != VCFXG_LINE_ROW) return give_up();
        std::string text(s.text_bytes, '\0');
        if (!gpu_ok(g, vcfxg_fetch_text(g, &text[0], text.size()), "fetch", err_fd)) return 1;
        phase("pipe: allele_freq rows");
        // the rows of the kept records: the AF rows follow the ROW lines in order
        LineEmitter em(text.data(), text.size(), out_fd);
        static const char kHead[] = "CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n";
        em.raw(kHead, sizeof kHead - 1);
        const char *r = text.data(), *te = text.data() + text.size();
        for (uint64_t i = 0; i < nl && r < te; i++) {
            if (st[i] != VCFXG_LINE_ROW) continue;
            const char *nl_ = (const char *)memchr(r, '\n', (size_t)(te - r));
            const char *re = nl_ ? nl_ + 1 : te;
            if (keep[i]) em.bytes(r, re);
            r = re;
        }
        em.finish();
        phase("pipe: rows written");
        return 0;
    }
    // a filter last: the header, then the kept records from the device input
    LineEmitter em(in.p, in.host_n, out_fd);
    em.bytes(in.p, in.p + ds);
    LineSource src(in, g, em);
    uint64_t prev = ds;
    for (uint64_t i = 0; i < nl; i++) {
        if (keep[i]) {
            const char *a = src.at(prev, ends[i]);
            if (!a) break;
            em.line(a, a + (ends[i] - prev));
        }
        prev = ends[i] + 1;
    }
    em.finish();
    if (!src.ok) return gpu_ok(g, VCFXG_E_HIP, "input_fetch", err_fd) ? 0 : 1;
    phase("pipe: records written");
    return 0;
}

}  // namespace

extern "C" int vcfx_pipe_main(int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    std::vector<Argv> stages;
    std::string why;
    if (argc == 2) {
        if (!split_chain(argv[1], stages, why)) {
            write_str(err_fd, "Error: vcfx_pipe: " + why + "\n");
            return 2;
        }
    } else if (argc > 2) {  // the words already split: "|" arguments separate the stages
        stages.assign(1, Argv{});
        for (int i = 1; i < argc; i++) {
            if (!strcmp(argv[i], "|")) stages.push_back(Argv{});
            else stages.back().push_back(argv[i]);
        }
        for (auto &st : stages)
            if (st.empty()) {
                write_str(err_fd, "Error: vcfx_pipe: empty stage\n");
                return 2;
            }
    } else {
        write_str(err_fd,
                  "Usage: vcfx_pipe 'VCFX_<tool> [args] | VCFX_<tool> [args] | ...'\n"
                  "       vcfx_pipe VCFX_<tool> [args] '|' VCFX_<tool> [args] ...\n"
                  "Runs the chain in one process on one device context; output identical to the shell pipeline.\n");
        return 2;
    }
    const char *f = getenv("VCFX_PIPE_FUSED");
    if (stages.size() >= 2 && !(f && f[0] == '0')) {
        std::vector<Stage> P(stages.size());
        std::string input;
        bool ok = true;
        for (size_t k = 0; k < stages.size() && ok; k++)
            ok = plan_stage(stages[k], k == 0, k + 1 == stages.size(), P[k], input);
        if (ok) {
            int replay = -1;
            const int rc = run_fused(P, input, in_fd, out_fd, err_fd, &replay);
            if (rc >= 0) return rc;
            if (rc == kFusedFallbackStdin) {
                const int r = run_chain(stages, replay, out_fd, err_fd);
                ::close(replay);
                return r;
            }
        }
    }
    return run_chain(stages, in_fd, out_fd, err_fd);
}
