// core_api_test.cpp -- exercises the vcfx core API (vcfx_core.h, vcfx_io.h) and prints every
// observable result.  Built twice by tests/test_core_api.py: against this project's
// libvcfx_core and against the reference's own src/vcfx_core.cpp (when /root/reference is
// present), and the two outputs must be identical; the output is also pinned by
// tests/golden/core_api_expected.txt.   usage: core_api_test DATA_DIR
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "vcfx_core.h"
#include "vcfx_io.h"

static std::ostringstream g_help;
static void help_cb() { g_help << "HELP"; }

static std::string show(const std::string &s) {
    std::string o = "<";
    for (char c : s) {
        if (c == '\n') o += "\\n";
        else if (c == '\r') o += "\\r";
        else if (c == '\t') o += "\\t";
        else o += c;
    }
    return o + ">";
}

template <class V>
static void print_fields(const char *what, const std::string &in, size_t n, const V &v) {
    std::cout << what << " " << show(in) << " n=" << n << " size=" << v.size() << ":";
    for (auto &f : v) std::cout << " " << show(std::string(f));
    std::cout << "\n";
}

int main(int argc, char **argv) {
    const std::string dir = argc > 1 ? argv[1] : ".";
    const char *inputs[] = {"", "a", "a,b", "a,", ",", ",,a", "a,,b,", ",,", "a\tb", "a\t", "\t", "\t\t",
                            "x;y;z", "k:v:", " a b ", "\t\na b\r\n", "AF=0.5;DP=3;DB"};
    for (const char *c : inputs) {
        const std::string s(c);
        auto sp = vcfx::split(s, ',');
        print_fields("split,", s, sp.size(), sp);
        auto st = vcfx::split(s, '\t');
        print_fields("split\\t", s, st.size(), st);
        std::cout << "trim " << show(s) << " -> " << show(vcfx::trim(s)) << "\n";
        std::vector<std::string> a{"stale"};
        size_t n = vcfx::split_tabs(s, a);
        print_fields("split_tabs", s, n, a);
        auto b = vcfx::split_tabs(s);
        print_fields("split_tabs1", s, b.size(), b);
        std::vector<std::string_view> c1;
        n = vcfx::split_tabs_view(s, c1);
        print_fields("split_tabs_view", s, n, c1);
        n = vcfx::split_char(s, ';', c1);
        print_fields("split_char;", s, n, c1);
        std::vector<std::string> d{"x", "y"};
        n = vcfx::split_string(s, ':', d);
        print_fields("split_string:", s, n, d);
        std::cout << "count_fields " << show(s) << " " << vcfx::count_fields(s) << "\n";
    }
    std::cout << "VCF " << vcfx::VCF::CHROM << vcfx::VCF::POS << vcfx::VCF::ID << vcfx::VCF::REF << vcfx::VCF::ALT
              << vcfx::VCF::QUAL << vcfx::VCF::FILTER << vcfx::VCF::INFO << vcfx::VCF::FORMAT
              << vcfx::VCF::FIRST_SAMPLE << vcfx::VCF::MIN_FIELDS << "\n";

    // flags
    std::vector<std::vector<std::string>> argvs = {
        {"tool"}, {"tool", "-h"}, {"tool", "--help"}, {"tool", "-v"}, {"tool", "x", "--version"},
        {"tool", "-h", "-v"}, {"tool", "--vers"}, {"tool", "-vh"}, {"-h"}};
    for (auto &av : argvs) {
        std::vector<char *> p;
        for (auto &x : av) p.push_back(const_cast<char *>(x.c_str()));
        p.push_back(nullptr);
        const int ac = (int)av.size();
        std::ostringstream os;
        g_help.str("");
        const bool fp = vcfx::flag_present(ac, p.data(), "--help", "-h");
        const bool fl = vcfx::flag_present(ac, p.data(), "--version");
        const bool hc = vcfx::handle_common_flags(ac, p.data(), "VCFX_t", help_cb, os);
        g_help << "|";
        const bool hh = vcfx::handle_help_flag(ac, p.data(), nullptr);
        const bool hv = vcfx::handle_version_flag(ac, p.data(), "VCFX_u", os);
        std::cout << "flags";
        for (auto &x : av) std::cout << " " << x;
        std::cout << " -> " << fp << fl << hc << hh << hv << " out=" << show(os.str()) << " help=" << show(g_help.str())
                  << "\n";
    }
    {
        std::ostringstream os;
        vcfx::print_error("bad thing", os);
        vcfx::print_version("VCFX_x", "9.9", os);
        std::cout << "print " << show(os.str()) << "\n";
    }

    // whole-stream readers
    const char *files[] = {"plain.vcf", "one.vcf.gz", "multi.vcf.bgz", "trunc.gz", "empty.vcf", "fake.gz",
                           "crlf.vcf",  "one_byte.txt", "magic_named.txt", "missing.vcf"};
    for (const char *f : files) {
        const std::string path = dir + "/" + f;
        std::string out = "seed";
        const bool ok = vcfx::read_file_maybe_compressed(path, out);
        std::cout << "read_file " << f << " ok=" << ok << " len=" << out.size() << " head=" << show(out.substr(0, 24))
                  << "\n";
        std::ifstream in(path, std::ios::binary);
        if (in.is_open()) {
            std::string o2 = "seed";
            const bool ok2 = vcfx::read_maybe_compressed(in, o2);
            std::cout << "read_stream " << f << " ok=" << ok2 << " len=" << o2.size() << " head=" << show(o2.substr(0, 24))
                      << "\n";
        }
    }

    // streaming reader (no truncated input: the reference spins on it)
    const char *sfiles[] = {"plain.vcf", "one.vcf.gz", "multi.vcf.bgz", "empty.vcf", "crlf.vcf", "one_byte.txt",
                            "noeol.vcf"};
    for (const char *f : sfiles) {
        std::ifstream fs;
        auto r = vcfx::make_streaming_reader(dir + "/" + f, fs);
        if (!r) {
            std::cout << "stream " << f << " null\n";
            continue;
        }
        std::cout << "stream " << f << " compressed=" << r->is_compressed() << " eof0=" << r->eof();
        std::string line;
        size_t n = 0, bytes = 0;
        std::string first, last;
        while (r->getline(line)) {
            if (!n) first = line;
            last = line;
            n++;
            bytes += line.size();
        }
        std::cout << " lines=" << n << " bytes=" << bytes << " first=" << show(first.substr(0, 20))
                  << " last=" << show(last.substr(0, 20)) << " eof=" << r->eof() << " err=" << r->error() << "\n";
    }
    {
        std::ifstream fs;
        auto r = vcfx::make_streaming_reader(dir + "/missing.vcf", fs);
        std::cout << "stream missing " << (r ? "reader" : "null") << "\n";
        std::istringstream ss("a\r\nb\n\nc\r");
        vcfx::StreamingGzipReader rd(ss);
        std::string l;
        std::cout << "stream sstream";
        while (rd.getline(l)) std::cout << " " << show(l);
        std::cout << " eof=" << rd.eof() << "\n";
        vcfx::StreamingGzipReader moved(std::move(rd));
        std::cout << "moved eof=" << moved.eof() << " getline=" << moved.getline(l) << "\n";
    }
    return 0;
}
