// record_filter_api.cpp -- the reference's VCFX_record_filter library interface
// (include/vcfx_record_filter.h) over the MI355X engine.
//
//   parseCriteria  VCFX_record_filter.cpp:176-202 / :89-171 (the drop-in's compile_filter)
//   recordPasses   :668-765, one record on the host (the scalar predicate)
//   processVCF     :767-805, every record on the GPU (vcfxg_record_filter_ex, legacy flags)
//   printHelp      :807-810
#include <stdlib.h>
#include <string.h>

#include <iterator>
#include <string>
#include <string_view>
#include <vector>

#include "hostio.h"
#include "tools.h"
#include "vcfx_record_filter.h"

using namespace vcfxh;

namespace {

// extractField (:207-229): the index-th tab field, empty when the line has fewer
std::string_view field(std::string_view line, int index) {
    size_t p = 0;
    for (int k = 0; k < index; k++) {
        const size_t t = line.find('\t', p);
        if (t == std::string_view::npos) return {};
        p = t + 1;
    }
    const size_t e = line.find('\t', p);
    return line.substr(p, e == std::string_view::npos ? std::string_view::npos : e - p);
}

// extractInfoValue (:234-267): "k=v" -> v; a flag token -> the flag itself
bool info_value(std::string_view info, std::string_view key, std::string_view &out) {
    if (info.empty() || info == ".") return false;
    size_t p = 0;
    while (p < info.size()) {
        size_t e = info.find(';', p);
        if (e == std::string_view::npos) e = info.size();
        const std::string_view tok = info.substr(p, e - p);
        const size_t eq = tok.find('=');
        if (eq != std::string_view::npos) {
            if (tok.substr(0, eq) == key) {
                out = tok.substr(eq + 1);
                return true;
            }
        } else if (tok == key) {
            out = tok;
            return true;
        }
        p = e + 1;
    }
    return false;
}

// parseDouble (:273-299): strtod on a NUL-terminated copy; `out` receives strtod's value even
// when it did not consume the whole view (the OR-mode QUAL of recordPasses compares it)
bool parse_double(std::string_view sv, double &out) {
    if (sv.empty()) return false;
    std::string tmp(sv);
    char *end = nullptr;
    out = strtod(tmp.c_str(), &end);
    return end == tmp.c_str() + tmp.size();
}

bool cmp_double(double a, FilterOp op, double b) {  // compareDouble (:310-320)
    switch (op) {
    case FilterOp::GT: return a > b;
    case FilterOp::GE: return a >= b;
    case FilterOp::LT: return a < b;
    case FilterOp::LE: return a <= b;
    case FilterOp::EQ: return a == b;
    case FilterOp::NE: return a != b;
    }
    return false;
}

bool cmp_string(std::string_view a, FilterOp op, const std::string &b) {  // compareString (:322-328)
    if (op == FilterOp::EQ) return a == b;
    if (op == FilterOp::NE) return a != b;
    return false;
}

// one criterion as recordPasses evaluates it; `strict` = AND mode (a failed parse fails it)
bool legacy_criterion(std::string_view line, const FilterCriterion &c, bool strict) {
    switch (c.target) {
    case TargetField::POS: {
        const std::string_view f = field(line, 1);
        double pos;
        if (f.empty() || !parse_double(f, pos)) return false;
        return cmp_double(pos, c.op, c.numericValue);
    }
    case TargetField::QUAL: {
        const std::string_view f = field(line, 5);
        double qual = 0.0;
        if (!f.empty() && f != ".") {
            if (!parse_double(f, qual) && strict) return false;
        }
        return cmp_double(qual, c.op, c.numericValue);
    }
    case TargetField::FILTER: return cmp_string(field(line, 6), c.op, c.stringValue);
    case TargetField::INFO_KEY: {
        std::string_view v;
        if (!info_value(field(line, 7), c.fieldName, v)) return false;
        if (c.fieldType == FieldType::NUMERIC) {
            double num;
            if (!parse_double(v, num)) return false;
            return cmp_double(num, c.op, c.numericValue);
        }
        return cmp_string(v, c.op, c.stringValue);
    }
    }
    return false;
}

// the criteria as the device evaluates the legacy semantics (vcfxg_record_filter_ex)
std::vector<vcfxg_criterion> legacy_abi(const std::vector<FilterCriterion> &cs, bool and_logic) {
    std::vector<vcfxg_criterion> out;
    out.reserve(cs.size());
    for (const auto &c : cs) {
        vcfxg_criterion a;
        memset(&a, 0, sizeof a);
        a.target = (int)c.target;
        a.op = (int)c.op;
        a.numeric = c.fieldType == FieldType::NUMERIC ? 1 : 0;
        a.value = c.numericValue;
        a.key = c.fieldName.data();
        a.key_len = c.fieldName.size();
        a.str = c.stringValue.data();
        a.str_len = c.stringValue.size();
        if (c.target == TargetField::FILTER) a.numeric = 0;  // always a string compare (:700-702)
        if (c.target == TargetField::QUAL && !and_logic) a.target = 4;  // OR mode: lenient QUAL (:736-739)
        out.push_back(a);
    }
    return out;
}

}  // namespace

bool parseCriteria(const std::string &criteriaStr, std::vector<FilterCriterion> &criteria) {
    criteria.clear();
    Out err(2);
    std::vector<Criterion> cs;
    if (!compile_filter(criteriaStr, cs, err)) return false;
    for (const auto &c : cs) {
        FilterCriterion f;
        f.fieldName = c.name;
        f.op = (FilterOp)c.op;
        f.target = (TargetField)c.target;
        f.fieldType = c.numeric ? FieldType::NUMERIC : FieldType::STRING;
        f.numericValue = c.numeric ? c.value : 0.0;
        f.stringValue = c.numeric ? std::string() : c.str;
        criteria.push_back(std::move(f));
    }
    return true;
}

bool recordPasses(const std::string &record, const std::vector<FilterCriterion> &criteria, bool useAndLogic) {
    const std::string_view line(record);
    for (const auto &c : criteria) {
        const bool pass = legacy_criterion(line, c, useAndLogic);
        if (useAndLogic && !pass) return false;
        if (!useAndLogic && pass) return true;
    }
    return useAndLogic;
}

void processVCF(std::istream &in, std::ostream &out, const std::vector<FilterCriterion> &criteria, bool useAndLogic) {
    const std::string buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    std::string ob;
    ob.reserve(1 << 20);
    auto flush = [&](bool force) {
        if (force || ob.size() > 512 * 1024) {
            out.write(ob.data(), (std::streamsize)ob.size());
            ob.clear();
        }
    };
    // getline lines before '#CHROM' (:775-790): empty -> "\n", '#' -> echoed, data -> warning
    size_t p = 0, data_start = buf.size();
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == std::string::npos) e = buf.size();
        const std::string_view line(buf.data() + p, e - p);
        const size_t next = e < buf.size() ? e + 1 : e;
        if (line.empty()) ob.push_back('\n');
        else if (line[0] == '#') {
            ob.append(line.data(), line.size());
            ob.push_back('\n');
            if (line.rfind("#CHROM", 0) == 0) {
                data_start = next;
                break;
            }
        } else {
            std::cerr << "Warning: data line before #CHROM => skipping.\n";
        }
        p = next;
    }
    if (data_start < buf.size()) {
        vcfxg_ctx *g = gpu(2);
        if (!g) {  // no device: the diagnostic is out; the header part is what can be written
            flush(true);
            return;
        }
        const std::vector<vcfxg_criterion> abi = legacy_abi(criteria, useAndLogic);
        uint64_t nl = 0;
        vcfxg_summary s;
        if (!gpu_ok(g, vcfxg_load_host(g, buf.data(), buf.size()), "load", 2) ||
            !gpu_ok(g, vcfxg_index(g, data_start, &nl), "index", 2) ||
            !gpu_ok(g, vcfxg_record_filter_ex(g, abi.data(), (int)abi.size(), useAndLogic ? 1 : 0, VCFXG_RF_KEEP_CR,
                                              &s),
                    "record_filter", 2)) {
            flush(true);
            return;
        }
        std::vector<uint64_t> ends(nl);
        std::vector<uint8_t> st(nl);
        if (!gpu_ok(g, vcfxg_line_ends(g, 0, nl, ends.data()), "line_ends", 2) ||
            !gpu_ok(g, vcfxg_fetch_lines(g, 0, nl, nullptr, nullptr, st.data()), "fetch_lines", 2)) {
            flush(true);
            return;
        }
        uint64_t prev = data_start;
        for (uint64_t i = 0; i < nl; i++) {
            const char *a = buf.data() + prev;
            const size_t len = (size_t)(ends[i] - prev);
            prev = ends[i] + 1;
            bool keep = st[i] == VCFXG_LINE_ROW || st[i] == VCFXG_LINE_HEADER;
            if (st[i] == VCFXG_LINE_RECHECK) keep = recordPasses(std::string(a, len), criteria, useAndLogic);
            if (st[i] == VCFXG_LINE_SKIP) ob.push_back('\n');
            else if (keep) {
                ob.append(a, len);
                ob.push_back('\n');
            }
            flush(false);
        }
    }
    flush(true);
}

void printHelp() { std::cout << rf_help_text(); }
