// Fused `VCFX_record_filter ... | VCFX_genotype_query ...` (BASELINE config 3) in one
// process: the filter and the genotype query both run on the device over the same
// device-resident input (vcfxg_filter_query), and the host reproduces what the second
// process would print for the first one's output stream (genotypeQueryStream,
// VCFX_genotype_query.cpp:527-617, fed with processFileMmap / processStdin output,
// VCFX_record_filter.cpp:406-549).
#include <string.h>

#include <string>
#include <vector>

#include "emit.h"
#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

extern "C" int vcfx_pipeline_filter_query(const char *filter, const char *logic, const char *input, const char *query,
                                          int strict, int gq_quiet, int in_fd, int out_fd, int err_fd) {
    Out err(err_fd);
    std::vector<Criterion> cs;
    if (!compile_filter(filter, cs, err)) {
        err.put("Error: failed to parse criteria.\n");
        return 1;
    }
    const bool and_logic = strcmp(logic, "or") != 0;
    Input in;
    in.gzip_ok = true;  // .vcf.gz / BGZF input is inflated (VCFX_GZIP=0: off)
    in.bgzf_device = true;  // BGZF members inflated on the device (the records stay there)
    bool stdin_mode = !input;
    if (input) {
        if (!in.open_file(input)) {
            err.put(std::string("Error: cannot open file '") + input + "'\n");
            return 1;
        }
    } else in.read_fd(in_fd, /*host_copy=*/false);  // kept records are read back from the device
    if (!in.decompress(err.fd)) return 1;
    LineEmitter em(in.p, in.host_n, out_fd);
    std::vector<std::string> held;  // genotype_query's buffered header lines (copies)
    auto flush_held = [&]() {
        if (held.empty()) return;
        for (auto &h : held) {
            em.raw(h.data(), h.size());
            em.raw("\n", 1);
        }
        em.finish();
        held.clear();
    };
    bool found = false;
    auto strip = [](const char *a, const char *b) { return (b > a && b[-1] == '\r') ? b - 1 : b; };
    // the filter's header prefix as the query sees it
    const char *p = in.p, *end = in.p + in.host_n, *ls, *le;
    size_t data_start = in.n;
    while (next_line(p, end, ls, le)) {
        const char *ae = strip(ls, le);
        if (ae == ls) continue;  // filter prints "\n"; the query skips empty lines
        if (*ls == '#') {
            held.emplace_back(ls, (size_t)(ae - ls));
            if (is_chrom_line(ls, (size_t)(ae - ls))) {
                found = true;
                data_start = (size_t)(p - in.p);
                break;
            }
            continue;
        }
        if (stdin_mode) err.put("Warning: data line before #CHROM => skipping.\n");
    }
    if (found && data_start < in.n) {
        vcfxg_ctx *g = gpu(err.fd);
        if (!g) return 1;
        uint64_t nl = 0;
        vcfxg_summary s;
        std::vector<vcfxg_criterion> abi = to_abi(cs);
        if (!load_input(g, in, err.fd) ||
            !gpu_ok(g,
                    vcfxg_filter_query_region(g, data_start, abi.data(), (int)abi.size(), and_logic ? 1 : 0, query,
                                              strlen(query), strict, &s),
                    "filter_query", err.fd))
            return 1;
        nl = s.n_lines;
        std::vector<uint64_t> ends(nl);
        std::vector<uint8_t> st(nl);
        if (!gpu_ok(g, vcfxg_line_ends(g, 0, nl, ends.data()), "line_ends", err.fd) ||
            !gpu_ok(g, vcfxg_fetch_lines(g, 0, nl, nullptr, nullptr, st.data()), "fetch_lines", err.fd))
            return 1;
        LineSource src(in, g, em);
        uint64_t prev = data_start;
        for (uint64_t i = 0; i < nl; i++) {
            const uint8_t v = st[i];
            const char *a = nullptr, *b = nullptr;
            if (v == VCFXG_LINE_HEADER || v == VCFXG_LINE_ROW || v == 7) {
                a = src.at(prev, ends[i]);
                if (!a) break;
                b = a + (ends[i] - prev);
            }
            prev = ends[i] + 1;
            if (v == VCFXG_LINE_HEADER) held.emplace_back(a, (size_t)(strip(a, b) - a));
            else if (v == VCFXG_LINE_ROW || v == 6 || v == 7) {
                flush_held();
                if (v == VCFXG_LINE_ROW) em.line(a, strip(a, b));
                else if (v == 7 && !gq_quiet) {
                    err.put("Warning: skipping line with <9 fields: ");
                    err.put(a, (size_t)(strip(a, b) - a));
                    err.put("\n");
                }
            }
        }
        if (!src.ok) {
            em.finish();
            return gpu_ok(g, VCFXG_E_HIP, "input_fetch", err.fd) ? 0 : 1;
        }
    }
    em.finish();
    if (!found && !gq_quiet) err.put("Error: No #CHROM line found in VCF.\n");
    return 0;
}
