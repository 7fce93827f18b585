// VCFX_ld_calculator --matrix: computeLDMatrixMmap (VCFX_ld_calculator.cpp:653-859, file
// path) and computeLD (:992-1079, stdin).  Input lines are passed through from the host
// copy; the M x M r^2 cells are computed and formatted on the GPU (vcfxg_ld_matrix).
#include <string.h>

#include <string>
#include <vector>

#include "emit.h"
#include "hostio.h"
#include "tools.h"

namespace vcfxh {

int ld_samples(const char *ls, const char *le);

bool run_ld_matrix(const Input &in, bool mmap_mode, bool quiet, const std::string &rchrom, bool has_region, int rs,
                   int re, int out_fd, Out &err) {
    LineEmitter em(in.p, in.n, out_fd);
    const char *p = in.p, *end = in.p + in.n, *ls, *le;
    bool found = false;
    int ns = 0;
    size_t data_start = in.n;
    while (next_line(p, end, ls, le)) {
        if (le == ls) {
            if (!mmap_mode) em.line(ls, le);  // the stdin path echoes empty lines
            continue;
        }
        if (*ls == '#') {
            em.line(ls, le);
            if (is_chrom_line(ls, (size_t)(le - ls))) {
                found = true;
                ns = ld_samples(ls, le);
                data_start = (size_t)(p - in.p);
                break;
            }
            continue;
        }
        if (mmap_mode) {
            if (!quiet) err.put("Error: data line before #CHROM\n");
        } else err.put("Error: encountered data line before #CHROM.\n");
        break;
    }
    uint64_t M = 0;
    vcfxg_ctx *g = nullptr;
    if (found && data_start < in.n) {
        g = gpu(err.fd);
        if (!g) return false;
        uint64_t nl = 0;
        if (!load_input(g, in, err.fd) ||
            !gpu_ok(g, vcfxg_index(g, data_start, &nl), "index", err.fd) ||
            !gpu_ok(g,
                    vcfxg_ld_prepare(g, ns, 0, rchrom.data(), rchrom.size(), has_region ? 1 : 0, rs, re,
                                     mmap_mode ? 0 : 1, &M),
                    "ld_prepare", err.fd))
            return false;
        // every line of the region is echoed (mmap: non-empty ones)
        std::vector<uint64_t> ends(nl);
        if (!gpu_ok(g, vcfxg_line_ends(g, 0, nl, ends.data()), "line_ends", err.fd)) return false;
        uint64_t prev = data_start;
        for (uint64_t i = 0; i < nl; i++) {
            const char *a = in.p + prev, *b = in.p + ends[i];
            prev = ends[i] + 1;
            if (b > a || !mmap_mode) em.line(a, b);
        }
    }
    if (M < 2) {
        const char *t = "#LD_MATRIX_START\nNo or only one variant in the region => no pairwise LD.\n#LD_MATRIX_END\n";
        em.raw(t, strlen(t));
        em.finish();
        return true;
    }
    // labels "CHROM:POS" from the device prefixes "CHROM\tPOS\tID"
    std::vector<uint64_t> poff(M + 1);
    std::string pre;
    {
        uint64_t bytes = 0;
        std::vector<uint64_t> tmp(M + 1);
        if (!gpu_ok(g, vcfxg_ld_prefixes(g, nullptr, ~(size_t)0, tmp.data()), "ld_prefixes", err.fd)) return false;
        bytes = tmp[M];
        pre.resize(bytes);
        if (!gpu_ok(g, vcfxg_ld_prefixes(g, &pre[0], bytes, poff.data()), "ld_prefixes", err.fd)) return false;
    }
    std::vector<std::string> label(M);
    for (uint64_t v = 0; v < M; v++) {
        size_t a = poff[v], t1 = pre.find('\t', a), t2 = pre.find('\t', t1 + 1);
        label[v] = pre.substr(a, t1 - a) + ":" + pre.substr(t1 + 1, t2 - t1 - 1);
    }
    uint64_t cells = 0;
    if (!gpu_ok(g, vcfxg_ld_matrix(g, mmap_mode ? 1 : 0, mmap_mode ? 0 : 1, &cells), "ld_matrix", err.fd)) return false;
    std::string body(cells, '\0');
    if (!gpu_ok(g, vcfxg_fetch_text(g, &body[0], cells), "fetch", err.fd)) return false;
    std::string head = "#LD_MATRIX_START\nIndex/Var";
    for (uint64_t j = 0; j < M; j++) head += "\t" + label[j];
    head += "\n";
    em.raw(head.data(), head.size());
    const uint64_t stride = 7 * M;
    for (uint64_t i = 0; i < M; i++) {
        em.raw(label[i].data(), label[i].size());
        em.raw(body.data() + i * stride, stride);
        em.raw("\n", 1);
    }
    em.raw("#LD_MATRIX_END\n", 15);
    em.finish();
    return true;
}

}  // namespace vcfxh
