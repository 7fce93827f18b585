// tool_dispatch.cpp -- name -> in-process tool entry.
#include <string.h>

#include "tools.h"

namespace vcfxh {
std::recursive_mutex &getopt_mutex() {
    static std::recursive_mutex m;
    return m;
}
}  // namespace vcfxh

extern "C" int vcfx_tool_main(const char *tool, int argc, char **argv, int in_fd, int out_fd, int err_fd) {
    const char *t = strrchr(tool, '/');
    t = t ? t + 1 : tool;
    if (!strcmp(t, "VCFX_allele_freq_calc")) return vcfx_tool_allele_freq_calc(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_genotype_query")) return vcfx_tool_genotype_query(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_record_filter")) return vcfx_tool_record_filter(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_variant_counter")) return vcfx_tool_variant_counter(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_ld_calculator")) return vcfx_tool_ld_calculator(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_nonref_filter")) return vcfx_tool_nonref_filter(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_hwe_tester")) return vcfx_tool_hwe_tester(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_dosage_calculator")) return vcfx_tool_dosage_calculator(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_missing_detector")) return vcfx_tool_missing_detector(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_allele_counter")) return vcfx_tool_allele_counter(argc, argv, in_fd, out_fd, err_fd);
    if (!strcmp(t, "VCFX_haplotype_phaser")) return vcfx_tool_haplotype_phaser(argc, argv, in_fd, out_fd, err_fd);
    return -100;
}
