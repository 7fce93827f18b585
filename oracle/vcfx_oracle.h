/*
 * vcfx_oracle.h -- CPU restatement of the VCFX hot-path tools.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product
 * path (vcfx_amd/, build/) never links or calls anything under oracle/.
 *
 * Pinned against: (1) the reference's own goldens (the expected outputs in jorgeMFS/VCFX tests,
 * copied as data into tests/golden/data/ref/), and (2) the reference binaries
 * compiled here from their own sources by oracle/Makefile.ref (outputs in
 * oracle/_ref/, see tests/golden/make_golden.py).
 */
#ifndef VCFX_ORACLE_H
#define VCFX_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    char *out;      /* stdout bytes (malloc'd) */
    size_t out_len;
    char *err;      /* stderr bytes (malloc'd) */
    size_t err_len;
    int rc;         /* exit code */
} oracle_result;

/* Run a restated tool exactly as `tool argv[1..]` would with `stdin_buf` on stdin.
 * tool is one of "VCFX_allele_freq_calc", "VCFX_record_filter", "VCFX_genotype_query",
 * "VCFX_ld_calculator", "VCFX_variant_counter".  argv[0] is used for getopt messages.
 * Files named in argv are read from disk (mmap semantics = whole file).
 * Returns 0 if the tool name is known, -1 otherwise. */
int oracle_main(const char *tool, int argc, char **argv, const char *stdin_buf,
                size_t stdin_len, oracle_result *res);
void oracle_result_free(oracle_result *res);

/* Per-record allele counts exactly as VCFX_allele_freq_calc's counting rule sees them
 * (processMmap, VCFX_allele_freq_calc.cpp:342-472 when stdin_mode==0; processStdin
 * :477-557 when 1).  For each data record that produces an output row, writes alt and
 * total; returns the number of rows (or -(rows needed) if cap is too small). */
long oracle_af_counts(const char *buf, size_t n, int stdin_mode, int32_t *alt,
                      int32_t *total, size_t cap);

/* r^2 of two int8 genotype vectors exactly as computeRsqFast (VCFX_ld_calculator.cpp:
 * 397-401 -> 352-393, x86 scalar body) computes it. */
double oracle_ld_rsq_fast(const int8_t *g1, const int8_t *g2, size_t n);
/* VCFX_haplotype_phaser calculateLDFast (VCFX_haplotype_phaser.cpp:366-470): r and r^2 */
void oracle_ph_ld(const int8_t *a, const int8_t *b, size_t n, double *r, double *r2);
/* parseGenotypeRaw (VCFX_ld_calculator.cpp:145-174). */
int oracle_ld_parse_gt_raw(const char *s, size_t len);

/* The glibc-printf "%.4f" rendering used by the stdin paths (ostream fixed/
 * setprecision(4)) and writeDouble4 (VCFX_allele_freq_calc.cpp:119-143). */
size_t oracle_fmt_fixed4(double v, char *buf);
size_t oracle_fmt_double4(double v, char *buf);

/* VCFX_hwe_tester: calculateHWE_chisq (VCFX_hwe_tester.cpp:290-315, libm exp/sqrt) and the
 * mmap path's 6-digit truncating appendDouble (:236-268). */
double oracle_hwe_pvalue(int homRef, int het, int homAlt);
size_t oracle_hwe_fmt_mmap(double v, char *buf);

#ifdef __cplusplus
}
#endif
#endif
