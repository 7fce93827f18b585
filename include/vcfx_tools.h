/*
 * vcfx_tools.h -- in-process C entry points of the VCFX_<tool> drop-ins (libvcfx_tools.so).
 *
 * Each function runs one tool invocation exactly as the reference executable would with the
 * same argv: argv[0] is the tool name, input comes from a file named in argv (the reference's
 * mmap path) or from in_fd (its stdin path), output bytes go to out_fd, diagnostics to
 * err_fd, and the return value is the process exit code.  The build's executables
 * (build/src/VCFX_<t>/VCFX_<t>) are thin main()s over these; FFI callers (ctypes, cgo, JNI)
 * bind them to run a tool without a process spawn while keeping one device context alive
 * across calls.  They replace:
 *   vcfx_tool_allele_freq_calc  main, VCFX_allele_freq_calc.cpp:590-646
 *   vcfx_tool_record_filter     main/run, VCFX_record_filter.cpp:584-658, 819-827
 *   vcfx_tool_genotype_query    main, VCFX_genotype_query.cpp:624-661
 *   vcfx_tool_ld_calculator     run/main, VCFX_ld_calculator.cpp:1084-1225
 *   vcfx_tool_nonref_filter     run/main, VCFX_nonref_filter.cpp:340-384, 646-652
 *   vcfx_tool_hwe_tester        run/main, VCFX_hwe_tester.cpp:414-449, 614-641, 688-694
 *   vcfx_tool_dosage_calculator run/main, VCFX_dosage_calculator.cpp:52-102, 614-620
 *   vcfx_tool_missing_detector  run/main, VCFX_missing_detector.cpp:943-997, 1010-1013
 *   vcfx_tool_allele_counter    parseArguments/main, VCFX_allele_counter.cpp:352-395, 1473-1536
 *   vcfx_tool_haplotype_phaser  run/main, VCFX_haplotype_phaser.cpp:478-569, 1336-1342
 *   vcfx_tool_variant_counter   run, VCFX_variant_counter.cpp:154-218
 *   vcfx_tool_main              the `vcfx <tool> ...` dispatch (src/vcfx_wrapper/vcfx.cpp:177-187)
 * Without a usable gfx950 device a tool that reaches the record loop writes
 * "no usable MI355X" to err_fd and returns 1 (no CPU fallback).
 */
#ifndef VCFX_TOOLS_H
#define VCFX_TOOLS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int vcfx_tool_allele_freq_calc(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_genotype_query(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_record_filter(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_variant_counter(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_ld_calculator(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_nonref_filter(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_hwe_tester(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_dosage_calculator(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_missing_detector(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_allele_counter(int argc, char **argv, int in_fd, int out_fd, int err_fd);
int vcfx_tool_haplotype_phaser(int argc, char **argv, int in_fd, int out_fd, int err_fd);
/* tool = "VCFX_<name>" (a leading path is ignored); -100 for an unknown tool */
int vcfx_tool_main(const char *tool, int argc, char **argv, int in_fd, int out_fd, int err_fd);
/* The same invocation over ngpu device contexts in this process (one host thread per rank;
 * SURVEY 8(b) vcfxg_shard_run, 8(e)): the record tools (allele_freq_calc, record_filter,
 * genotype_query, nonref_filter, dosage_calculator, hwe_tester, missing_detector,
 * allele_counter) on a file input run each rank on its record range of the file, cut at
 * i*size/ngpu and advanced past the next '\n' (VCFX_allele_counter.cpp:889-901);
 * ld_calculator (streaming) on its share of the pair rows.  Output bytes, stderr text and exit
 * code are those of the single-context run; global counts are all-reduced over the rank clique
 * (vcfxg_comm: RCCL on distinct devices).  Other invocations run as vcfx_tool_main.  The
 * executables call it when VCFX_NGPU (a count, or "all") asks for more than one rank; more
 * ranks than devices share devices round robin. */
int vcfx_tool_main_sharded(const char *tool, int argc, char **argv, int in_fd, int out_fd, int err_fd, int ngpu);
/* host-only plan of that run (no device): the ranks used (1 = unsharded), *kind 0 unsharded /
 * 1 record views / 2 LD rows / 3 record views of a BGZF file, and for kinds 1 and 3 the world + 1
 * cut offsets into cuts (kind 3: offsets into the inflated bytes, cuts[0] = the header's end) */
int vcfx_shard_plan(const char *tool, int argc, char **argv, int ngpu, uint64_t *cuts, int *kind);
/* `VCFX_record_filter --filter F --logic L [-i input] | VCFX_genotype_query -g Q [--strict] [-q]`
 * fused in one device pass (BASELINE config 3); input = NULL reads in_fd.  The return value is
 * genotype_query's exit code; record_filter's stderr is written to err_fd first. */
int vcfx_pipeline_filter_query(const char *filter, const char *logic, const char *input, const char *query, int strict,
                               int gq_quiet, int in_fd, int out_fd, int err_fd);

/* `vcfx_pipe 'VCFX_<t> [args] | VCFX_<t> [args] | ...'` (argc == 2: one chain string with shell
 * quoting; argc > 2: the words, "|" separating stages): the reference's stdin -> stdout chaining
 * (README.md:60-66) in one process on one device context, stdout byte-identical to the shell
 * pipeline.  record_filter / genotype_query / nonref_filter stages ending in allele_freq_calc
 * or a filter run fused (the input in HBM once, one walk per stage, decisions AND-ed); other
 * chains run stage by stage in-process.  Exit code: the last stage's (VCFX_PIPEFAIL=1: the last
 * non-zero); VCFX_PIPE_FUSED=0 forces the stage-by-stage schedule. */
int vcfx_pipe_main(int argc, char **argv, int in_fd, int out_fd, int err_fd);

#ifdef __cplusplus
}
#endif
#endif
