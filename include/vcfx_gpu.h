/*
 * vcfx_gpu.h -- C ABI of the MI355X VCF record engine (libvcfx_gpu.so).
 *
 * The drop-in boundary for VCFX's per-line hot path.  The reference has no FFI for this
 * path: its callers reach it through the VCFX_<tool> processes, whose
 * main()s are re-implemented in vcfx_amd/csrc/tools/ on top of this ABI.  Each entry
 * point below names the reference function(s) whose per-record work it replaces.
 *
 * Conventions: plain pointers and sizes; every function returns VCFXG_OK (0) or a
 * negative vcfxg_status and never throws; buffers are caller-owned unless stated; one
 * vcfxg_ctx per device, used by one host thread; all work is ordered on the context's
 * HIP stream (vcfxg_stream()).  There is no CPU fallback: without a usable gfx950 device
 * vcfxg_open() fails with VCFXG_E_NODEV.
 */
#ifndef VCFX_GPU_H
#define VCFX_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vcfxg_ctx vcfxg_ctx;

enum vcfxg_status {
    VCFXG_OK = 0,
    VCFXG_E_NODEV = -1,   /* no HIP device / not gfx950 */
    VCFXG_E_HIP = -2,     /* HIP runtime error (vcfxg_last_error has the text) */
    VCFXG_E_ARG = -3,     /* bad argument */
    VCFXG_E_NOMEM = -4,   /* device or host allocation failed */
    VCFXG_E_STATE = -5,   /* call out of order (e.g. no input loaded / not indexed) */
    VCFXG_E_CAP = -6,     /* caller buffer too small */
    VCFXG_E_DATA = -7     /* the input data is invalid (a BGZF member that does not inflate as zlib would) */
};

/* input semantics of the reference tools: file = the mmap path, stdin = the getline path */
enum vcfxg_mode { VCFXG_MODE_FILE = 0, VCFXG_MODE_STDIN = 1 };

/* per-line status codes written by the record kernels (one byte per line of the indexed
 * region) */
enum vcfxg_line_status {
    VCFXG_LINE_SKIP = 0,     /* empty, '#' header, or a data line the tool skips silently */
    VCFXG_LINE_ROW = 1,      /* data line that produces output (AF row / kept record) */
    VCFXG_LINE_DROP = 2,     /* data line evaluated and not kept (filters) */
    VCFXG_LINE_WARN = 3,     /* data line the tool reports on stderr ("fewer than 9 fields") */
    VCFXG_LINE_HEADER = 4,   /* '#' line (pass-through tools print it) */
    VCFXG_LINE_RECHECK = 5   /* vcfxg_record_filter_ex: the line needs strtod's prefix value (host) */
};

typedef struct {
    uint64_t n_lines;      /* lines in the indexed region */
    uint64_t rows;         /* output rows (AF) / kept records (filters) */
    uint64_t data_lines;   /* data lines seen (AF "Processed V variants from L data lines") */
    uint64_t warn_lines;   /* lines flagged VCFXG_LINE_WARN */
    uint64_t text_bytes;   /* bytes of device-formatted output text (AF) */
    uint64_t general_records; /* records that took the general (non fixed-stride) GT path */
} vcfxg_summary;

const char *vcfxg_version(void);
int vcfxg_device_count(int *n);
int vcfxg_open(int device, vcfxg_ctx **out);
void vcfxg_close(vcfxg_ctx *ctx);
const char *vcfxg_last_error(const vcfxg_ctx *ctx);
/* the hipStream_t every call of this context is ordered on */
void *vcfxg_stream(vcfxg_ctx *ctx);
/* record HIP events around each kernel launch (see vcfxg_kernel_ms) */
int vcfxg_set_profiling(vcfxg_ctx *ctx, int enable);
/* time only the named kernel (nullptr or "": every kernel); the launches' events are read
   when the figures are asked for, so a profiled loop makes no event queries between calls */
int vcfxg_set_profiling_only(vcfxg_ctx *ctx, const char *kernel);
/* elapsed ms of the last launch of the named kernel ("af_records", "line_index", ...) */
int vcfxg_kernel_ms(vcfxg_ctx *ctx, const char *kernel, float *ms);
/* accumulated event time and launch count of the named kernel since the last reset */
int vcfxg_kernel_stats(vcfxg_ctx *ctx, const char *kernel, double *total_ms, uint64_t *launches);
int vcfxg_reset_kernel_stats(vcfxg_ctx *ctx);

/* ---- input ---------------------------------------------------------------------------
 * The whole input (file or stdin bytes) is made device-resident once; record kernels read
 * it straight from HBM.  Replaces MappedFile::open (VCFX_allele_freq_calc.cpp:47-70) and
 * the std::getline loops' buffering. */
int vcfxg_load_host(vcfxg_ctx *ctx, const char *host, size_t n);
/* Streaming form of the same (SURVEY 8(b) vcfxg_ingest; the pipe paths of processStdin,
 * VCFX_allele_freq_calc.cpp:477-557, VCFX_record_filter.cpp:498-549, VCFX_genotype_query.cpp:
 * 527-617): vcfxg_ingest_begin starts a new input (size_hint = expected bytes, may be 0);
 * each vcfxg_ingest appends n bytes with an asynchronous H2D copy, so the caller's next read
 * overlaps the transfer; the device buffer grows as needed.  The call with is_final_chunk
 * set completes the input, which is then loaded exactly as by vcfxg_load_host.  Every
 * chunk's host bytes must stay valid until that final call returns.
 * vcfxg_load_host(h, n) == vcfxg_ingest_begin(n) + vcfxg_ingest(h, n, 1). */
int vcfxg_ingest_begin(vcfxg_ctx *ctx, size_t size_hint);
int vcfxg_ingest(vcfxg_ctx *ctx, const char *host, size_t n, int is_final_chunk);
/* wait until the copies of the ingested bytes [0, upto) have completed (their host buffers
 * may then be reused: a pinned staging ring) */
int vcfxg_ingest_wait(vcfxg_ctx *ctx, size_t upto);
/* BGZF (.vcf.gz) input inflated on the device (the reference reads it through zlib,
 * StreamingGzipReader, src/vcfx_core.cpp:144-354, members inflated in sequence with inflateReset
 * at each, :270-277).  Appends the inflated bytes of n_members consecutive BGZF members to the
 * input being ingested: comp[0, comp_n) holds them (host memory), member i = the gzip member at
 * comp[src_off, src_off + src_len) (BSIZE + 1 bytes; the caller has checked its header: gzip magic,
 * CM 8, FLG exactly FEXTRA, the 'BC' subfield) whose trailer's ISIZE is out_len (<= 65536).  The
 * compressed bytes are copied to the device and each member is inflated by one wave, its CRC-32
 * checked against the trailer.  head[0, head_n): the first inflated bytes as the caller has them on
 * the host (the load-time hints are taken from them; may be NULL).  A member whose deflate stream
 * zlib would refuse, that does not end at its trailer, or whose size or CRC-32 differs, fails the
 * call with VCFXG_E_DATA (*bad_member = the first such member) and the ingest is abandoned: the
 * caller then inflates on the host, where zlib reports the damage as the reference does. */
typedef struct {
    uint64_t src_off;  /* the member's first byte in comp */
    uint32_t src_len;  /* the member's bytes (BSIZE + 1) */
    uint32_t out_len;  /* its ISIZE */
} vcfxg_bgzf_member;
int vcfxg_ingest_bgzf(vcfxg_ctx *ctx, const void *comp, size_t comp_n, const vcfxg_bgzf_member *members,
                      size_t n_members, const char *head, size_t head_n, uint64_t *bad_member);
/* The compressed bytes for vcfxg_ingest_bgzf copied to the device piece by piece while the caller
 * still reads the file (a pinned staging ring): bytes [offset, offset + n) of a comp_total-byte
 * stream, in order (offset 0 first; each piece starts where the last ended), asynchronous;
 * vcfxg_ingest_wait(ctx, offset + n) waits for the copy (the host buffer may then be reused).
 * Between vcfxg_ingest_begin and vcfxg_ingest_bgzf, which then takes comp = NULL and
 * comp_n = comp_total. */
int vcfxg_bgzf_stage(vcfxg_ctx *ctx, const void *host, size_t n, size_t offset, size_t comp_total);
/* While staging: launch the inflate of the stream's next `count` members (in chain order from the
 * first; every byte of them already staged), overlapping the copies still to come.  VCFXG_E_CAP:
 * their output does not fit the input buffer as allocated (vcfxg_ingest_begin's size hint) --
 * nothing launched; vcfxg_ingest_bgzf inflates them after growing it.  vcfxg_ingest_bgzf(comp =
 * NULL) then takes the whole member list, launches the members not launched yet and checks every
 * member's CRC-32. */
int vcfxg_bgzf_inflate(vcfxg_ctx *ctx, const vcfxg_bgzf_member *members, size_t count);
/* Members of the last vcfxg_ingest_bgzf that the lane decoder (one member per lane) handed to the
 * wave decoder (one member per wave): stored and fixed-code blocks, codes zlib allows only as a
 * special case, members under 384 bytes, damaged streams (diagnostic; the output is the same). */
uint64_t vcfxg_bgzf_handed_over(const vcfxg_ctx *ctx);
/* page-locked host memory (H2D at the full PCIe rate, asynchronous), for staging rings */
int vcfxg_host_alloc(vcfxg_ctx *ctx, size_t n, void **out);
void vcfxg_host_free(vcfxg_ctx *ctx, void *p);
/* copy input bytes [offset, offset + n) of the loaded input back to host memory (pass-through
 * tools whose stdin was streamed to the device without a host copy write kept records from
 * these) */
int vcfxg_input_fetch(vcfxg_ctx *ctx, uint64_t offset, size_t n, void *host);
/* device copy of the loaded input (read-only view; valid until the next load) */
const void *vcfxg_input_device_ptr(vcfxg_ctx *ctx);

/* ---- K1: record index ------------------------------------------------------------------
 * Newline scan over [data_start, n): line i spans [start_i, end_i) with end_i the offset
 * of its '\n' (or n).  Replaces findNewlineSIMD (VCFX_allele_freq_calc.cpp:150-187,
 * VCFX_record_filter.cpp:28-60, VCFX_genotype_query.cpp:139-171, VCFX_variant_counter.cpp:
 * 46-89, VCFX_ld_calculator.cpp:91-137) and the line loops around them. */
int vcfxg_index(vcfxg_ctx *ctx, size_t data_start, uint64_t *n_lines);
/* copy line end offsets [first, first+count) to host */
int vcfxg_line_ends(vcfxg_ctx *ctx, uint64_t first, uint64_t count, uint64_t *out);

/* ---- K2: allele frequency --------------------------------------------------------------
 * Per data line: FORMAT -> GT index, per-sample GT -> (ALT, total) allele counts, freq =
 * alt/total (fp64, correctly rounded), formatted row "CHROM\tPOS\tID\tREF\tALT\t%.4f\n"
 * with the mode's rounding rule.  Replaces processMmap (VCFX_allele_freq_calc.cpp:342-472)
 * and processStdin (:477-557) per-record work: findGTIndex :298-316, extractGT :321-337,
 * parseGenotypeAndCount :262-293, writeDouble4 :119-143 / setprecision(4) :553-555. */
int vcfxg_allele_freq(vcfxg_ctx *ctx, int mode, vcfxg_summary *out);
/* vcfxg_index(data_start) + vcfxg_allele_freq(mode) in one call, with the same results and
 * context state as the two calls (the context is indexed afterwards).  The default device
 * schedule for inputs whose first records average >= 512 B is the walk (one HBM pass: each
 * wave walks the records of one chunk, predicting a record's end from the previous record
 * and validating it by the sample sweep itself); otherwise the index sweep + head pass +
 * sample sweep.  VCFXG_AF_FUSED in the environment at vcfxg_open selects a schedule for
 * measurement: 3 = the two-sweep schedule with the line count read back, 7 = the walk, 8 = the
 * two-sweep schedule with one host synchronisation (all results identical). */
int vcfxg_allele_freq_region(vcfxg_ctx *ctx, size_t data_start, int mode, vcfxg_summary *out);
/* ---- K2: genotype query ----------------------------------------------------------------
 * Per line status (vcfxg_line_status): ROW = some sample's GT sub-field matches `query`
 * (flexible: phase- and order-normalised diploid compare; strict: byte equality), DROP,
 * WARN (fewer than 9 fields), HEADER ('#'), SKIP (empty).  The query is pre-parsed here
 * exactly as main() does (parseDiploidAlleles incl. its partial assignment, then sort).
 * strip_cr evaluates each line without a trailing '\r' (the line as VCFX_record_filter
 * emits it, for the fused record_filter | genotype_query pipeline).  Replaces
 * genotypeQueryMmap / genotypeQueryStream per-record work (VCFX_genotype_query.cpp:433-617):
 * skipToField :223-230, findGTIndex :176-194, extractNthField :199-218,
 * genotypeMatchesFast :275-316, checkAnySampleMatches :322-345. */
int vcfxg_genotype_query(vcfxg_ctx *ctx, const char *query, size_t qlen, int strict, int strip_cr,
                         vcfxg_summary *out);

/* ---- K3: record filter -----------------------------------------------------------------
 * One compiled criterion of VCFX_record_filter (FilterCriterion, VCFX_record_filter.h:37-44,
 * as produced by parseSingleCriterion :89-171): target = 0 POS, 1 QUAL, 2 FILTER, 3 INFO
 * key; op = 0 >, 1 >=, 2 <, 3 <=, 4 ==, 5 !=; numeric = the value parsed fully by strtod
 * (value = that double); key = the INFO key (field name); str = the string value. */
typedef struct {
    int target;
    int op;
    int numeric;
    double value;
    const char *key;
    size_t key_len;
    const char *str;
    size_t str_len;
} vcfxg_criterion;

/* Per line status: ROW = data line passes (AND: all criteria, OR: any), DROP, HEADER ('#',
 * printed without its '\r'), SKIP = empty after '\r' strip (printed as "\n").  Numeric
 * comparisons are exact: strtod(field) is never approximated (see vcfxg_num.h).  Replaces
 * evaluateLine / evaluateCriterion (VCFX_record_filter.cpp:333-401), extractField :207-229,
 * extractInfoValue :234-267, parseDouble :273-299 per record. */
int vcfxg_record_filter(vcfxg_ctx *ctx, const vcfxg_criterion *crit, int n, int and_logic, vcfxg_summary *out);
/* The same with the legacy free-function semantics available (VCFX_record_filter.h:99-102,
 * .cpp:668-805, which no tool calls): flags VCFXG_RF_KEEP_CR evaluates each line with its
 * trailing '\r' (processVCF reads with std::getline); criterion target 4 is QUAL as recordPasses
 * treats it in OR mode (an unparsable QUAL compares as whatever strtod made of it: such lines
 * get status VCFXG_LINE_RECHECK for the caller to decide); a numeric FILTER criterion is passed
 * by the caller as the string criterion recordPasses makes of it. */
#define VCFXG_RF_KEEP_CR 1
int vcfxg_record_filter_ex(vcfxg_ctx *ctx, const vcfxg_criterion *crit, int n, int and_logic, int flags,
                           vcfxg_summary *out);

/* Fused `VCFX_record_filter ... | VCFX_genotype_query ...`: the filter as above, then the
 * genotype query on the lines the filter keeps, evaluated as the filter prints them ('\r'
 * stripped).  Status of a filter-kept data line: ROW = query matches, 6 = no match, 7 =
 * "<9 fields" warning; other lines keep the filter's status. */
int vcfxg_filter_query(vcfxg_ctx *ctx, const vcfxg_criterion *crit, int n, int and_logic, const char *query,
                       size_t qlen, int strict, vcfxg_summary *out);

/* vcfxg_index(data_start) followed by vcfxg_record_filter / vcfxg_genotype_query /
 * vcfxg_filter_query, in one call: the same per-line statuses, line ends, summary and context
 * state (the context is indexed afterwards).  For inputs whose first records average >= 512 B
 * the device walks the records without a separate index sweep (one HBM pass: the walk keeps
 * each record's first 8 tab offsets for the filter, the query's fixed-stride sweep validates
 * the record ends it predicts); VCFXG_FQ_WALK=1 / -1 in the environment at vcfxg_open forces /
 * disables that schedule.  Replace the per-record loops of processFileMmap / processStdin
 * (VCFX_record_filter.cpp:406-549) and genotypeQueryMmap / genotypeQueryStream
 * (VCFX_genotype_query.cpp:433-617) including their line splitting. */
int vcfxg_record_filter_region(vcfxg_ctx *ctx, size_t data_start, const vcfxg_criterion *crit, int n, int and_logic,
                               vcfxg_summary *out);
int vcfxg_genotype_query_region(vcfxg_ctx *ctx, size_t data_start, const char *query, size_t qlen, int strict,
                                int strip_cr, vcfxg_summary *out);
int vcfxg_filter_query_region(vcfxg_ctx *ctx, size_t data_start, const vcfxg_criterion *crit, int n, int and_logic,
                              const char *query, size_t qlen, int strict, vcfxg_summary *out);

/* ---- VCFX_nonref_filter (a per-sample GT reducer on the same path) ----
 * Over the indexed region: per line status 1 keep / 2 drop (every sample hom-ref), 4 '#'
 * line, 0 empty; rows = kept lines, data_lines = evaluated lines, general_records = lines
 * off the fixed-stride sweep.  mode VCFXG_MODE_FILE restates filterNonRefMmap +
 * allSamplesHomRefDirect (VCFX_nonref_filter.cpp:458-551, 248-312; '\r' stripped),
 * VCFXG_MODE_STDIN filterNonRef + isDefinitelyHomRef (:553-636, 419-449).  Data lines
 * before '#CHROM' are the caller's (the tool warns and passes them through). */
int vcfxg_nonref_filter(vcfxg_ctx *ctx, int mode, vcfxg_summary *out);
/* The same over the data region from data_start without a separate index (the filter /
 * query walk with the nonref reducer; index + vcfxg_nonref_filter for short records). */
int vcfxg_nonref_filter_region(vcfxg_ctx *ctx, size_t data_start, int mode, vcfxg_summary *out);

/* ---- VCFX_hwe_tester (a per-sample GT reducer on the same path) -------
 * Over the data region from data_start (the caller passes the end of the leading '#' lines,
 * as performHWE_Mmap's header loop :466-472 skips them): per data line the genotype classes
 * of parseGenotypeForHWE (VCFX_hwe_tester.cpp:339-378) over every sample, the row rules of
 * performHWE_Mmap (:475-558, mode VCFXG_MODE_FILE) or performHWE_Stdin (:572-607, mode
 * VCFXG_MODE_STDIN), and the rows "CHROM\tPOS\tID\tREF\tALT\t<p>\n" with the p-value of
 * calculateHWE_chisq (:278-315) as appendDouble's truncated 6 digits (:236-268, file) or
 * setprecision(6) (stdin).  Text via vcfxg_fetch_text (without the column header line);
 * rows = output rows, general_records = lines off the fixed-stride sweep.  For long records the
 * device walks them as for the allele frequencies (one HBM pass).
 * The p-value's exp() is the device's: a row whose 6 digits it cannot settle (the values a few
 * ulps either side print differently; practically never) is listed by vcfxg_hwe_rechecks, and
 * the caller writes the 8 bytes at text_offset from the host libm's value of the same counts. */
typedef struct {
    uint64_t text_offset; /* offset of the row's 8 p-value bytes in the fetched text */
    int32_t hom_ref, het, hom_alt;
    int32_t reserved;
} vcfxg_hwe_recheck;
int vcfxg_hwe_region(vcfxg_ctx *ctx, size_t data_start, int mode, vcfxg_summary *out);
/* rows of the last vcfxg_hwe_region call that need the host's p-value: *n = their number,
 * the first min(*n, cap) copied to out (any order) */
int vcfxg_hwe_rechecks(vcfxg_ctx *ctx, vcfxg_hwe_recheck *out, uint64_t cap, uint64_t *n);

/* ---- VCFX_dosage_calculator (a per-sample GT map on the same path) ---
 * Over the data lines from data_start (the byte after the '#CHROM' line; data lines before
 * it are the caller's error): per line the row "CHROM\tPOS\tID\tREF\tALT\t" + one dosage
 * per sample (number of non-zero alleles of a diploid GT, or "NA"), comma separated, "NA" for
 * the record when FORMAT has no GT, of processFileMmap (VCFX_dosage_calculator.cpp:375-588,
 * mode VCFXG_MODE_FILE: '\r' stripped) or calculateDosage (:209-360, mode VCFXG_MODE_STDIN);
 * findGTIndexRaw :160-178, extractGTFromSample :182-203, parseDosageInline :111-156 per
 * sample.  Text via vcfxg_fetch_text (without the column header); rows = output rows,
 * warn_lines = lines with fewer than 10 fields (the caller prints the warning),
 * general_records = lines off the fixed-stride sweep; per-line statuses via
 * vcfxg_fetch_lines (1 row, 3 warning, 0 skipped). */
int vcfxg_dosage_region(vcfxg_ctx *ctx, size_t data_start, int mode, vcfxg_summary *out);

/* ---- VCFX_missing_detector (a per-sample GT predicate on the same path) -
 * Over the lines from data_start (the caller passes the end of the leading '#' lines): per
 * line status 0 empty (after the file mode's '\r' strip), 4 '#' line, 1 data line kept as it
 * is, VCFXG_LINE_MISSING a data line with a missing genotype -- some sample's first ':' sub-
 * field holds a '.' that starts or ends it or touches '/' or '|' (hasMissingGenotypeInSamples,
 * VCFX_missing_detector.cpp:290-336).  vcfxg_fetch_lines gives the statuses and, as alt /
 * total, a flagged line's INFO field [start, end) relative to the line start (the caller
 * writes "MISSING_GENOTYPES=1" into it).  mode VCFXG_MODE_FILE: processMmapZeroCopy
 * (:450-589, '\r' dropped); VCFXG_MODE_STDIN: detectMissingGenotypes (:860-911).
 * data_lines = data lines, rows = flagged lines, general_records = lines ending in '\n' whose
 * sample columns hold any '.' (0: the file mode's pre-scan, sampleColumnsHaveAnyDots
 * :371-445, passes the input through unchanged). */
#define VCFXG_LINE_MISSING 6
int vcfxg_missing_region(vcfxg_ctx *ctx, size_t data_start, int mode, vcfxg_summary *out);

/* ---- VCFX_allele_counter (a per-sample GT reducer, a row per sample) ----
 * Over the indexed lines [first_line, last_line): per data line (non-empty, not '#'; no '\r'
 * handling, as in the reference) the REF / ALT allele counts of parseGenotypeRaw
 * (VCFX_allele_counter.cpp:267-294: digit runs of the sample's GT, 0 counting as REF) for each
 * output slot's sample, formatted as the reference does:
 *   kind 0: "CHROM\tPOS\tID\tREF\tALT\t<name>\t<ref>\t<alt>\n" per slot,
 *   kind 1: "CHROM\tPOS\tID\tREF\tALT\t<sum ref>\t<sum alt>\t<rows>\n" per record,
 *   kind 2: the two counts as int8 bytes per slot.
 * seq 0 = countAllelesMmapMT / processChunk (:550-642, 786-950): every slot a row, a sample past
 * the record's last tab counts 0 / 0, counts printed as int8_t; seq 1 = countAllelesUnified
 * (:1266-1468) / countAllelesStream (:1122-1260): a forward-only cursor (a slot reads the
 * largest index so far), rows stop at the first sample that starts at or past the line end.
 * Text (without the column header) via vcfxg_fetch_text / vcfxg_fetch_text_range; per-line
 * statuses via vcfxg_fetch_lines (1 data line, 4 '#CHROM' line, 0 other).  rows = output rows,
 * data_lines = data lines, warn_lines = '#CHROM' lines in the range (countAllelesStream
 * re-selects at each: the caller splits the range there), general_records = lines off the
 * fixed-stride sweep. */
typedef struct {
    const uint32_t *sample;   /* per output slot: the sample's index (sampleIndices) */
    uint64_t m;               /* output slots */
    const char *names;        /* the slots' sample names, concatenated */
    const uint64_t *name_off; /* m + 1 offsets into names */
    int seq;                  /* selection semantics (above) */
    int kind;                 /* 0 text, 1 aggregate, 2 binary */
} vcfxg_ac_params;
int vcfxg_allele_counter(vcfxg_ctx *ctx, uint64_t first_line, uint64_t last_line, const vcfxg_ac_params *params,
                         vcfxg_summary *out);

/* ---- VCFX_haplotype_phaser (LD reuse in block phasing) ------------------
 * Over the lines from data_start (the byte after the '#CHROM' line): per line status 1 variant,
 * 4 '#' line, 3 "<10 fields", 7 invalid POS, 8 no GT in FORMAT, 0 empty (mode VCFXG_MODE_FILE:
 * phaseHaplotypesMmap / ...MmapStreaming, '\r' stripped first; VCFXG_MODE_STDIN: phaseHaplotypes
 * / ...Streaming, an empty line skipped before the strip), VCFX_haplotype_phaser.cpp:607-1259.
 * Each variant's genotypes are parseGenotypeFast codes (:312-357, the GT sub-field's allele sum,
 * -1 missing); for every variant v > 0 the device computes calculateLDFast (:366-470) of (v - 1,
 * v) over the shorter sample list -- the pair groupVariants (:1275-1322) and the streaming loops
 * test, since the block's last variant is always the previous one -- and the block rule:
 * r^2 >= threshold (and r > 0 when v's CHROM is "1").  n_samples_hint: the header's sample
 * count (the genotype row width; wider records are handled by a second pass).  rows = variants;
 * the text (vcfxg_fetch_text) holds each variant's entry "v:(CHROM:POS)" back to back. */
int vcfxg_haplotype_phaser(vcfxg_ctx *ctx, size_t data_start, int mode, double threshold, uint32_t n_samples_hint,
                           vcfxg_summary *out);
/* per variant of the last call: flags (bit 0 the pair with the previous variant passes the block
 * rule, bit 1 both have the same CHROM; 0 for variant 0), r2 (may be NULL) and the entries'
 * text offsets (n_variants + 1) */
int vcfxg_phaser_variants(vcfxg_ctx *ctx, uint8_t *flags, double *r2, uint64_t *entry_offsets);

/* ---- variant counter -------------------------------------------------------------------
 * Per line status: ROW = data line with >= 8 tab-separated columns (counted), WARN = fewer
 * columns, SKIP = empty or '#'.  strip_cr: drop a trailing '\r' first (file path).
 * Replaces countVariantsMmap / countVariants per-line work (VCFX_variant_counter.cpp:
 * 182-202, 317-389) and hasEightColumnsFast :31-44.  rows = Total Variants. */
int vcfxg_variant_count(vcfxg_ctx *ctx, int strip_cr, vcfxg_summary *out);

/* ---- K4: linkage disequilibrium ---------------------------------------------------------
 * vcfxg_ld_prepare: every data line of the indexed region with >= 10 fields and an integer
 * POS (and inside the region when has_region) becomes a variant: n_samples int8 genotype
 * codes (0/1/2, -1 missing) from each sample's GT prefix, its sums and own variance, and a
 * "CHROM\tPOS\tID" text prefix (ID "." -> "CHROM:POS" when id_dot_to_pos).  Replaces the
 * per-record parse of computeLDStreamingMmap / computeLDMatrixMmap (VCFX_ld_calculator.cpp:
 * 555-613, 697-759): fastParseInt :188-197, extractGT :177-185, parseGenotypeRaw :145-174,
 * LDVariantOpt::computeStats :243-258. */
int vcfxg_ld_prepare(vcfxg_ctx *ctx, int n_samples, int id_dot_to_pos, const char *region_chrom, size_t region_len,
                     int has_region, int region_start, int region_end, int parse_mode, uint64_t *n_variants);
/* vcfxg_index(data_start) + vcfxg_ld_prepare in one call, with the same variants, codes, sums and
 * prefixes.  For records averaging >= 512 B and n_samples <= 4096 the device walks the records
 * without a separate index sweep (one HBM pass) and synchronises with the host once; other
 * inputs take the two calls.  The context is NOT indexed afterwards (call vcfxg_index before
 * vcfxg_line_ends or a per-line call); vcfxg_ld_stream_chunk / vcfxg_ld_fetch_pairs follow as
 * after vcfxg_ld_prepare.  Replaces the same reference code as the two calls it fuses. */
int vcfxg_ld_prepare_region(vcfxg_ctx *ctx, size_t data_start, int n_samples, int id_dot_to_pos,
                            const char *region_chrom, size_t region_len, int has_region, int region_start,
                            int region_end, int parse_mode, uint64_t *n_variants);
/* parse_mode: 0 = fastParseInt POS + parseGenotypeRaw on the GT prefix (file paths, stdin
 * streaming); 1 = the stdin matrix path's std::stoi POS + parseGenotype on the whole
 * sample field (computeLD :1021-1045, parseGenotype :468-482). */
/* the variants' "CHROM\tPOS\tID" prefixes (concatenated) and M+1 offsets */
int vcfxg_ld_prefixes(vcfxg_ctx *ctx, char *text, size_t cap, uint64_t *offsets);
/* Matrix mode body: 7*M*M bytes, row-major, cell (i, j) = "\t" + r^2 text ("1.0000" on the
 * diagonal).  gate = computeRsqFast's own-variance gate (file path) vs computeRsq (stdin);
 * printf4 = setprecision(4) (stdin) vs formatR2 (file).  Replaces the matrix loops of
 * computeLDMatrixMmap :767-858 and computeLD :1050-1078. */
int vcfxg_ld_matrix(vcfxg_ctx *ctx, int gate, int printf4, uint64_t *cell_bytes);
/* Streaming-window pairs for new variants j in [j0, j1): every i with j - window <= i < j
 * (pruned when max_dist > 0 and same CHROM with |POS_j - POS_i| > max_dist), r^2 exactly as
 * computeRsqFast (:397-401 -> :352-393; int8 MFMA sums + correctly rounded fp64 epilogue),
 * kept when r^2 >= threshold, formatted as the reference's output lines (formatR2 :200-211)
 * in its order (j, then i ascending).  Text via vcfxg_fetch_text.  Replaces the window
 * loop of computeLDStreamingMmap :616-646 / computeLDStreaming :954-983. */
int vcfxg_ld_stream_chunk(vcfxg_ctx *ctx, uint64_t j0, uint64_t j1, uint64_t window, double threshold, int max_dist,
                          uint64_t *n_pairs, uint64_t *text_bytes);
/* pairs [first, first + count) of the last vcfxg_ld_stream_chunk call, in output order: variant
 * indices (i < j, into the prepared variants) and the fp64 r^2 each line's text was formatted
 * from (the value computeRsqFast returns, VCFX_ld_calculator.cpp:352-401); any pointer may be NULL */
int vcfxg_ld_fetch_pairs(vcfxg_ctx *ctx, uint64_t first, uint64_t count, uint32_t *vi, uint32_t *vj, double *r2);
/* checks the int8 MFMA operand layout the LD kernels assume (0 mismatches expected) */
int vcfxg_selftest_mfma_i8(vcfxg_ctx *ctx, int *mismatches);
/* checks the FP4 (e2m1, block-scaled) MFMA operand layout of the fast LD kernel */
int vcfxg_selftest_mfma_fp4(vcfxg_ctx *ctx, int *mismatches);

/* ---- multi-GPU shard plan (host-only, needs no device) ---------------
 * world + 1 cut offsets over the data region [lo, n) of `data`: cut i is lo + i*(n - lo)/world
 * advanced to the first line start at or after it (the reference's own split,
 * VCFX_allele_counter.cpp:889-901); shard i = [cuts[i], cuts[i+1]) holds whole records.  The
 * multi-GPU runner (vcfx_amd/shard.py, one process per GPU over torch.distributed / RCCL) hands
 * each rank its shard as a zero-copy view (VCFX_INPUT_VIEW). */
int vcfxg_shard_cuts(const char *data, size_t n, size_t lo, int world, uint64_t *cuts);

/* ---- rank cliques (SURVEY 8(b) vcfxg_shard_run's RCCL lifetime; 8(e) the count all-reduce) ----
 * A clique of n contexts, one per rank of an in-process multi-GPU run (vcfx_tool_main_sharded,
 * include/vcfx_tools.h: one host thread per rank).  On n distinct devices the reductions run
 * over RCCL (librccl loaded at run time; ncclCommInitAll + ncclAllReduce on each rank's stream,
 * over xGMI); ranks sharing a device (a rehearsal on one GPU) reduce on the host.  VCFX_RCCL=0
 * forces the host reduction; VCFX_RCCL=1 forms an RCCL clique for n = 1 too (the one-GPU check of
 * the RCCL path).  vcfxg_comm_allreduce_u64: every rank calls it from its own thread with the
 * same count (<= 64); on return vals holds the sums over all ranks (the host reduction's when the
 * status is not VCFXG_OK). */
typedef struct vcfxg_comm vcfxg_comm;
int vcfxg_comm_init(vcfxg_ctx *const *ctxs, int n, vcfxg_comm **out);
int vcfxg_comm_allreduce_u64(vcfxg_comm *comm, int rank, uint64_t *vals, size_t count);
int vcfxg_comm_uses_rccl(const vcfxg_comm *comm);
/* RCCL all-reduces run by the clique, and how many of them disagreed with the host reduction
 * every call also performs (the vote before the collective: no rank enters it unless every rank
 * staged its values; on any failure all ranks get the host sums and a non-zero status) */
int vcfxg_comm_rccl_stats(vcfxg_comm *comm, uint64_t *calls, uint64_t *mismatches);
void vcfxg_comm_destroy(vcfxg_comm *comm);

/* occurrences of `byte` in the device input's bytes [from, n) (one HBM sweep; the fused chain
 * of vcfx_pipe checks the records for '\r' with it) */
int vcfxg_count_byte(vcfxg_ctx *ctx, uint64_t from, int byte, uint64_t *count);
/* the schedule the last region call took ("af_walk", "af_walk_gt_first", "af_two_sweep", "fq_walk",
 * "fq_two_sweep", ...): a diagnostic for tests; VCFXG_SCHEDULE_LOG=path appends one line per call */
const char *vcfxg_last_schedule(const vcfxg_ctx *ctx);

/* device-formatted output text (without the column header line) */
int vcfxg_fetch_text(vcfxg_ctx *ctx, char *host, size_t cap);
/* bytes [offset, offset + n) of that text (outputs larger than one host buffer) */
int vcfxg_fetch_text_range(vcfxg_ctx *ctx, uint64_t offset, size_t n, void *host);
/* per-line results of the last record kernel: any pointer may be NULL */
int vcfxg_fetch_lines(vcfxg_ctx *ctx, uint64_t first, uint64_t count, int32_t *alt, int32_t *total,
                      uint8_t *status);

#ifdef __cplusplus
}
#endif
#endif
