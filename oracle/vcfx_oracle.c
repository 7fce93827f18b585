/*
 * vcfx_oracle.c -- CPU restatement (plain C) of the five VCFX hot-path tools, both
 * input modes (file = the reference's mmap path, stdin = its getline path).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for parity tests, smoke() and bench.py's
 * cpu_baseline leg.  Nothing in the product (vcfx_amd/, build/) links or calls it.
 *
 * Every function cites the reference function it restates; citations are
 * /root/reference/src/<dir>/<file>:<line>.  Parity of this restatement is pinned by
 * tests/test_oracle.py against (a) the reference's committed goldens and (b) goldens
 * produced by the reference binaries built from source (oracle/Makefile.ref).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; x86-64 default = no FMA, which is
 * what the reference's double arithmetic assumes).
 */
#define _GNU_SOURCE
#include "vcfx_oracle.h"

#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <getopt.h>
#include <limits.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

/* ------------------------------------------------------------------------------------ */
/* growable byte buffer                                                                 */
/* ------------------------------------------------------------------------------------ */
typedef struct { char *p; size_t n, cap; } ob_t;

static void ob_reserve(ob_t *b, size_t extra) {
    if (b->n + extra <= b->cap) return;
    size_t nc = b->cap ? b->cap : 4096;
    while (nc < b->n + extra) nc *= 2;
    b->p = (char *)realloc(b->p, nc);
    b->cap = nc;
}
static void ob_put(ob_t *b, const char *s, size_t n) {
    ob_reserve(b, n);
    if (n) memcpy(b->p + b->n, s, n);
    b->n += n;
}
static void ob_putc(ob_t *b, char c) { ob_reserve(b, 1); b->p[b->n++] = c; }
static void ob_puts(ob_t *b, const char *s) { ob_put(b, s, strlen(s)); }
static void ob_printf(ob_t *b, const char *fmt, ...) {
    char tmp[512];
    va_list ap;
    va_start(ap, fmt);
    int k = vsnprintf(tmp, sizeof tmp, fmt, ap);
    va_end(ap);
    if (k < (int)sizeof tmp) { ob_put(b, tmp, (size_t)k); return; }
    char *big = (char *)malloc((size_t)k + 1);
    va_start(ap, fmt);
    vsnprintf(big, (size_t)k + 1, fmt, ap);
    va_end(ap);
    ob_put(b, big, (size_t)k);
    free(big);
}

typedef struct { const char *p; size_t n; } sv_t;
static sv_t sv(const char *p, size_t n) { sv_t s = {p, n}; return s; }
static int sv_eq(sv_t a, const char *s, size_t n) { return a.n == n && (n == 0 || memcmp(a.p, s, n) == 0); }
static int sv_eqs(sv_t a, const char *s) { return sv_eq(a, s, strlen(s)); }

/* line iterator: std::getline and the mmap loops split identically: segments between
 * '\n', the tail after the last '\n' only if non-empty. */
typedef struct { const char *p, *end; } lines_t;
static int next_line(lines_t *it, const char **ls, const char **le) {
    if (it->p >= it->end) return 0;
    const char *nl = (const char *)memchr(it->p, '\n', (size_t)(it->end - it->p));
    *ls = it->p;
    *le = nl ? nl : it->end;
    it->p = nl ? nl + 1 : it->end;
    return 1;
}
static int starts_chrom(const char *s, size_t n) { return n >= 6 && memcmp(s, "#CHROM", 6) == 0; }

/* read a whole file (the reference mmaps it) */
static int read_file(const char *path, char **data, size_t *n) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    struct stat st;
    if (fstat(fd, &st) < 0) { close(fd); return -1; }
    size_t sz = (size_t)st.st_size;
    char *buf = (char *)malloc(sz ? sz : 1);
    size_t got = 0;
    while (got < sz) {
        ssize_t k = read(fd, buf + got, sz - got);
        if (k <= 0) break;
        got += (size_t)k;
    }
    close(fd);
    *data = buf;
    *n = got;
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* number formatting                                                                    */
/* ------------------------------------------------------------------------------------ */
/* OutputBuffer::writeDouble4, VCFX_allele_freq_calc.cpp:119-143 */
size_t oracle_fmt_double4(double val, char *buf) {
    size_t k = 0;
    if (val < 0) { buf[k++] = '-'; val = -val; }
    unsigned long long scaled = (unsigned long long)(val * 10000.0 + 0.5);
    unsigned long long ip = scaled / 10000, fp = scaled % 10000;
    if (ip == 0) buf[k++] = '0';
    else {
        char t[24]; int i = 0;
        while (ip > 0) { t[i++] = (char)('0' + ip % 10); ip /= 10; }
        while (i > 0) buf[k++] = t[--i];
    }
    buf[k++] = '.';
    buf[k++] = (char)('0' + (fp / 1000) % 10);
    buf[k++] = (char)('0' + (fp / 100) % 10);
    buf[k++] = (char)('0' + (fp / 10) % 10);
    buf[k++] = (char)('0' + fp % 10);
    return k;
}
/* std::fixed << std::setprecision(4) == printf("%.4f") (libstdc++ uses vsnprintf) */
size_t oracle_fmt_fixed4(double v, char *buf) { return (size_t)sprintf(buf, "%.4f", v); }

/* ==================================================================================== */
/* VCFX_allele_freq_calc                                                                */
/* ==================================================================================== */
/* findGTIndex, VCFX_allele_freq_calc.cpp:298-316 */
static int af_find_gt_index(sv_t f) {
    const char *p = f.p, *end = f.p + f.n;
    int idx = 0;
    while (p < end) {
        const char *fs = p;
        while (p < end && *p != ':') ++p;
        if (p - fs == 2 && fs[0] == 'G' && fs[1] == 'T') return idx;
        idx++;
        if (p < end) ++p;
    }
    return -1;
}
/* extractGT, VCFX_allele_freq_calc.cpp:321-337 */
static sv_t af_extract_gt(sv_t s, int gi) {
    const char *p = s.p, *end = s.p + s.n;
    for (int i = 0; i < gi && p < end; ++i) {
        while (p < end && *p != ':') ++p;
        if (p < end) ++p;
    }
    if (p >= end) return sv(NULL, 0);
    const char *g = p;
    while (p < end && *p != ':') ++p;
    return sv(g, (size_t)(p - g));
}
/* parseGenotypeAndCount, VCFX_allele_freq_calc.cpp:262-293 */
static void af_count(sv_t gt, int *alt, int *total) {
    const char *p = gt.p, *end = gt.p + gt.n;
    while (p < end) {
        while (p < end && (*p == '/' || *p == '|')) ++p;
        if (p >= end) break;
        const char *a = p;
        while (p < end && *p != '/' && *p != '|') ++p;
        if (a == p) continue;
        if (*a == '.') continue;
        int zero = 1, num = 1;
        for (const char *c = a; c < p; ++c) {
            if (*c < '0' || *c > '9') { num = 0; break; }
            if (*c != '0') zero = 0;
        }
        if (!num) continue;
        (*total)++;
        if (!zero) (*alt)++;
    }
}
/* findTabSIMD scalar semantics (first '\t', scalar tail also stops at '\n'):
 * VCFX_allele_freq_calc.cpp:189-200 */
static const char *af_find_tab(const char *p, const char *end) {
    while (p < end && *p != '\t' && *p != '\n') ++p;
    return p;
}
/* getField, VCFX_allele_freq_calc.cpp:247-256 */
static sv_t af_get_field(const char *ls, const char *le, int idx) {
    const char *p = ls;
    for (int i = 0; i < idx && p < le; ++i) {
        p = af_find_tab(p, le);
        if (p < le) ++p;
    }
    if (p >= le) return sv(NULL, 0);
    const char *fe = af_find_tab(p, le);
    return sv(p, (size_t)(fe - p));
}

typedef void (*af_row_fn)(void *u, sv_t prefix_from_line_start, int alt, int total);

/* processMmap, VCFX_allele_freq_calc.cpp:342-472 (row callback instead of buffer) */
static void af_mmap_core(const char *data, size_t n, int quiet, ob_t *out, ob_t *err,
                         size_t *variants, size_t *datalines, int32_t *alt_o, int32_t *tot_o,
                         size_t cap, long *rows) {
    const char *p = data, *end = data + n;
    int found = 0;
    size_t lc = 0, vc = 0;
    if (out) ob_puts(out, "CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n");
    while (p < end) {
        const char *ls = p;
        const char *le = (const char *)memchr(p, '\n', (size_t)(end - p));
        if (!le) le = end;
        const char *ae = le;
        if (ae > ls && ae[-1] == '\r') --ae;
        if (ls == ae) { p = le + 1; continue; }
        if (*ls == '#') {
            if (ae - ls >= 6 && memcmp(ls, "#CHROM", 6) == 0) found = 1;
            p = le + 1;
            continue;
        }
        if (!found) {
            if (!quiet && err) ob_puts(err, "Warning: Data line encountered before #CHROM header. Skipping.\n");
            p = le + 1;
            continue;
        }
        lc++;
        sv_t f[5];
        for (int i = 0; i < 5; i++) f[i] = af_get_field(ls, ae, i);
        sv_t fmt = af_get_field(ls, ae, 8);
        if (fmt.n == 0) { p = le + 1; continue; }
        int gi = af_find_gt_index(fmt);
        if (gi < 0) { p = le + 1; continue; }
        int alt = 0, tot = 0;
        const char *s = ls;
        int fi = 0;
        while (fi < 9 && s < ae) {
            s = af_find_tab(s, ae);
            if (s < ae) { ++s; ++fi; }
        }
        while (s < ae) {
            const char *se = af_find_tab(s, ae);
            sv_t g = af_extract_gt(sv(s, (size_t)(se - s)), gi);
            if (g.n) af_count(g, &alt, &tot);
            if (se >= ae) break;
            s = se + 1;
        }
        double freq = tot > 0 ? (double)alt / (double)tot : 0.0;
        if (out) {
            for (int i = 0; i < 5; i++) { ob_put(out, f[i].p, f[i].n); ob_putc(out, '\t'); }
            char nb[64];
            size_t k = oracle_fmt_double4(freq, nb);
            ob_put(out, nb, k);
            ob_putc(out, '\n');
        }
        if (rows) {
            if ((size_t)*rows < cap) { alt_o[*rows] = alt; tot_o[*rows] = tot; }
            (*rows)++;
        }
        vc++;
        p = le + 1;
    }
    *variants = vc;
    *datalines = lc;
}

/* the stdin path's field split (VCFX_allele_freq_calc.cpp:509-518): no empty last field
 * after a trailing tab */
static size_t af_split_stdin(const char *ls, const char *le, sv_t *f, size_t cap, size_t *total) {
    size_t nf = 0, start = 0, len = (size_t)(le - ls);
    while (start < len) {
        const char *t = (const char *)memchr(ls + start, '\t', len - start);
        if (!t) { if (nf < cap) f[nf] = sv(ls + start, len - start); nf++; break; }
        if (nf < cap) f[nf] = sv(ls + start, (size_t)(t - (ls + start)));
        nf++;
        start = (size_t)(t - ls) + 1;
    }
    *total = nf;
    return nf;
}

/* processStdin, VCFX_allele_freq_calc.cpp:477-557 */
static void af_stdin_core(const char *data, size_t n, int quiet, ob_t *out, ob_t *err,
                          int32_t *alt_o, int32_t *tot_o, size_t cap, long *rows) {
    lines_t it = {data, data + n};
    const char *ls, *le;
    int found = 0;
    if (out) ob_puts(out, "CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n");
    while (next_line(&it, &ls, &le)) {
        if (ls == le) continue;
        if (*ls == '#') {
            if (starts_chrom(ls, (size_t)(le - ls))) found = 1;
            continue;
        }
        if (!found) {
            if (!quiet && err) ob_puts(err, "Warning: Data line encountered before #CHROM header. Skipping.\n");
            continue;
        }
        /* first 9 fields + iterate samples by rescanning (same split rule) */
        sv_t f[9];
        size_t nf = 0;
        af_split_stdin(ls, le, f, 9, &nf);
        if (nf < 9) {
            if (!quiet && err) ob_puts(err, "Warning: Skipping invalid VCF line (fewer than 9 fields).\n");
            continue;
        }
        int gi = af_find_gt_index(f[8]);
        if (gi < 0) continue;
        int alt = 0, tot = 0;
        /* fields[9..]: walk the same split from after field 8 */
        size_t len = (size_t)(le - ls);
        size_t start = (size_t)(f[8].p + f[8].n - ls);
        /* position after FORMAT: if FORMAT was the last field (no tab) there are no samples */
        if (start < len) {
            start += 1; /* skip the tab */
            while (start < len) {
                const char *t = (const char *)memchr(ls + start, '\t', len - start);
                sv_t s = t ? sv(ls + start, (size_t)(t - (ls + start))) : sv(ls + start, len - start);
                sv_t g = af_extract_gt(s, gi);
                if (g.n) af_count(g, &alt, &tot);
                if (!t) break;
                start = (size_t)(t - ls) + 1;
            }
        }
        double freq = tot > 0 ? (double)alt / (double)tot : 0.0;
        if (out) {
            for (int i = 0; i < 5; i++) { ob_put(out, f[i].p, f[i].n); ob_putc(out, '\t'); }
            char nb[64];
            size_t k = oracle_fmt_fixed4(freq, nb);
            ob_put(out, nb, k);
            ob_putc(out, '\n');
        }
        if (rows) {
            if ((size_t)*rows < cap) { alt_o[*rows] = alt; tot_o[*rows] = tot; }
            (*rows)++;
        }
    }
}

long oracle_af_counts(const char *buf, size_t n, int stdin_mode, int32_t *alt, int32_t *total,
                      size_t cap) {
    long rows = 0;
    if (stdin_mode) af_stdin_core(buf, n, 1, NULL, NULL, alt, total, cap, &rows);
    else {
        size_t v, l;
        af_mmap_core(buf, n, 1, NULL, NULL, &v, &l, alt, total, cap, &rows);
    }
    return (size_t)rows <= cap ? rows : -rows;
}

/* printHelp, VCFX_allele_freq_calc.cpp:562-585 */
static void af_help(ob_t *o) {
    ob_puts(o,
        "VCFX_allele_freq_calc v1.1 - High-performance allele frequency calculator\n\n"
        "Usage:\n"
        "  VCFX_allele_freq_calc [OPTIONS] [input.vcf]\n"
        "  VCFX_allele_freq_calc [OPTIONS] < input.vcf > output.tsv\n\n"
        "Options:\n"
        "  -i, --input FILE   Input VCF file (uses memory-mapping for best performance)\n"
        "  -q, --quiet        Suppress informational messages\n"
        "  -h, --help         Display this help message and exit\n"
        "  -v, --version      Show program version and exit\n\n"
        "Description:\n"
        "  Calculates allele frequency for each variant in a VCF file.\n"
        "  Allele frequency is computed as (#ALT alleles) / (total #alleles),\n"
        "  counting any non-zero numeric allele (1,2,3,...) as ALT.\n\n"
        "Output Format:\n"
        "  CHROM  POS  ID  REF  ALT  Allele_Frequency\n\n"
        "Performance:\n"
        "  - Memory-mapped I/O: Use -i flag for ~15-20x faster processing\n"
        "  - SIMD acceleration for line/field scanning\n"
        "  - Zero-copy parsing with string_view\n\n"
        "Examples:\n"
        "  VCFX_allele_freq_calc -i input.vcf > frequencies.tsv\n"
        "  VCFX_allele_freq_calc < input.vcf > frequencies.tsv\n");
}

/* getopt error messages go to stderr; capture them by pointing stderr at a memstream */
typedef struct { FILE *saved; char *buf; size_t len; FILE *mem; } errcap_t;
static void errcap_begin(errcap_t *c) {
    fflush(stderr);
    c->buf = NULL; c->len = 0;
    c->mem = open_memstream(&c->buf, &c->len);
    c->saved = stderr;
    stderr = c->mem;
}
static void errcap_end(errcap_t *c, ob_t *err) {
    fflush(c->mem);
    stderr = c->saved;
    fclose(c->mem);
    if (c->len) ob_put(err, c->buf, c->len);
    free(c->buf);
}

/* main, VCFX_allele_freq_calc.cpp:590-646 */
static int af_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    const char *input = NULL;
    int quiet = 0;
    static struct option lo[] = {{"input", required_argument, NULL, 'i'},
                                 {"quiet", no_argument, NULL, 'q'},
                                 {"help", no_argument, NULL, 'h'},
                                 {"version", no_argument, NULL, 'v'},
                                 {NULL, 0, NULL, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    int opt, rc = -1;
    while ((opt = getopt_long(argc, argv, "i:qhv", lo, NULL)) != -1) {
        if (opt == 'i') input = optarg;
        else if (opt == 'q') quiet = 1;
        else if (opt == 'h') { af_help(out); rc = 0; break; }
        else if (opt == 'v') { ob_puts(out, "VCFX_allele_freq_calc v1.1\n"); rc = 0; break; }
        else { af_help(out); rc = 1; break; }
    }
    errcap_end(&ec, err);
    if (rc >= 0) return rc;
    if (!input && optind < argc) input = argv[optind];
    if (input) {
        char *data; size_t n;
        if (read_file(input, &data, &n) < 0) {
            ob_printf(err, "Error: Cannot open file: %s\n", input);
            return 1;
        }
        if (!quiet) ob_printf(err, "Processing %s (%zu MB)\n", input, n / (1024 * 1024));
        size_t v, l;
        af_mmap_core(data, n, quiet, out, err, &v, &l, NULL, NULL, 0, NULL);
        if (!quiet) ob_printf(err, "Processed %zu variants from %zu data lines\n", v, l);
        free(data);
    } else {
        if (inn == 0) { af_help(out); return 1; }
        af_stdin_core(in, inn, quiet, out, err, NULL, NULL, 0, NULL);
    }
    return 0;
}

/* ==================================================================================== */
/* common flags (vcfx_core.h:31-62, vcfx_core.cpp:31-44)                                 */
/* ==================================================================================== */
static int flag_present(int argc, char **argv, const char *l, const char *s) {
    for (int i = 1; i < argc; ++i)
        if (strcmp(argv[i], l) == 0 || (s && strcmp(argv[i], s) == 0)) return 1;
    return 0;
}
/* returns 1 if handled */
static int common_flags(int argc, char **argv, const char *tool, void (*help)(ob_t *), ob_t *out) {
    if (flag_present(argc, argv, "--help", "-h")) { help(out); return 1; }
    if (flag_present(argc, argv, "--version", "-v")) {
        ob_printf(out, "%s version %s\n", tool, "1.1.4");
        return 1;
    }
    return 0;
}

/* ==================================================================================== */
/* VCFX_variant_counter                                                                 */
/* ==================================================================================== */
static void vc_help(ob_t *o) {
    ob_puts(o,
        "VCFX_variant_counter: Counts the total number of valid variants in a VCF.\n\n"
        "Usage:\n"
        "  VCFX_variant_counter [options] [input.vcf]\n"
        "  VCFX_variant_counter [options] < input.vcf\n\n"
        "Options:\n"
        "  -h, --help        Show this help.\n"
        "  -s, --strict      Fail on any data line with <8 columns.\n\n"
        "Description:\n"
        "  Reads a VCF from file argument or stdin. For each data line,\n"
        "  we check if it has >=8 columns; if it does, we count it; if fewer columns:\n"
        "   * if --strict => we exit with error,\n"
        "   * otherwise => we skip with a warning.\n"
        "  When a file is provided directly, uses memory-mapped I/O for faster processing.\n"
        "  Finally, we print 'Total Variants: X'.\n\n"
        "Example:\n"
        "  VCFX_variant_counter input.vcf          # Fast memory-mapped mode\n"
        "  VCFX_variant_counter < input.vcf        # Stdin mode\n"
        "  VCFX_variant_counter --strict input.vcf\n");
}
/* hasEightColumnsFast, VCFX_variant_counter.cpp:31-44 */
static int vc_has8(const char *s, size_t n) {
    if (n == 0) return 0;
    const char *p = s, *end = s + n;
    for (int i = 0; i < 7; i++) {
        p = (const char *)memchr(p, '\t', (size_t)(end - p));
        if (!p) return 0;
        p++;
    }
    return 1;
}
/* processLine / processLineMmap, VCFX_variant_counter.cpp:182-202, 293-313 */
static int vc_line(const char *s, size_t n, int ln, int *count, int strict, ob_t *err) {
    if (n == 0 || s[0] == '#') return 1;
    if (vc_has8(s, n)) { (*count)++; return 1; }
    if (strict) { ob_printf(err, "Error: line %d has <8 columns.\n", ln); return 0; }
    ob_printf(err, "Warning: skipping line %d with <8 columns.\n", ln);
    return 1;
}
/* countVariantsMmap, VCFX_variant_counter.cpp:317-389 */
static int vc_mmap(const char *d, size_t n, int strict, ob_t *err) {
    const char *p = d, *end = d + n;
    int count = 0, ln = 0;
    while (p < end) {
        const char *le = (const char *)memchr(p, '\n', (size_t)(end - p));
        if (!le) le = end;
        ln++;
        size_t len = (size_t)(le - p);
        if (len > 0 && *p != '#') {
            if (p[len - 1] == '\r') len--;
            if (vc_has8(p, len)) count++;
            else if (strict) { ob_printf(err, "Error: line %d has <8 columns.\n", ln); return -1; }
            else ob_printf(err, "Warning: skipping line %d with <8 columns.\n", ln);
        }
        p = le + 1;
    }
    return count;
}
/* countVariants, VCFX_variant_counter.cpp:204-221 */
static int vc_stdin(const char *d, size_t n, int strict, ob_t *err) {
    lines_t it = {d, d + n};
    const char *ls, *le;
    int count = 0, ln = 0;
    while (next_line(&it, &ls, &le)) {
        ln++;
        if (!vc_line(ls, (size_t)(le - ls), ln, &count, strict, err)) return -1;
    }
    return count;
}
/* countVariantsGzip, VCFX_variant_counter.cpp:223-290 */
static int vc_gzip(const char *d, size_t n, int strict, ob_t *err) {
    enum { CHUNK = 65536 };
    z_stream s;
    memset(&s, 0, sizeof s);
    if (inflateInit2(&s, 15 + 32) != Z_OK) { ob_puts(err, "Error: inflateInit2 failed.\n"); return -1; }
    static char outb[CHUNK];
    ob_t buf = {0};
    size_t off = 0, ip = 0;
    int count = 0, ln = 0, ret = Z_OK;
    do {
        size_t take = n - ip < CHUNK ? n - ip : CHUNK;
        const char *chunk = d + ip;
        ip += take;
        s.avail_in = (uInt)take;
        if (s.avail_in == 0 && ip >= n) break;
        s.next_in = (Bytef *)chunk;
        do {
            s.avail_out = CHUNK;
            s.next_out = (Bytef *)outb;
            ret = inflate(&s, Z_NO_FLUSH);
            if (ret == Z_STREAM_ERROR || ret == Z_NEED_DICT || ret == Z_DATA_ERROR || ret == Z_MEM_ERROR) {
                ob_puts(err, "Error: decompression failed.\n");
                inflateEnd(&s); free(buf.p);
                return -1;
            }
            size_t have = CHUNK - s.avail_out;
            if (have > 0) {
                ob_put(&buf, outb, have);
                for (;;) {
                    const char *nl = (const char *)memchr(buf.p + off, '\n', buf.n - off);
                    if (!nl) break;
                    size_t pos = (size_t)(nl - buf.p);
                    ln++;
                    if (!vc_line(buf.p + off, pos - off, ln, &count, strict, err)) {
                        inflateEnd(&s); free(buf.p);
                        return -1;
                    }
                    off = pos + 1;
                }
                if (off > 0 && off > buf.n / 2) {
                    memmove(buf.p, buf.p + off, buf.n - off);
                    buf.n -= off;
                    off = 0;
                }
            }
        } while (s.avail_out == 0);
    } while (ret != Z_STREAM_END);
    if (off < buf.n) {
        ln++;
        if (!vc_line(buf.p + off, buf.n - off, ln, &count, strict, err)) {
            inflateEnd(&s); free(buf.p);
            return -1;
        }
    }
    inflateEnd(&s);
    free(buf.p);
    return count;
}
/* run, VCFX_variant_counter.cpp:116-180 + main :399-405 */
static int vc_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_variant_counter", vc_help, out)) return 0;
    int show = 0, strict = 0;
    static struct option lo[] = {{"help", no_argument, 0, 'h'}, {"strict", no_argument, 0, 's'}, {0, 0, 0, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    for (;;) {
        int c = getopt_long(argc, argv, "hs", lo, NULL);
        if (c == -1) break;
        if (c == 'h') show = 1;
        else if (c == 's') strict = 1;
        else show = 1;
    }
    errcap_end(&ec, err);
    if (show) { vc_help(out); return 0; }
    int total;
    if (optind < argc) {
        char *d; size_t n;
        if (read_file(argv[optind], &d, &n) < 0) {
            ob_printf(err, "Error: cannot open file: %s\n", argv[optind]);
            return 1;
        }
        total = n ? vc_mmap(d, n, strict, err) : 0;
        free(d);
    } else {
        if (inn == 0) total = 0;
        else if (inn >= 2 && (unsigned char)in[0] == 0x1f && (unsigned char)in[1] == 0x8b)
            total = vc_gzip(in, inn, strict, err);
        else total = vc_stdin(in, inn, strict, err);
    }
    if (total < 0) return 1;
    ob_printf(out, "Total Variants: %d\n", total);
    return 0;
}

/* ==================================================================================== */
/* VCFX_genotype_query                                                                  */
/* ==================================================================================== */
static void gq_help(ob_t *o) {
    ob_puts(o,
        "VCFX_genotype_query\n"
        "Usage: VCFX_genotype_query [OPTIONS] [input.vcf]\n\n"
        "Options:\n"
        "  -g, --genotype-query GT  Genotype to query (e.g., \"0/1\", \"1|1\")\n"
        "  -i, --input FILE         Input VCF file (uses fast memory-mapped I/O)\n"
        "  --strict                 Exact string matching (no normalization)\n"
        "  -q, --quiet              Suppress warning messages to stderr\n"
        "  -h, --help               Display this help message and exit\n"
        "  -v, --version            Show program version and exit\n\n"
        "Description:\n"
        "  Filters a VCF to retain only lines where at least one sample has the\n"
        "  specified genotype in the 'GT' subfield.\n\n"
        "  By default, phasing is unified (0|1 matches 0/1) and allele order is\n"
        "  normalized (1/0 matches 0/1). Use --strict for exact matching.\n\n"
        "Performance:\n"
        "  File input mode (-i) uses memory-mapped I/O with SIMD optimization,\n"
        "  providing 40-50x speedup over stdin mode for large files.\n\n"
        "Examples:\n"
        "  # Flexible matching (0/1 matches 0|1, 1/0, 1|0)\n"
        "  VCFX_genotype_query -g \"0/1\" < input.vcf > het.vcf\n"
        "  VCFX_genotype_query -g \"0/1\" -i input.vcf > het.vcf\n\n"
        "  # Strict matching (only exact 0|1)\n"
        "  VCFX_genotype_query -g \"0|1\" --strict < input.vcf > phased_het.vcf\n");
}
/* findGTIndex, VCFX_genotype_query.cpp:176-194 */
static int gq_find_gt_index(sv_t f) {
    const char *p = f.p, *end = f.p + f.n, *fs = f.p;
    int idx = 0;
    while (p <= end) {
        if (p == end || *p == ':') {
            if (p - fs == 2 && fs[0] == 'G' && fs[1] == 'T') return idx;
            idx++;
            fs = p + 1;
        }
        p++;
    }
    return -1;
}
/* extractNthField, VCFX_genotype_query.cpp:199-218 */
static sv_t gq_nth(sv_t s, int n) {
    if (n < 0) return sv(NULL, 0);
    const char *p = s.p, *end = s.p + s.n, *fs = s.p;
    int fi = 0;
    while (p <= end) {
        if (p == end || *p == ':') {
            if (fi == n) return sv(fs, (size_t)(p - fs));
            fi++;
            fs = p + 1;
        }
        p++;
    }
    return sv(NULL, 0);
}
/* skipToField, VCFX_genotype_query.cpp:223-230 */
static const char *gq_skip(const char *p, const char *end, int n) {
    for (int i = 0; i < n && p < end; i++) {
        p = (const char *)memchr(p, '\t', (size_t)(end - p));
        if (!p) return NULL;
        p++;
    }
    return p;
}
/* parseDiploidAlleles, VCFX_genotype_query.cpp:246-272 (partial assignment on failure is
 * observable through the query parse and is kept) */
static int gq_parse_diploid(sv_t g, int *a1, int *a2) {
    size_t sep = (size_t)-1;
    for (size_t i = 0; i < g.n; i++)
        if (g.p[i] == '|' || g.p[i] == '/') { sep = i; break; }
    if (sep == (size_t)-1 || sep == 0 || sep == g.n - 1) return 0;
    sv_t f = sv(g.p, sep);
    if (sv_eqs(f, ".")) return 0;
    unsigned v = 0;
    *a1 = 0;
    for (size_t i = 0; i < f.n; i++) {
        if (!isdigit((unsigned char)f.p[i])) return 0;
        v = v * 10u + (unsigned)(f.p[i] - '0');
        *a1 = (int)v;
    }
    sv_t s = sv(g.p + sep + 1, g.n - sep - 1);
    if (sv_eqs(s, ".")) return 0;
    v = 0;
    *a2 = 0;
    for (size_t i = 0; i < s.n; i++) {
        if (!isdigit((unsigned char)s.p[i])) return 0;
        v = v * 10u + (unsigned)(s.p[i] - '0');
        *a2 = (int)v;
    }
    return 1;
}
/* genotypeMatchesFast, VCFX_genotype_query.cpp:275-316 */
static int gq_match(sv_t gt, sv_t q, int qa, int qb, int strict) {
    if (strict) return gt.n == q.n && memcmp(gt.p, q.p, gt.n) == 0;
    if (gt.n == 3 && q.n == 3) {
        char s = gt.p[1];
        if (s != '|' && s != '/') return 0;
        char g0 = gt.p[0], g1 = gt.p[2];
        if (g0 == '.' || g1 == '.') return 0;
        if (!isdigit((unsigned char)g0) || !isdigit((unsigned char)g1)) return 0;
        int ga = g0 - '0', gb = g1 - '0';
        if (ga > gb) { int t = ga; ga = gb; gb = t; }
        if (qa > qb) { int t = qa; qa = qb; qb = t; }
        return ga == qa && gb == qb;
    }
    int a1, a2;
    if (!gq_parse_diploid(gt, &a1, &a2)) return 0;
    if (a1 > a2) { int t = a1; a1 = a2; a2 = t; }
    if (qa > qb) { int t = qa; qa = qb; qb = t; }
    return a1 == qa && a2 == qb;
}
/* checkAnySampleMatches, VCFX_genotype_query.cpp:322-345 */
static int gq_any(const char *ls, const char *le, int gi, sv_t q, int qa, int qb, int strict) {
    const char *p = gq_skip(ls, le, 9);
    if (!p) return 0;
    while (p < le) {
        const char *se = (const char *)memchr(p, '\t', (size_t)(le - p));
        if (!se) se = le;
        sv_t g = gq_nth(sv(p, (size_t)(se - p)), gi);
        if (g.n && gq_match(g, q, qa, qb, strict)) return 1;
        p = se + 1;
    }
    return 0;
}
/* genotypeQueryMmap, VCFX_genotype_query.cpp:433-517 */
static void gq_mmap(const char *d, size_t n, ob_t *out, ob_t *err, sv_t q, int qa, int qb, int strict, int quiet) {
    if (n == 0) return;
    const char *p = d, *end = d + n;
    int found = 0;
    while (p < end) {
        const char *le = (const char *)memchr(p, '\n', (size_t)(end - p));
        if (!le) le = end;
        if (le == p) { p = le + 1; continue; }
        size_t len = (size_t)(le - p);
        if (p[0] == '#') {
            if (starts_chrom(p, len)) found = 1;
            ob_put(out, p, len);
            ob_putc(out, '\n');
        } else {
            if (!found) {
                if (!quiet) ob_puts(err, "Error: No #CHROM header found before data lines.\n");
                return;
            }
            const char *fs = gq_skip(p, le, 8);
            if (!fs) {
                if (!quiet) ob_puts(err, "Warning: skipping line with <9 fields\n");
                p = le + 1;
                continue;
            }
            const char *fe = (const char *)memchr(fs, '\t', (size_t)(le - fs));
            if (!fe) fe = le;
            int gi = gq_find_gt_index(sv(fs, (size_t)(fe - fs)));
            if (gi < 0) { p = le + 1; continue; }
            if (gq_any(p, le, gi, q, qa, qb, strict)) { ob_put(out, p, len); ob_putc(out, '\n'); }
        }
        p = le + 1;
    }
}
/* genotypeQueryStream, VCFX_genotype_query.cpp:527-617 */
static void gq_stream(const char *d, size_t n, ob_t *out, ob_t *err, sv_t q, int strict, int quiet) {
    int found = 0;
    int qa = -1, qb = -1;
    if (!strict) {
        gq_parse_diploid(q, &qa, &qb);
        if (qa > qb) { int t = qa; qa = qb; qb = t; }
    }
    ob_t hdr = {0};   /* buffered header lines, each followed by '\n' */
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        size_t len = (size_t)(le - ls);
        if (len == 0) continue;
        if (ls[0] == '#') {
            ob_put(&hdr, ls, len);
            ob_putc(&hdr, '\n');
            if (starts_chrom(ls, len)) found = 1;
        } else {
            if (!found) {
                if (!quiet) ob_puts(err, "Error: No #CHROM header found before data lines.\n");
                free(hdr.p);
                return;
            }
            if (hdr.n) { ob_put(out, hdr.p, hdr.n); hdr.n = 0; }
            const char *fs = gq_skip(ls, le, 8);
            if (!fs) {
                if (!quiet) {
                    ob_puts(err, "Warning: skipping line with <9 fields: ");
                    ob_put(err, ls, len);
                    ob_putc(err, '\n');
                }
                continue;
            }
            const char *fe = (const char *)memchr(fs, '\t', (size_t)(le - fs));
            if (!fe) fe = le;
            int gi = gq_find_gt_index(sv(fs, (size_t)(fe - fs)));
            if (gi < 0) continue;
            if (gq_any(ls, le, gi, q, qa, qb, strict)) { ob_put(out, ls, len); ob_putc(out, '\n'); }
        }
    }
    free(hdr.p);
    if (!found && !quiet) ob_puts(err, "Error: No #CHROM line found in VCF.\n");
}
/* parseArguments :379-428 + main :624-661 */
static int gq_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_genotype_query", gq_help, out)) return 0;
    const char *query = NULL, *input = NULL;
    int strict = 0, quiet = 0, ok = 1, early = -1;
    static struct option lo[] = {{"genotype-query", required_argument, NULL, 'g'},
                                 {"input", required_argument, NULL, 'i'},
                                 {"strict", no_argument, NULL, 's'},
                                 {"quiet", no_argument, NULL, 'q'},
                                 {"help", no_argument, NULL, 'h'},
                                 {"version", no_argument, NULL, 'v'},
                                 {NULL, 0, NULL, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    int opt;
    while ((opt = getopt_long(argc, argv, "g:i:qhv", lo, NULL)) != -1) {
        if (opt == 'g') query = optarg;
        else if (opt == 'i') input = optarg;
        else if (opt == 's') strict = 1;
        else if (opt == 'q') quiet = 1;
        else if (opt == 'h') { gq_help(out); early = 0; break; }
        else if (opt == 'v') { ob_puts(out, "VCFX_genotype_query version 1.0\n"); early = 0; break; }
        else { ok = 0; break; }
    }
    errcap_end(&ec, err);
    if (early >= 0) return early;
    if (ok && optind < argc && (!input || !*input)) input = argv[optind];
    if (!ok || !query || !*query) {
        ob_printf(err, "Usage: %s -g \"0/1\" [--strict] [-i FILE] [-q]\n", argv[0]);
        ob_puts(err, "Use --help for usage.\n");
        return 1;
    }
    sv_t q = sv(query, strlen(query));
    int qa = -1, qb = -1;
    if (!strict) {
        gq_parse_diploid(q, &qa, &qb);
        if (qa > qb) { int t = qa; qa = qb; qb = t; }
    }
    if (input && *input) {
        char *d; size_t n;
        if (read_file(input, &d, &n) < 0) {
            ob_printf(err, "Error: Cannot open file: %s\n", input);
            return 1;
        }
        gq_mmap(d, n, out, err, q, qa, qb, strict, quiet);
        free(d);
    } else {
        gq_stream(in, inn, out, err, q, strict, quiet);
    }
    return 0;
}

/* ==================================================================================== */
/* VCFX_nonref_filter (a per-sample GT reducer on the same path)     */
/* ==================================================================================== */
static void nr_help(ob_t *o) {  /* displayHelp, VCFX_nonref_filter.cpp:386-417 */
    ob_puts(o,
        "VCFX_nonref_filter: Exclude variants if all samples are homozygous reference.\n\n"
        "Usage:\n"
        "  VCFX_nonref_filter [options] [input.vcf]\n"
        "  VCFX_nonref_filter [options] < input.vcf > output.vcf\n\n"
        "Options:\n"
        "  -h, --help          Show this help message\n"
        "  -i, --input FILE    Input VCF file (uses fast memory-mapped I/O)\n\n"
        "Description:\n"
        "  Reads VCF lines. For each variant, we check each sample's genotype. If a\n"
        "  genotype is polyploid, all alleles must be '0'. If a genotype is missing\n"
        "  or partial, we consider it not guaranteed hom-ref => keep variant.\n"
        "  If we find at least one sample not hom-ref, we print the variant. Otherwise,\n"
        "  we skip it.\n\n"
        "Performance:\n"
        "  File input (-i) uses memory-mapped I/O for 100-1000x faster processing\n"
        "  compared to stdin. Features include:\n"
        "  - SIMD-optimized line scanning (AVX2/SSE2)\n"
        "  - Zero-copy string parsing with string_view\n"
        "  - 1MB output buffering\n"
        "  - Direct GT field extraction (avoids full sample parsing)\n"
        "  - Early termination on first non-homref sample\n\n"
        "Examples:\n"
        "  VCFX_nonref_filter -i input.vcf > filtered.vcf    # Fast (mmap)\n"
        "  VCFX_nonref_filter input.vcf > filtered.vcf       # Fast (mmap)\n"
        "  VCFX_nonref_filter < input.vcf > filtered.vcf     # Slower (stdin)\n\n");
}
/* allSamplesHomRefDirect's per-sample test (mmap), :286-300: "0s0" (s '/' or '|') at
 * length 3, otherwise every byte '/', '|' or '0' */
static int nr_homref_mmap(sv_t g) {
    if (g.n == 3) return g.p[0] == '0' && (g.p[1] == '/' || g.p[1] == '|') && g.p[2] == '0';
    if (!g.n) return 0;
    for (size_t i = 0; i < g.n; i++)
        if (g.p[i] != '/' && g.p[i] != '|' && g.p[i] != '0') return 0;
    return 1;
}
/* isDefinitelyHomRef (stdin), :419-449 */
static int nr_homref_stream(sv_t g) {
    if (!g.n) return 0;
    if (g.n == 3 && g.p[0] == '0' && (g.p[1] == '/' || g.p[1] == '|') && g.p[2] == '0') return 1;
    for (size_t i = 0; i < g.n; i++)
        if (g.p[i] != '/' && g.p[i] != '|' && g.p[i] != '0') return 0;
    return 1;
}
/* skipToField :224-231: the byte after the n-th tab, or NULL */
static const char *nr_skip(const char *p, const char *end, int n) {
    int k = 0;
    while (p < end && k < n) {
        if (*p == '\t') k++;
        p++;
    }
    return k == n ? p : NULL;
}
/* allSamplesHomRefDirect :248-312 (1 = every sample hom-ref: the line is dropped) */
static int nr_all_homref_mmap(const char *ls, const char *le, int gi) {
    if (!nr_skip(ls, le, 8)) return 0;
    const char *p = nr_skip(ls, le, 9);
    if (!p) return 0;
    while (p < le) {
        const char *se = (const char *)memchr(p, '\t', (size_t)(le - p));
        if (!se) se = le;
        sv_t smp = sv(p, (size_t)(se - p));
        if (!smp.n) return 0;
        sv_t g;
        if (gi == 0) {
            const char *c = (const char *)memchr(smp.p, ':', smp.n);
            g = c ? sv(smp.p, (size_t)(c - smp.p)) : smp;
        } else {
            g = gq_nth(smp, gi);  /* extractNthField :179-197 (empty when absent) */
        }
        if (!nr_homref_mmap(g)) return 0;
        p = se;
        if (p < le && *p == '\t') p++;
    }
    return 1;
}
/* filterNonRefMmap :458-551 */
static void nr_mmap(const char *d, size_t n, ob_t *out, ob_t *err) {
    if (n == 0) return;
    const char *p = d, *end = d + n;
    int found = 0;
    while (p < end) {
        const char *le = (const char *)memchr(p, '\n', (size_t)(end - p));
        if (!le) le = end;
        const char *ae = le;
        if (ae > p && ae[-1] == '\r') ae--;
        size_t len = (size_t)(ae - p);
        const char *next = le + 1;
        if (len == 0) { ob_putc(out, '\n'); p = next; continue; }
        if (p[0] == '#') {
            ob_put(out, p, len);
            ob_putc(out, '\n');
            if (starts_chrom(p, len)) found = 1;
            p = next;
            continue;
        }
        if (!found) {
            ob_puts(err, "Warning: VCF data line encountered before #CHROM. Passing line.\n");
            ob_put(out, p, len);
            ob_putc(out, '\n');
            p = next;
            continue;
        }
        const char *fs = nr_skip(p, ae, 8);
        int keep = 1;
        if (fs) {
            const char *fe = (const char *)memchr(fs, '\t', (size_t)(ae - fs));
            if (!fe) fe = ae;
            int gi = gq_find_gt_index(sv(fs, (size_t)(fe - fs)));  /* findGTIndex :317-335 */
            if (gi >= 0) keep = !nr_all_homref_mmap(p, ae, gi);
        }
        if (keep) { ob_put(out, p, len); ob_putc(out, '\n'); }
        p = next;
    }
}
/* std::getline(ss, tok, ':') over s: the k-th token (0-based), *ntok = tokens */
static sv_t nr_getline_tok(sv_t s, int k, int *ntok) {
    int t = 0;
    sv_t r = {NULL, 0};
    const char *p = s.p, *e = s.p + s.n;
    while (p < e) {  /* getline yields no token for an empty remainder */
        const char *c = (const char *)memchr(p, ':', (size_t)(e - p));
        const char *te = c ? c : e;
        if (t == k) r = sv(p, (size_t)(te - p));
        t++;
        p = c ? c + 1 : e;
    }
    *ntok = t;
    return r;
}
/* filterNonRef (stdin) :553-636 */
static void nr_stream(const char *d, size_t n, ob_t *out, ob_t *err) {
    int found = 0;
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        size_t len = (size_t)(le - ls);
        if (len == 0) { ob_putc(out, '\n'); continue; }
        if (ls[0] == '#') {
            ob_put(out, ls, len);
            ob_putc(out, '\n');
            if (starts_chrom(ls, len)) found = 1;
            continue;
        }
        if (!found) {
            ob_puts(err, "Warning: VCF data line encountered before #CHROM. Passing line.\n");
            ob_put(out, ls, len);
            ob_putc(out, '\n');
            continue;
        }
        /* vcfx::split_tabs: a trailing tab yields an empty last field */
        size_t nf = 1;
        for (const char *q = ls; q < le; q++) nf += *q == '\t';
        int keep = 1;
        if (nf >= 10) {
            const char *fs = nr_skip(ls, le, 8);
            const char *fe = (const char *)memchr(fs, '\t', (size_t)(le - fs));
            sv_t fmt = sv(fs, (size_t)(fe - fs));
            int gi = -1, nt = 0;
            for (int k = 0;; k++) {
                sv_t f = nr_getline_tok(fmt, k, &nt);
                if (k >= nt) break;
                if (f.n == 2 && f.p[0] == 'G' && f.p[1] == 'T') { gi = k; break; }
            }
            if (gi >= 0) {
                int all = 1;
                const char *p = fe + 1;
                for (;;) {
                    const char *se = (const char *)memchr(p, '\t', (size_t)(le - p));
                    if (!se) se = le;
                    int ntok;
                    sv_t g = nr_getline_tok(sv(p, (size_t)(se - p)), gi, &ntok);
                    if (gi >= ntok || !nr_homref_stream(g)) { all = 0; break; }
                    if (se == le) break;
                    p = se + 1;
                }
                keep = !all;
            }
        }
        if (keep) { ob_put(out, ls, len); ob_putc(out, '\n'); }
    }
}
/* run :340-384 + main :646-652 */
static int nr_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_nonref_filter", nr_help, out)) return 0;
    const char *input = NULL;
    int help = 0;
    static struct option lo[] = {{"help", no_argument, NULL, 'h'},
                                 {"input", required_argument, NULL, 'i'},
                                 {NULL, 0, NULL, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    int opt;
    while ((opt = getopt_long(argc, argv, "hi:", lo, NULL)) != -1) {
        if (opt == 'i') input = optarg;
        else help = 1;
    }
    errcap_end(&ec, err);
    if ((!input || !*input) && optind < argc) input = argv[optind];
    if (help) {
        nr_help(out);
        return 0;
    }
    if (input && *input && strcmp(input, "-") != 0) {
        char *d; size_t n;
        if (read_file(input, &d, &n) < 0) {
            ob_printf(err, "Error: Cannot open file: %s\n", input);
            return 0;
        }
        nr_mmap(d, n, out, err);
        free(d);
    } else {
        nr_stream(in, inn, out, err);
    }
    return 0;
}

/* ==================================================================================== */
/* VCFX_record_filter                                                                   */
/* ==================================================================================== */
enum { OP_GT, OP_GE, OP_LT, OP_LE, OP_EQ, OP_NE };
enum { T_POS, T_QUAL, T_FILTER, T_INFO };
typedef struct {
    char *name; size_t name_n;
    int op, numeric, target;
    double num;
    char *str; size_t str_n;
} rf_crit;

/* trimView, VCFX_record_filter.cpp:65-71 */
static sv_t rf_trim(sv_t s) {
    while (s.n && (s.p[0] == ' ' || s.p[0] == '\t')) { s.p++; s.n--; }
    while (s.n && (s.p[s.n - 1] == ' ' || s.p[s.n - 1] == '\t')) s.n--;
    return s;
}
static size_t sv_find(sv_t h, const char *needle) {
    size_t k = strlen(needle);
    if (k > h.n) return (size_t)-1;
    for (size_t i = 0; i + k <= h.n; i++)
        if (memcmp(h.p + i, needle, k) == 0) return i;
    return (size_t)-1;
}
/* strtod over a view that must be consumed whole (parseDouble, :273-299) */
static int rf_parse_double(sv_t s, double *out) {
    if (s.n == 0) return 0;
    char stackb[64];
    char *b = s.n < sizeof stackb ? stackb : (char *)malloc(s.n + 1);
    memcpy(b, s.p, s.n);
    b[s.n] = 0;
    char *e;
    *out = strtod(b, &e);
    int ok = e == b + s.n;
    if (b != stackb) free(b);
    return ok;
}
/* parseSingleCriterion, VCFX_record_filter.cpp:89-171 */
static int rf_parse_one(sv_t tok, rf_crit *c, ob_t *err) {
    static const char *ops[] = {">=", "<=", "==", "!=", ">", "<"};
    static const int opv[] = {OP_GE, OP_LE, OP_EQ, OP_NE, OP_GT, OP_LT};
    size_t pos = (size_t)-1, ol = 0;
    int op = 0;
    for (int i = 0; i < 6; i++) {
        size_t p = sv_find(tok, ops[i]);
        if (p != (size_t)-1) { pos = p; ol = strlen(ops[i]); op = opv[i]; break; }
    }
    if (pos == (size_t)-1) {
        ob_puts(err, "Error: no operator found in '"); ob_put(err, tok.p, tok.n); ob_puts(err, "'.\n");
        return 0;
    }
    sv_t name = rf_trim(sv(tok.p, pos));
    sv_t val = rf_trim(sv(tok.p + pos + ol, tok.n - pos - ol));
    if (name.n == 0) { ob_puts(err, "Error: empty field name in '"); ob_put(err, tok.p, tok.n); ob_puts(err, "'.\n"); return 0; }
    if (val.n == 0) { ob_puts(err, "Error: no value in '"); ob_put(err, tok.p, tok.n); ob_puts(err, "'.\n"); return 0; }
    c->name = (char *)malloc(name.n + 1); memcpy(c->name, name.p, name.n); c->name[name.n] = 0; c->name_n = name.n;
    c->op = op;
    if (sv_eqs(name, "POS")) c->target = T_POS;
    else if (sv_eqs(name, "QUAL")) c->target = T_QUAL;
    else if (sv_eqs(name, "FILTER")) c->target = T_FILTER;
    else c->target = T_INFO;
    double d;
    c->numeric = rf_parse_double(val, &d);
    c->str = (char *)malloc(val.n + 1);
    c->str_n = 0;
    if (c->numeric) { c->num = d; }
    else { memcpy(c->str, val.p, val.n); c->str[val.n] = 0; c->str_n = val.n; c->num = 0.0; }
    return 1;
}
/* VCFXRecordFilter::parseCriteria, VCFX_record_filter.cpp:176-202 */
static int rf_parse_criteria(const char *s, rf_crit **out, int *nout, ob_t *err) {
    sv_t all = sv(s, strlen(s));
    size_t start = 0;
    int n = 0, cap = 4;
    rf_crit *v = (rf_crit *)calloc((size_t)cap, sizeof *v);
    while (start < all.n) {
        const char *semi = (const char *)memchr(all.p + start, ';', all.n - start);
        size_t end = semi ? (size_t)(semi - all.p) : all.n;
        sv_t tok = rf_trim(sv(all.p + start, end - start));
        if (tok.n) {
            if (n == cap) { cap *= 2; v = (rf_crit *)realloc(v, (size_t)cap * sizeof *v); }
            memset(&v[n], 0, sizeof v[n]);
            if (!rf_parse_one(tok, &v[n], err)) { *out = v; *nout = n; return 0; }
            n++;
        }
        start = end + 1;
    }
    *out = v;
    *nout = n;
    if (n == 0) { ob_printf(err, "Error: no valid criteria in '%s'.\n", s); return 0; }
    return 1;
}
/* extractField, VCFX_record_filter.cpp:207-229 */
static sv_t rf_field(sv_t line, int idx) {
    const char *p = line.p, *end = line.p + line.n;
    int cur = 0;
    while (cur < idx && p < end) { if (*p == '\t') cur++; p++; }
    if (cur < idx) return sv(NULL, 0);
    const char *fs = p;
    while (p < end && *p != '\t') p++;
    return sv(fs, (size_t)(p - fs));
}
/* extractInfoValue, VCFX_record_filter.cpp:234-267 */
static int rf_info_value(sv_t info, sv_t key, sv_t *val) {
    if (info.n == 0 || sv_eqs(info, ".")) return 0;
    size_t pos = 0;
    while (pos < info.n) {
        const char *semi = (const char *)memchr(info.p + pos, ';', info.n - pos);
        size_t te = semi ? (size_t)(semi - info.p) : info.n;
        sv_t tok = sv(info.p + pos, te - pos);
        const char *eq = (const char *)memchr(tok.p, '=', tok.n);
        if (eq) {
            sv_t k = sv(tok.p, (size_t)(eq - tok.p));
            if (k.n == key.n && memcmp(k.p, key.p, k.n) == 0) { *val = sv(eq + 1, tok.n - k.n - 1); return 1; }
        } else if (tok.n == key.n && memcmp(tok.p, key.p, key.n) == 0) { *val = tok; return 1; }
        pos = te + 1;
    }
    return 0;
}
/* compareDouble / compareString, VCFX_record_filter.cpp:310-328 */
static int rf_cmpd(double x, int op, double y) {
    switch (op) {
    case OP_GT: return x > y;
    case OP_GE: return x >= y;
    case OP_LT: return x < y;
    case OP_LE: return x <= y;
    case OP_EQ: return x == y;
    case OP_NE: return x != y;
    }
    return 0;
}
static int rf_cmps(sv_t s, int op, const char *t, size_t tn) {
    int eq = s.n == tn && (tn == 0 || memcmp(s.p, t, tn) == 0);
    if (op == OP_EQ) return eq;
    if (op == OP_NE) return !eq;
    return 0;
}
/* evaluateCriterion, VCFX_record_filter.cpp:333-378 */
static int rf_eval1(sv_t line, const rf_crit *c) {
    double x;
    switch (c->target) {
    case T_POS: {
        sv_t f = rf_field(line, 1);
        if (f.n == 0) return 0;
        if (!rf_parse_double(f, &x)) return 0;
        return rf_cmpd(x, c->op, c->num);
    }
    case T_QUAL: {
        sv_t f = rf_field(line, 5);
        if (f.n == 0 || sv_eqs(f, ".")) return rf_cmpd(0.0, c->op, c->num);
        if (!rf_parse_double(f, &x)) return 0;
        return rf_cmpd(x, c->op, c->num);
    }
    case T_FILTER: {
        sv_t f = rf_field(line, 6);
        if (c->numeric) return 0;
        return rf_cmps(f, c->op, c->str, c->str_n);
    }
    default: {
        sv_t info = rf_field(line, 7), v;
        if (!rf_info_value(info, sv(c->name, c->name_n), &v)) return 0;
        if (c->numeric) {
            if (!rf_parse_double(v, &x)) return 0;
            return rf_cmpd(x, c->op, c->num);
        }
        return rf_cmps(v, c->op, c->str, c->str_n);
    }
    }
}
/* evaluateLine, VCFX_record_filter.cpp:383-401 */
static int rf_eval(sv_t line, const rf_crit *c, int n, int and_logic) {
    if (and_logic) {
        for (int i = 0; i < n; i++) if (!rf_eval1(line, &c[i])) return 0;
        return 1;
    }
    for (int i = 0; i < n; i++) if (rf_eval1(line, &c[i])) return 1;
    return 0;
}
static void rf_help(ob_t *o) {
    ob_puts(o,
        "VCFX_record_filter: Filter VCF data lines by multiple criteria.\n\n"
        "Usage:\n"
        "  VCFX_record_filter [options] --filter \"CRITERIA\" [input.vcf]\n"
        "  VCFX_record_filter [options] --filter \"CRITERIA\" < input.vcf > output.vcf\n\n"
        "Options:\n"
        "  -f, --filter \"...\"   One or more criteria separated by semicolons, e.g.\n"
        "                        \"POS>10000; QUAL>=30; AF<0.05; FILTER==PASS\"\n"
        "                        Each criterion must use an operator among >,>=,<,<=,==,!=\n\n"
        "  -l, --logic and|or    'and' => a line must pass all criteria (default)\n"
        "                        'or'  => pass if any criterion is satisfied.\n"
        "  -i <file>             Input file (uses memory-mapped I/O for speed)\n"
        "  -q, --quiet           Suppress warnings\n"
        "  -h, --help            Show this help.\n\n"
        "Fields:\n"
        "  POS => numeric, QUAL => numeric, FILTER => string.\n"
        "  Others => assumed to be an INFO key. We try numeric parse if the criterion is numeric, else string.\n\n"
        "Performance:\n"
        "  Pass file directly for memory-mapped I/O (fastest).\n"
        "  Uses SIMD-optimized parsing on x86_64.\n"
        "  Zero-copy string_view parsing eliminates allocations.\n\n"
        "Example:\n"
        "  VCFX_record_filter --filter \"POS>=1000;FILTER==PASS;DP>10\" --logic and input.vcf\n"
        "  VCFX_record_filter -f \"QUAL>=30\" < in.vcf > out.vcf\n");
}
/* processFileMmap :406-493 (file mode) and processStdin :498-549 */
static void rf_process(const char *d, size_t n, int stdin_mode, const rf_crit *c, int nc, int and_logic,
                       ob_t *out, ob_t *err) {
    lines_t it = {d, d + n};
    const char *ls, *le;
    int found = 0;
    while (next_line(&it, &ls, &le)) {
        sv_t line = sv(ls, (size_t)(le - ls));
        if (line.n && line.p[line.n - 1] == '\r') line.n--;
        if (line.n == 0) { ob_putc(out, '\n'); continue; }
        if (line.p[0] == '#') {
            ob_put(out, line.p, line.n);
            ob_putc(out, '\n');
            if (starts_chrom(line.p, line.n)) found = 1;
            continue;
        }
        if (!found) {
            if (stdin_mode) ob_puts(err, "Warning: data line before #CHROM => skipping.\n");
            continue;
        }
        if (rf_eval(line, c, nc, and_logic)) { ob_put(out, line.p, line.n); ob_putc(out, '\n'); }
    }
}
/* run, VCFX_record_filter.cpp:584-658 + main :819-827 */
static int rf_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_record_filter", rf_help, out)) return 0;
    const char *crit = NULL, *logic = "and", *input = NULL;
    int show = 0;
    static struct option lo[] = {{"help", no_argument, 0, 'h'},
                                 {"filter", required_argument, 0, 'f'},
                                 {"logic", required_argument, 0, 'l'},
                                 {"quiet", no_argument, 0, 'q'},
                                 {0, 0, 0, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    for (;;) {
        int c = getopt_long(argc, argv, "hf:l:i:q", lo, NULL);
        if (c == -1) break;
        if (c == 'h') show = 1;
        else if (c == 'f') crit = optarg;
        else if (c == 'l') logic = optarg;
        else if (c == 'i') input = optarg;
        else if (c == 'q') {}
        else show = 1;
    }
    errcap_end(&ec, err);
    if (optind < argc && (!input || !*input)) input = argv[optind];
    if (show || argc == 1) { rf_help(out); return 0; }
    if (!crit || !*crit) {
        ob_puts(err, "Error: must provide --filter \"CRITERIA\".\n");
        rf_help(out);
        return 1;
    }
    int and_logic;
    if (strcmp(logic, "and") == 0) and_logic = 1;
    else if (strcmp(logic, "or") == 0) and_logic = 0;
    else { ob_puts(err, "Error: logic must be 'and' or 'or'.\n"); return 1; }
    rf_crit *cv = NULL;
    int nc = 0, rc = 0;
    if (!rf_parse_criteria(crit, &cv, &nc, err)) {
        ob_puts(err, "Error: failed to parse criteria.\n");
        rc = 1;
    } else if (input && *input && strcmp(input, "-") != 0) {
        char *d; size_t n;
        if (read_file(input, &d, &n) < 0) {
            ob_printf(err, "Error: cannot open file '%s'\n", input);
            rc = 1;
        } else {
            if (n) rf_process(d, n, 0, cv, nc, and_logic, out, err);
            free(d);
        }
    } else {
        rf_process(in, inn, 1, cv, nc, and_logic, out, err);
    }
    for (int i = 0; i < nc; i++) { free(cv[i].name); free(cv[i].str); }
    free(cv);
    return rc;
}

/* ==================================================================================== */
/* VCFX_ld_calculator                                                                   */
/* ==================================================================================== */
/* parseGenotypeRaw, VCFX_ld_calculator.cpp:145-174 */
int oracle_ld_parse_gt_raw(const char *s, size_t len) {
    if (len == 0) return -1;
    if (len == 1 && s[0] == '.') return -1;
    if (len == 3 && s[0] == '.' && (s[1] == '/' || s[1] == '|') && s[2] == '.') return -1;
    size_t sep = 0;
    for (size_t i = 0; i < len; i++) if (s[i] == '/' || s[i] == '|') { sep = i; break; }
    if (sep == 0 || sep >= len - 1) return -1;
    unsigned a1 = 0, a2 = 0;
    for (size_t i = 0; i < sep; i++) {
        char c = s[i];
        if (c == '.' || c < '0' || c > '9') return -1;
        a1 = a1 * 10u + (unsigned)(c - '0');
    }
    for (size_t i = sep + 1; i < len; i++) {
        char c = s[i];
        if (c == '.' || c < '0' || c > '9') return -1;
        a2 = a2 * 10u + (unsigned)(c - '0');
    }
    if ((int)a1 > 1 || (int)a2 > 1) return -1;
    return (int)(a1 + a2);
}
/* computeRsqSIMD x86 scalar body, VCFX_ld_calculator.cpp:352-393 */
static double ld_rsq(const int8_t *g1, const int8_t *g2, size_t sz) {
    int n = 0;
    long sx = 0, sy = 0, sxy = 0, sx2 = 0, sy2 = 0;
    for (size_t i = 0; i < sz; i++) {
        int8_t x = g1[i], y = g2[i];
        if (x >= 0 && y >= 0) { n++; sx += x; sy += y; sxy += x * y; sx2 += x * x; sy2 += y * y; }
    }
    if (n < 2) return 0.0;
    double mx = (double)sx / n, my = (double)sy / n;
    double cov = (double)sxy / n - mx * my;
    double vx = (double)sx2 / n - mx * mx;
    double vy = (double)sy2 / n - my * my;
    if (vx <= 0.0 || vy <= 0.0) return 0.0;
    double r = cov / (sqrt(vx) * sqrt(vy));
    return r * r;
}
typedef struct {
    char *chrom; size_t chrom_n;
    int pos;
    char *id; size_t id_n;
    int8_t *g;
    double varX;
} ld_var;
/* LDVariantOpt::computeStats, VCFX_ld_calculator.cpp:243-258 (varX is what the fast
 * path's own-variance gate reads) */
static double ld_varx(const int8_t *g, int n) {
    int vc = 0;
    long s = 0, s2 = 0;
    for (int i = 0; i < n; i++) if (g[i] >= 0) { vc++; s += g[i]; s2 += g[i] * g[i]; }
    if (vc <= 0) return 0;
    double m = (double)s / vc;
    return (double)s2 / vc - m * m;
}
double oracle_ld_rsq_fast(const int8_t *g1, const int8_t *g2, size_t n) {
    if (ld_varx(g1, (int)n) <= 0.0 || ld_varx(g2, (int)n) <= 0.0) return 0.0;
    return ld_rsq(g1, g2, n);
}
/* formatR2 / formatInt, VCFX_ld_calculator.cpp:200-225 */
static void ld_fmt_r2(ob_t *o, double r2) {
    if (r2 <= 0.0) { ob_put(o, "0.0000", 6); return; }
    if (r2 >= 1.0) { ob_put(o, "1.0000", 6); return; }
    char b[6] = {'0', '.'};
    int v = (int)(r2 * 10000.0 + 0.5);
    if (v > 9999) v = 9999;
    b[5] = (char)('0' + v % 10); v /= 10;
    b[4] = (char)('0' + v % 10); v /= 10;
    b[3] = (char)('0' + v % 10); v /= 10;
    b[2] = (char)('0' + v % 10);
    ob_put(o, b, 6);
}
/* fastParseInt, VCFX_ld_calculator.cpp:188-197 (wraps like the reference's int math) */
static int ld_parse_int(const char *s, size_t n, int *r) {
    if (n == 0) return 0;
    unsigned v = 0;
    for (size_t i = 0; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        v = v * 10u + (unsigned)(s[i] - '0');
    }
    *r = (int)v;
    return 1;
}
static void ld_free(ld_var *v) { free(v->chrom); free(v->id); free(v->g); }
/* parse a data line into a variant; 0 = skip.  Shared by computeLDStreamingMmap (:555-613)
 * and computeLDMatrixMmap (:697-759); id_dot_to_pos selects streaming's '.'->chrom:pos */
static int ld_parse_line(const char *ls, size_t len, int ns, const char *rchrom, int rs, int re,
                         int id_dot_to_pos, ld_var *v, int *region_skip) {
    const char *fst[10];
    size_t fl[10];
    int fc = 0;
    size_t start = 0;
    *region_skip = 0;
    for (size_t i = 0; i <= len && fc < 10; i++) {
        if (i == len || ls[i] == '\t') { fst[fc] = ls + start; fl[fc] = i - start; fc++; start = i + 1; }
    }
    if (fc < 10) return 0;
    int pos;
    if (!ld_parse_int(fst[1], fl[1], &pos)) return 0;
    if (rchrom && *rchrom) {
        size_t rl = strlen(rchrom);
        if (fl[0] != rl || memcmp(fst[0], rchrom, rl) != 0 || pos < rs || pos > re) { *region_skip = 1; return 0; }
    }
    v->chrom = (char *)malloc(fl[0] + 1); memcpy(v->chrom, fst[0], fl[0]); v->chrom_n = fl[0];
    v->pos = pos;
    if (id_dot_to_pos && fl[2] == 1 && fst[2][0] == '.') {
        char tmp[64];
        int k = snprintf(tmp, sizeof tmp, ":%d", pos);
        v->id = (char *)malloc(fl[0] + (size_t)k + 1);
        memcpy(v->id, fst[0], fl[0]);
        memcpy(v->id + fl[0], tmp, (size_t)k);
        v->id_n = fl[0] + (size_t)k;
    } else {
        v->id = (char *)malloc(fl[2] + 1); memcpy(v->id, fst[2], fl[2]); v->id_n = fl[2];
    }
    v->g = (int8_t *)malloc((size_t)(ns > 0 ? ns : 1));
    for (int i = 0; i < ns; i++) v->g[i] = -1;
    const char *s = fst[9], *end = ls + len;
    int si = 0;
    while (s < end && si < ns) {
        const char *se = s;
        while (se < end && *se != '\t') se++;
        size_t sl = (size_t)(se - s), gl = sl;
        for (size_t i = 0; i < sl; i++) if (s[i] == ':') { gl = i; break; }
        if (gl > 0) v->g[si] = (int8_t)oracle_ld_parse_gt_raw(s, gl);
        si++;
        s = se + 1;
    }
    v->varX = ld_varx(v->g, ns);
    return 1;
}
static double ld_rsq_fast_v(const ld_var *a, const ld_var *b, int ns) {
    if (a->varX <= 0.0 || b->varX <= 0.0) return 0.0;
    return ld_rsq(a->g, b->g, (size_t)ns);
}
static void ld_emit_pair(ob_t *o, const ld_var *p, const ld_var *v, double r2) {
    ob_put(o, p->chrom, p->chrom_n); ob_putc(o, '\t');
    ob_printf(o, "%d", p->pos); ob_putc(o, '\t');
    ob_put(o, p->id, p->id_n); ob_putc(o, '\t');
    ob_put(o, v->chrom, v->chrom_n); ob_putc(o, '\t');
    ob_printf(o, "%d", v->pos); ob_putc(o, '\t');
    ob_put(o, v->id, v->id_n); ob_putc(o, '\t');
    ld_fmt_r2(o, r2);
    ob_putc(o, '\n');
}
static int ld_count_samples(const char *ls, size_t len) {
    int t = 0;
    for (size_t i = 0; i < len; i++) if (ls[i] == '\t') t++;
    return t >= 9 ? t - 8 : 0;
}
/* computeLDStreamingMmap :511-648 (mmap=1) and computeLDStreaming :864-987 (mmap=0) */
static void ld_stream(const char *d, size_t n, int mmap_mode, const char *rchrom, int rs, int re, size_t W,
                      double thr, int maxd, int quiet, ob_t *out, ob_t *err) {
    ob_puts(out, "#VAR1_CHROM\tVAR1_POS\tVAR1_ID\tVAR2_CHROM\tVAR2_POS\tVAR2_ID\tR2\n");
    int found = 0, ns = 0;
    /* window = deque of the last W variants (W may be huge: std::stoul("-1")) */
    size_t cap = 64, head = 0, cnt = 0;
    ld_var *win = (ld_var *)calloc(cap, sizeof *win);
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        size_t len = (size_t)(le - ls);
        if (len == 0) continue;
        if (ls[0] == '#') {
            if (!found && starts_chrom(ls, len)) { found = 1; ns = ld_count_samples(ls, len); }
            continue;
        }
        if (!found) {
            if (mmap_mode) { if (!quiet) ob_puts(err, "Error: data line before #CHROM\n"); }
            else ob_puts(err, "Error: encountered data line before #CHROM.\n");
            break;
        }
        ld_var v;
        int rsk;
        if (!ld_parse_line(ls, len, ns, rchrom, rs, re, 1, &v, &rsk)) continue;
        for (size_t k = 0; k < cnt; k++) {
            const ld_var *p = &win[head + k];
            if (mmap_mode && maxd > 0 && p->chrom_n == v.chrom_n && memcmp(p->chrom, v.chrom, v.chrom_n) == 0) {
                int dd = v.pos - p->pos;
                if (dd < 0) dd = -dd;
                if (dd > maxd) continue;
            }
            double r2 = ld_rsq_fast_v(p, &v, ns);
            if (r2 >= thr) ld_emit_pair(out, p, &v, r2);
        }
        if (head + cnt == cap) {
            if (head > 0) { memmove(win, win + head, cnt * sizeof *win); head = 0; }
            else { cap *= 2; win = (ld_var *)realloc(win, cap * sizeof *win); }
        }
        win[head + cnt] = v;
        cnt++;
        if (cnt > W) { ld_free(&win[head]); head++; cnt--; }
    }
    for (size_t k = 0; k < cnt; k++) ld_free(&win[head + k]);
    free(win);
}
/* computeLDMatrixMmap :653-859 */
static void ld_matrix_mmap(const char *d, size_t n, const char *rchrom, int rs, int re, int quiet,
                           ob_t *out, ob_t *err) {
    int found = 0, ns = 0;
    size_t M = 0, cap = 64;
    ld_var *vs = (ld_var *)calloc(cap, sizeof *vs);
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        size_t len = (size_t)(le - ls);
        if (len == 0) continue;
        if (ls[0] == '#') {
            ob_put(out, ls, len); ob_putc(out, '\n');
            if (!found && starts_chrom(ls, len)) { found = 1; ns = ld_count_samples(ls, len); }
            continue;
        }
        if (!found) { if (!quiet) ob_puts(err, "Error: data line before #CHROM\n"); break; }
        ld_var v;
        int rsk;
        if (ld_parse_line(ls, len, ns, rchrom, rs, re, 0, &v, &rsk)) {
            if (M == cap) { cap *= 2; vs = (ld_var *)realloc(vs, cap * sizeof *vs); }
            vs[M++] = v;
        }
        ob_put(out, ls, len); ob_putc(out, '\n');
    }
    if (M < 2) {
        ob_puts(out, "#LD_MATRIX_START\nNo or only one variant in the region => no pairwise LD.\n#LD_MATRIX_END\n");
    } else {
        ob_puts(out, "#LD_MATRIX_START\nIndex/Var");
        for (size_t j = 0; j < M; j++) {
            ob_putc(out, '\t'); ob_put(out, vs[j].chrom, vs[j].chrom_n); ob_printf(out, ":%d", vs[j].pos);
        }
        ob_putc(out, '\n');
        for (size_t i = 0; i < M; i++) {
            ob_put(out, vs[i].chrom, vs[i].chrom_n); ob_printf(out, ":%d", vs[i].pos);
            for (size_t j = 0; j < M; j++) {
                ob_putc(out, '\t');
                if (i == j) ob_put(out, "1.0000", 6);
                else ld_fmt_r2(out, ld_rsq_fast_v(&vs[i], &vs[j], ns));
            }
            ob_putc(out, '\n');
        }
        ob_puts(out, "#LD_MATRIX_END\n");
    }
    for (size_t i = 0; i < M; i++) ld_free(&vs[i]);
    free(vs);
}
/* std::stoi-like parse: leading isspace, optional sign, >=1 digit, fits int; partial ok */
static int cxx_stoi(const char *s, long *out) {
    errno = 0;
    char *e;
    long v = strtol(s, &e, 10);
    if (e == s) return 0;
    if (errno == ERANGE || v < INT_MIN || v > INT_MAX) return 0;
    *out = v;
    return 1;
}
/* parseGenotype (stdin matrix), VCFX_ld_calculator.cpp:468-482 */
static int ld_parse_gt_stoi(const char *s, size_t n) {
    if (n == 0 || (n == 1 && s[0] == '.') || (n == 3 && (memcmp(s, "./.", 3) == 0 || memcmp(s, ".|.", 3) == 0)))
        return -1;
    char *g = (char *)malloc(n + 1);
    for (size_t i = 0; i < n; i++) g[i] = s[i] == '|' ? '/' : s[i];
    g[n] = 0;
    char *sl = (char *)memchr(g, '/', n);
    int r = -1;
    if (sl) {
        *sl = 0;
        const char *a1 = g, *a2 = sl + 1;
        long i1, i2;
        if (*a1 && *a2 && strcmp(a1, ".") != 0 && strcmp(a2, ".") != 0 && cxx_stoi(a1, &i1) && cxx_stoi(a2, &i2)) {
            if (!(i1 < 0 || i2 < 0 || i1 > 1 || i2 > 1)) r = i1 == i2 ? (i1 == 0 ? 0 : 2) : 1;
        }
    }
    free(g);
    return r;
}
/* computeRsq (stdin matrix), VCFX_ld_calculator.cpp:487-506 */
static double ld_rsq_int(const int *g1, const int *g2, int sz) {
    int n = 0;
    long sx = 0, sy = 0, sxy = 0, sx2 = 0, sy2 = 0;
    for (int i = 0; i < sz; i++) {
        int x = g1[i], y = g2[i];
        if (x < 0 || y < 0) continue;
        n++; sx += x; sy += y; sxy += x * y; sx2 += x * x; sy2 += y * y;
    }
    if (n < 2) return 0.0;
    double mx = (double)sx / n, my = (double)sy / n;
    double cov = ((double)sxy / n) - (mx * my);
    double vx = ((double)sx2 / n) - (mx * mx);
    double vy = ((double)sy2 / n) - (my * my);
    if (vx <= 0.0 || vy <= 0.0) return 0.0;
    double r = cov / (sqrt(vx) * sqrt(vy));
    return r * r;
}
/* computeLD (stdin matrix), VCFX_ld_calculator.cpp:992-1079 */
static void ld_matrix_stdin(const char *d, size_t n, const char *rchrom, int rs, int re, ob_t *out, ob_t *err) {
    int found = 0, ns = 0;
    size_t M = 0, cap = 64;
    typedef struct { char *chrom; size_t cn; int pos; int *g; } var_t;
    var_t *vs = (var_t *)calloc(cap, sizeof *vs);
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        size_t len = (size_t)(le - ls);
        if (len == 0) { ob_putc(out, '\n'); continue; }
        if (ls[0] == '#') {
            ob_put(out, ls, len); ob_putc(out, '\n');
            if (!found && starts_chrom(ls, len)) {
                found = 1;
                int t = 0;
                for (size_t i = 0; i < len; i++) if (ls[i] == '\t') t++;
                ns = t + 1 > 9 ? t + 1 - 9 : 0;  /* split_tabs keeps a trailing empty field */
            }
            continue;
        }
        if (!found) { ob_puts(err, "Error: encountered data line before #CHROM.\n"); break; }
        /* split_tabs (vcfx_io.h:59-76): every tab separates, trailing empty field kept */
        size_t nf = 1;
        for (size_t i = 0; i < len; i++) if (ls[i] == '\t') nf++;
        if (nf < 10) { ob_put(out, ls, len); ob_putc(out, '\n'); continue; }
        const char **fp = (const char **)malloc(nf * sizeof *fp);
        size_t *fl = (size_t *)malloc(nf * sizeof *fl);
        size_t k = 0, st = 0;
        for (size_t i = 0; i <= len; i++)
            if (i == len || ls[i] == '\t') { fp[k] = ls + st; fl[k] = i - st; k++; st = i + 1; }
        char *f1 = (char *)malloc(fl[1] + 1); memcpy(f1, fp[1], fl[1]); f1[fl[1]] = 0;
        long pv;
        int okp = cxx_stoi(f1, &pv);
        free(f1);
        if (!okp) { ob_put(out, ls, len); ob_putc(out, '\n'); free(fp); free(fl); continue; }
        if (rchrom && *rchrom) {
            size_t rl = strlen(rchrom);
            if (fl[0] != rl || memcmp(fp[0], rchrom, rl) != 0 || pv < rs || pv > re) {
                ob_put(out, ls, len); ob_putc(out, '\n'); free(fp); free(fl); continue;
            }
        }
        if (M == cap) { cap *= 2; vs = (var_t *)realloc(vs, cap * sizeof *vs); }
        var_t *v = &vs[M++];
        v->chrom = (char *)malloc(fl[0] + 1); memcpy(v->chrom, fp[0], fl[0]); v->cn = fl[0];
        v->pos = (int)pv;
        v->g = (int *)malloc(sizeof(int) * (size_t)(ns > 0 ? ns : 1));
        for (int s = 0; s < ns; s++) v->g[s] = -1;
        for (int s = 0; s < ns; s++) {
            if ((size_t)(9 + s) >= nf) break;
            v->g[s] = ld_parse_gt_stoi(fp[9 + s], fl[9 + s]);
        }
        free(fp); free(fl);
        ob_put(out, ls, len); ob_putc(out, '\n');
    }
    if (M < 2) {
        ob_puts(out, "#LD_MATRIX_START\nNo or only one variant in the region => no pairwise LD.\n#LD_MATRIX_END\n");
    } else {
        ob_puts(out, "#LD_MATRIX_START\nIndex/Var");
        for (size_t j = 0; j < M; j++) { ob_putc(out, '\t'); ob_put(out, vs[j].chrom, vs[j].cn); ob_printf(out, ":%d", vs[j].pos); }
        ob_putc(out, '\n');
        char nb[64];
        for (size_t i = 0; i < M; i++) {
            ob_put(out, vs[i].chrom, vs[i].cn); ob_printf(out, ":%d", vs[i].pos);
            for (size_t j = 0; j < M; j++) {
                if (i == j) ob_puts(out, "\t1.0000");
                else {
                    size_t kk = oracle_fmt_fixed4(ld_rsq_int(vs[i].g, vs[j].g, ns), nb);
                    ob_putc(out, '\t'); ob_put(out, nb, kk);
                }
            }
            ob_putc(out, '\n');
        }
        ob_puts(out, "#LD_MATRIX_END\n");
    }
    for (size_t i = 0; i < M; i++) { free(vs[i].chrom); free(vs[i].g); }
    free(vs);
}
static void ld_help(ob_t *o) {
    ob_puts(o,
        "VCFX_ld_calculator: Calculate pairwise LD (r^2) for variants in a VCF region.\n"
        "Version 2.0 - Extreme-performance with mmap, SIMD, and multi-threading.\n\n"
        "Usage:\n"
        "  VCFX_ld_calculator [options] < input.vcf\n"
        "  VCFX_ld_calculator [options] -i input.vcf\n\n"
        "Options:\n"
        "  -i, --input FILE          Input VCF file (uses memory-mapping for best performance)\n"
        "  -r, --region <chr:s-e>    Only compute LD for variants in [start, end] on 'chr'\n"
        "  -w, --window <N>          Window size in variants (default: 1000)\n"
        "  -d, --max-distance <BP>   Max base-pair distance between pairs (0=unlimited)\n"
        "  -t, --threshold <R2>      Only output pairs with r\xc2\xb2 >= threshold (default: 0.0)\n"
        "  -n, --threads <N>         Number of threads (default: auto)\n"
        "  -m, --matrix              Use matrix mode (MxM output) instead of streaming\n"
        "                            WARNING: O(M\xc2\xb2) time - avoid for >10K variants\n"
        "  -q, --quiet               Suppress informational messages\n"
        "  -h, --help                Show this help message\n"
        "  -v, --version             Show program version\n\n"
        "Modes:\n"
        "  Default (streaming): Outputs LD pairs incrementally using a sliding window.\n"
        "                       Memory: O(window * samples) - constant for any file size.\n"
        "                       Time: O(M * window) - linear in variant count.\n"
        "  Matrix mode:         Produces an MxM matrix of all pairwise r\xc2\xb2 values.\n"
        "                       Memory: O(M * samples) where M is number of variants.\n"
        "                       Time: O(M\xc2\xb2) - avoid for >10K variants!\n\n"
        "Performance:\n"
        "  - Memory-mapped I/O: Use -i flag for extreme speed\n"
        "  - SIMD-accelerated r\xc2\xb2 computation (NEON/AVX2/SSE2)\n"
        "  - Multi-threaded matrix computation\n"
        "  - Distance-based pruning with --max-distance\n\n"
        "Example:\n"
        "  # Fast streaming mode with file input\n"
        "  VCFX_ld_calculator -i input.vcf -w 500 -t 0.2 > ld_pairs.txt\n\n"
        "  # Streaming with distance limit (biology: LD decays with distance)\n"
        "  VCFX_ld_calculator -i input.vcf --max-distance 500000 > ld_pairs.txt\n\n"
        "  # Matrix mode (small regions only)\n"
        "  VCFX_ld_calculator -i input.vcf -m -r chr1:10000-20000 > ld_matrix.txt\n");
}
/* parseRegion, VCFX_ld_calculator.cpp:448-463 */
static int ld_parse_region(const char *r, char **chrom, int *rs, int *re) {
    const char *c = strchr(r, ':');
    if (!c) return 0;
    const char *dash = strchr(c + 1, '-');
    if (!dash) return 0;
    char *a = strndup(c + 1, (size_t)(dash - c - 1));
    long s, e;
    int ok = cxx_stoi(a, &s) && cxx_stoi(dash + 1, &e);
    free(a);
    if (!ok || s > e) return 0;
    *chrom = strndup(r, (size_t)(c - r));
    *rs = (int)s;
    *re = (int)e;
    return 1;
}
/* run, VCFX_ld_calculator.cpp:1084-1209 + main :1219-1225 */
static int ld_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_ld_calculator", ld_help, out)) return 0;
    static struct option lo[] = {{"help", no_argument, 0, 'h'},      {"version", no_argument, 0, 'v'},
                                 {"input", required_argument, 0, 'i'}, {"region", required_argument, 0, 'r'},
                                 {"streaming", no_argument, 0, 's'}, {"matrix", no_argument, 0, 'm'},
                                 {"window", required_argument, 0, 'w'}, {"threshold", required_argument, 0, 't'},
                                 {"threads", required_argument, 0, 'n'}, {"max-distance", required_argument, 0, 'd'},
                                 {"quiet", no_argument, 0, 'q'},      {0, 0, 0, 0}};
    int show = 0, matrix = 0, maxd = 0, quiet = 0, rc = -1;
    size_t W = 1000;
    double thr = 0.0;
    const char *region = NULL, *input = NULL;
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    for (;;) {
        int c = getopt_long(argc, argv, "hvi:r:smw:t:n:d:q", lo, NULL);
        if (c == -1) break;
        if (c == 'h') show = 1;
        else if (c == 'v') { ob_puts(out, "VCFX_ld_calculator v2.0\n"); rc = 0; break; }
        else if (c == 'i') input = optarg;
        else if (c == 'r') region = optarg;
        else if (c == 's') matrix = 0;
        else if (c == 'm') matrix = 1;
        else if (c == 'w') {
            /* std::stoul: strtoul semantics, throws if nothing parsed or ERANGE */
            errno = 0;
            char *e;
            unsigned long v = strtoul(optarg, &e, 10);
            if (e == optarg || errno == ERANGE) { ob_printf(err, "Error: Invalid window size '%s'\n", optarg); rc = 1; break; }
            W = v == 0 ? 1 : v;
        } else if (c == 't') {
            errno = 0;
            char *e;
            double v = strtod(optarg, &e);
            if (e == optarg || errno == ERANGE) { ob_printf(err, "Error: Invalid threshold '%s'\n", optarg); rc = 1; break; }
            if (v < 0.0) v = 0.0;
            if (v > 1.0) v = 1.0;
            thr = v;
        } else if (c == 'n') {
            long v;
            if (!cxx_stoi(optarg, &v)) { ob_printf(err, "Error: Invalid thread count '%s'\n", optarg); rc = 1; break; }
        } else if (c == 'd') {
            long v;
            if (!cxx_stoi(optarg, &v)) { ob_printf(err, "Error: Invalid max-distance '%s'\n", optarg); rc = 1; break; }
            maxd = v < 0 ? 0 : (int)v;
        } else if (c == 'q') quiet = 1;
        else show = 1;
    }
    errcap_end(&ec, err);
    if (rc >= 0) return rc;
    if (optind < argc && (!input || !*input)) input = argv[optind];
    if (show) { ld_help(out); return 0; }
    char *rchrom = NULL;
    int rs = 0, re = 0;
    if (region && *region) {
        if (!ld_parse_region(region, &rchrom, &rs, &re)) {
            ob_printf(err, "Error parsing region '%s'. Use e.g. chr1:10000-20000\n", region);
            return 1;
        }
    }
    if (input && *input) {
        char *d = NULL; size_t n = 0;
        if (read_file(input, &d, &n) < 0 || n == 0) {
            free(d);
            ob_printf(err, "Error: cannot open file '%s'\n", input);
            free(rchrom);
            return 1;
        }
        if (matrix) ld_matrix_mmap(d, n, rchrom, rs, re, quiet, out, err);
        else ld_stream(d, n, 1, rchrom, rs, re, W, thr, maxd, quiet, out, err);
        free(d);
    } else {
        if (matrix) ld_matrix_stdin(in, inn, rchrom, rs, re, out, err);
        else ld_stream(in, inn, 0, rchrom, rs, re, W, thr, 0, quiet, out, err);
    }
    free(rchrom);
    return 0;
}

/* ==================================================================================== */
/* ==================================================================================== */
/* VCFX_hwe_tester                                                 */
/* ==================================================================================== */
/* chi2_pvalue_1df, VCFX_hwe_tester.cpp:278-287 (Abramowitz-Stegun erfc, libm exp/sqrt) */
double oracle_hwe_pvalue(int homRef, int het, int homAlt) {
    /* calculateHWE_chisq :290-315 */
    int N = homRef + het + homAlt;
    if (N < 1) return 1.0;
    double p = (2.0 * homRef + het) / (2.0 * N);
    double q = 1.0 - p;
    if (p <= 0.0 || p >= 1.0) return 1.0;
    double eh = N * p * p, ee = N * 2.0 * p * q, ea = N * q * q;
    double obs[3] = {homRef, het, homAlt}, ex[3] = {eh, ee, ea}, chi2 = 0.0;
    for (int k = 0; k < 3; k++) {
        double t = 0.0;
        if (ex[k] > 0.0) {
            double diff = fabs(obs[k] - ex[k]) - 0.5;
            if (diff < 0.0) diff = 0.0;
            t = (diff * diff) / ex[k];
        }
        chi2 = k == 0 ? t : chi2 + t;
    }
    if (chi2 <= 0.0) return 1.0;
    if (chi2 > 700.0) return 0.0;
    double x = sqrt(chi2 * 0.5);
    double t = 1.0 / (1.0 + 0.3275911 * x);
    double y = t * (0.254829592 + t * (-0.284496736 + t * (1.421413741 + t * (-1.453152027 + t * 1.061405429))));
    return y * exp(-x * x);
}
/* OutputBuffer::appendDouble, VCFX_hwe_tester.cpp:236-268: truncated 6-digit fraction */
size_t oracle_hwe_fmt_mmap(double val, char *buf) {
    size_t k = 0;
    if (val < 0) { buf[k++] = '-'; val = -val; }
    long long ip = (long long)val;
    double frac = val - ip;
    char t[24]; int i = 0;
    if (ip == 0) t[i++] = '0';
    else while (ip > 0) { t[i++] = (char)('0' + ip % 10); ip /= 10; }
    while (i > 0) buf[k++] = t[--i];
    buf[k++] = '.';
    for (int d = 0; d < 6; d++) {
        frac *= 10.0;
        int digit = (int)frac;
        buf[k++] = (char)('0' + digit);
        frac -= digit;
    }
    return k;
}
/* parseGenotypeForHWE :339-378: 0 homRef, 1 het, 2 homAlt, -1 otherwise */
static int hwe_parse(const char *p, const char *end) {
    if (p >= end) return -1;
    const char *c = (const char *)memchr(p, ':', (size_t)(end - p));
    if (c) end = c;
    while (p < end && (*p == ' ' || *p == '\r')) p++;
    if (p >= end || *p == '.') return -1;
    if (*p < '0' || *p > '9') return -1;
    int a1 = 0;
    while (p < end && *p >= '0' && *p <= '9') { a1 = a1 * 10 + (*p - '0'); p++; }
    if (p >= end || (*p != '/' && *p != '|')) return -1;
    p++;
    if (p >= end || *p == '.') return -1;
    if (*p < '0' || *p > '9') return -1;
    int a2 = 0;
    while (p < end && *p >= '0' && *p <= '9') { a2 = a2 * 10 + (*p - '0'); p++; }
    if (a1 > 1 || a2 > 1) return -1;
    if (a1 == 0 && a2 == 0) return 0;
    if (a1 == 1 && a2 == 1) return 2;
    return 1;
}
/* skipToField / getField :321-336 (findTabSIMD = first '\t' in [p, end)) */
static const char *hwe_skip(const char *p, const char *le, int idx) {
    for (int i = 0; i < idx && p < le; i++) {
        const char *t = (const char *)memchr(p, '\t', (size_t)(le - p));
        if (!t) return NULL;
        p = t + 1;
    }
    return p < le ? p : NULL;
}
static sv_t hwe_field(const char *ls, const char *le, int idx) {
    const char *p = hwe_skip(ls, le, idx);
    if (!p) return sv(NULL, 0);
    const char *t = (const char *)memchr(p, '\t', (size_t)(le - p));
    return sv(p, (size_t)((t ? t : le) - p));
}
static void hwe_count(const char *sp, const char *le, int *c) {
    c[0] = c[1] = c[2] = 0;
    while (sp < le) {
        const char *nt = (const char *)memchr(sp, '\t', (size_t)(le - sp));
        if (!nt) nt = le;
        int g = hwe_parse(sp, nt);
        if (g >= 0) c[g]++;
        sp = nt + 1;
    }
}
/* performHWE_Mmap :455-559 */
static void hwe_mmap(const char *d, size_t n, ob_t *out) {
    if (n == 0) return;
    ob_puts(out, "CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n");
    const char *p = d, *end = d + n;
    while (p < end) {
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        const char *le = nl ? nl : end;
        size_t len = (size_t)(le - p);
        if (len > 0 && p[len - 1] == '\r') len--;
        const char *ae = p + len;
        if (len == 0 || *p == '#') { p = le + 1; continue; }
        sv_t f[5];
        for (int k = 0; k < 5; k++) f[k] = hwe_field(p, ae, k);
        sv_t fmt = hwe_field(p, ae, 8);
        const char *ss = hwe_skip(p, ae, 9);
        if (f[0].n == 0 || f[1].n == 0 || f[4].n == 0 || memchr(f[4].p, ',', f[4].n) ||
            fmt.n < 2 || memcmp(fmt.p, "GT", 2) != 0 || !ss) { p = le + 1; continue; }
        int c[3];
        hwe_count(ss, ae, c);
        for (int k = 0; k < 5; k++) { ob_put(out, f[k].p, f[k].n); ob_putc(out, '\t'); }
        char b[40];
        ob_put(out, b, oracle_hwe_fmt_mmap(oracle_hwe_pvalue(c[0], c[1], c[2]), b));
        ob_putc(out, '\n');
        p = le + 1;
    }
}
/* performHWE_Stdin :565-608 (split_tabs: a trailing tab is an empty last field) */
static void hwe_stdin(const char *d, size_t n, ob_t *out) {
    ob_puts(out, "CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n");
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        if (le == ls) continue;
        if (le[-1] == '\r') le--;
        if (le == ls || *ls == '#') continue;
        sv_t f[10];
        size_t nf = 0;
        const char *q = ls;
        for (;;) {
            const char *t = (const char *)memchr(q, '\t', (size_t)(le - q));
            if (nf < 10) f[nf] = sv(q, (size_t)((t ? t : le) - q));
            nf++;
            if (!t) break;
            q = t + 1;
        }
        if (nf < 10 || memchr(f[4].p, ',', f[4].n) || f[8].n < 2 || memcmp(f[8].p, "GT", 2) != 0) continue;
        int c[3] = {0, 0, 0};
        hwe_count(f[9].p, le, c);
        if (f[9].p == le) c[0] = c[1] = c[2] = 0;  /* a lone empty sample field */
        for (int k = 0; k < 5; k++) { ob_put(out, f[k].p, f[k].n); ob_putc(out, '\t'); }
        ob_printf(out, "%.6f\n", oracle_hwe_pvalue(c[0], c[1], c[2]));
    }
}
static void hwe_help(ob_t *o) {  /* displayHelp :394-412 */
    ob_puts(o,
        "VCFX_hwe_tester: Perform Hardy-Weinberg Equilibrium (HWE) tests on a biallelic VCF.\n\n"
        "Usage:\n"
        "  VCFX_hwe_tester [options] [input.vcf]\n"
        "  VCFX_hwe_tester [options] < input.vcf\n\n"
        "Options:\n"
        "  -i, --input FILE   Input VCF file (uses memory-mapping for best performance)\n"
        "  -q, --quiet        Suppress informational messages\n"
        "  -h, --help         Show this help.\n\n"
        "Description:\n"
        "  Reads each variant line, ignoring multi-allelic calls. For biallelic lines,\n"
        "  collects genotypes as 0/0, 0/1, 1/1, then uses chi-square test with Yates'\n"
        "  continuity correction to produce a p-value for HWE.\n\n"
        "Performance:\n"
        "  Uses memory-mapped I/O and SIMD for ~20x speedup over stdin mode.\n\n"
        "Example:\n"
        "  VCFX_hwe_tester -i input.vcf > results.txt\n"
        "  VCFX_hwe_tester < input.vcf > results.txt\n");
}
/* main :688-694 -> VCFXHWETester::run :614-641, parseArgs :414-449 */
static int hwe_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_hwe_tester", hwe_help, out)) return 0;
    const char *input = NULL;
    int quiet = 0, help = 0;
    static struct option lo[] = {{"help", no_argument, NULL, 'h'},
                                 {"input", required_argument, NULL, 'i'},
                                 {"quiet", no_argument, NULL, 'q'},
                                 {NULL, 0, NULL, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    int opt;
    while ((opt = getopt_long(argc, argv, "hi:q", lo, NULL)) != -1) {
        if (opt == 'i') input = optarg;
        else if (opt == 'q') quiet = 1;
        else help = 1;
    }
    errcap_end(&ec, err);
    if (!input && optind < argc) input = argv[optind];
    if (help) { hwe_help(out); return 0; }
    if (input) {
        char *d; size_t n;
        if (read_file(input, &d, &n) < 0) {
            ob_printf(err, "Error: Cannot open file: %s\n", input);
            return 1;
        }
        if (!quiet) ob_printf(err, "Processing %s (%zu bytes)...\n", input, n);
        hwe_mmap(d, n, out);
        free(d);
    } else {
        hwe_stdin(in, inn, out);
    }
    return 0;
}

/* ==================================================================================== */
/* VCFX_dosage_calculator                                          */
/* ==================================================================================== */
/* parseDosageInline, VCFX_dosage_calculator.cpp:111-156: -1 = NA (absurdly long numbers
 * wrap modulo 2^32, as the reference's int accumulation does) */
static int dose_parse(const char *gt, size_t n) {
    if (n == 0) return -1;
    int dosage = 0, count = 0;
    size_t pos = 0;
    while (pos < n) {
        while (pos < n && (gt[pos] == '/' || gt[pos] == '|')) pos++;
        if (pos >= n) break;
        if (gt[pos] == '.') return -1;
        uint32_t allele = 0;
        int dig = 0;
        while (pos < n && gt[pos] >= '0' && gt[pos] <= '9') {
            allele = allele * 10u + (uint32_t)(gt[pos] - '0');
            dig = 1;
            pos++;
        }
        if (!dig) return -1;
        /* `allele > 0` on a non-negative int accumulation: the reference build (g++ -O3)
         * tests it as `!= 0` (signed overflow is undefined), so a wrapped 2^31 counts */
        if (allele != 0) dosage++;
        if (++count > 2) return -1;
    }
    return count == 2 ? dosage : -1;
}
/* findGTIndexRaw :160-178 (exact "GT" token) */
static int dose_gt_index(const char *f, size_t n) {
    int idx = 0;
    size_t start = 0;
    for (size_t pos = 0; pos <= n; pos++) {
        if (pos == n || f[pos] == ':') {
            if (pos - start == 2 && f[start] == 'G' && f[start + 1] == 'T') return idx;
            idx++;
            start = pos + 1;
        }
    }
    return -1;
}
/* one record [ls, ls + len): the row, or the warning (processFileMmap :464-576 /
 * calculateDosage :248-352); returns 1 for a row, 0 for "fewer than 10 fields" */
static int dose_line(const char *ls, size_t len, ob_t *out) {
    const char *f[10];
    size_t fl[10];
    int nf = 0;
    size_t fs = 0;
    for (size_t i = 0; i <= len && nf < 10; i++) {
        if (i == len || ls[i] == '\t') {
            f[nf] = ls + fs;
            fl[nf] = i - fs;
            nf++;
            fs = i + 1;
        }
    }
    if (nf < 10) return 0;
    for (int k = 0; k < 5; k++) { ob_put(out, f[k], fl[k]); ob_putc(out, '\t'); }
    const int gi = dose_gt_index(f[8], fl[8]);
    if (gi < 0) { ob_puts(out, "NA\n"); return 1; }
    const char *sp = f[9], *le = ls + len;
    int first = 1;
    while (sp < le) {  /* extractGTFromSample :182-203 */
        const char *se = (const char *)memchr(sp, '\t', (size_t)(le - sp));
        if (!se) se = le;
        if (!first) ob_putc(out, ',');
        first = 0;
        int cur = 0, d = -1;
        const char *fst = sp;
        for (const char *q = sp; q <= se; q++) {
            if (q == se || *q == ':') {
                if (cur == gi) {
                    if (q > fst) d = dose_parse(fst, (size_t)(q - fst));
                    break;
                }
                cur++;
                fst = q + 1;
            }
        }
        if (d < 0) ob_puts(out, "NA");
        else ob_putc(out, (char)('0' + d));
        sp = se < le ? se + 1 : le;
    }
    ob_putc(out, '\n');
    return 1;
}
static void dose_help(ob_t *o) {  /* displayHelp :24-47 */
    ob_puts(o,
        "VCFX_dosage_calculator: Calculate genotype dosage for each variant in a VCF file.\n\n"
        "Usage:\n"
        "  VCFX_dosage_calculator [options] [input.vcf]\n"
        "  VCFX_dosage_calculator [options] < input.vcf > dosage_output.txt\n\n"
        "Options:\n"
        "  -i, --input FILE  Input VCF file (uses mmap for best performance)\n"
        "  -q, --quiet       Suppress warning messages\n"
        "  -h, --help        Display this help message and exit\n\n"
        "Description:\n"
        "  For each variant in the input VCF, the tool computes the dosage for each sample\n"
        "  based on the genotype (GT) field. Dosage is defined as the number of alternate\n"
        "  alleles (i.e. each allele > 0 counts as 1). Thus:\n"
        "    0/0  => dosage 0\n"
        "    0/1  => dosage 1\n"
        "    1/1  => dosage 2\n"
        "    1/2  => dosage 2  (each alternate, regardless of numeric value, counts as 1)\n\n"
        "Performance:\n"
        "  When using -i/--input, the tool uses memory-mapped I/O for\n"
        "  ~10-15x faster processing of large files.\n\n"
        "Example:\n"
        "  VCFX_dosage_calculator -i input.vcf > dosage_output.txt\n"
        "  VCFX_dosage_calculator < input.vcf > dosage_output.txt\n");
}
static const char kDoseHdr[] = "CHROM\tPOS\tID\tREF\tALT\tDosages\n";
static const char kDoseNoHdr[] = "Error: VCF header (#CHROM) not found before variant records.\n";
static const char kDoseWarn[] = "Warning: Skipping VCF line with fewer than 10 fields.\n";
/* processFileMmap :375-588; returns the exit code */
static int dose_mmap(const char *path, int quiet, ob_t *out, ob_t *err) {
    char *d;
    size_t n;
    if (read_file(path, &d, &n) < 0) {
        ob_printf(err, "Error: cannot open file '%s'\n", path);
        return 1;
    }
    if (n == 0) { free(d); return 0; }
    ob_t o = {0};
    ob_puts(&o, kDoseHdr);
    int hdr = 0, rc = 0;
    const char *p = d, *end = d + n;
    while (p < end) {
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        const char *le = nl ? nl : end;
        size_t len = (size_t)(le - p);
        if (len > 0 && p[len - 1] == '\r') len--;
        if (len == 0) { p = le + 1; continue; }
        if (*p == '#') {
            if (len >= 6 && memcmp(p, "#CHROM", 6) == 0) hdr = 1;
            p = le + 1;
            continue;
        }
        if (!hdr) { ob_puts(err, kDoseNoHdr); rc = 1; break; }
        if (!dose_line(p, len, &o) && !quiet) ob_puts(err, kDoseWarn);
        p = le + 1;
    }
    if (rc == 0) ob_put(out, o.p, o.n);  /* (the error path never writes its buffer) */
    free(o.p);
    free(d);
    return rc;
}
/* calculateDosage :209-360 (getline: no '\r' strip; the warning ignores -q) */
static void dose_stdin(const char *d, size_t n, ob_t *out, ob_t *err) {
    ob_t o = {0};
    ob_puts(&o, kDoseHdr);
    int hdr = 0, bad = 0;
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        if (le == ls) continue;
        if (*ls == '#') {
            if (starts_chrom(ls, (size_t)(le - ls))) hdr = 1;
            continue;
        }
        if (!hdr) { ob_puts(err, kDoseNoHdr); bad = 1; break; }
        if (!dose_line(ls, (size_t)(le - ls), &o)) ob_puts(err, kDoseWarn);
    }
    if (!bad) ob_put(out, o.p, o.n);
    free(o.p);
}
/* main :614-620 -> run :52-102 */
static int dose_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_dosage_calculator", dose_help, out)) return 0;
    const char *input = NULL;
    int quiet = 0, help = 0;
    static struct option lo[] = {{"help", no_argument, NULL, 'h'},
                                 {"input", required_argument, NULL, 'i'},
                                 {"quiet", no_argument, NULL, 'q'},
                                 {NULL, 0, NULL, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    int opt;
    while ((opt = getopt_long(argc, argv, "hi:q", lo, NULL)) != -1) {
        if (opt == 'i') input = optarg;
        else if (opt == 'q') quiet = 1;
        else help = 1;
    }
    errcap_end(&ec, err);
    if (!input && optind < argc) input = argv[optind];
    if (help) { dose_help(out); return 0; }
    if (input) return dose_mmap(input, quiet, out, err);
    dose_stdin(in, inn, out, err);
    return 0;
}

/* ==================================================================================== */
/* VCFX_allele_counter                                             */
/* ==================================================================================== */
/* parseGenotypeRaw, VCFX_allele_counter.cpp:267-294: '.' tokens skipped, digit runs count
 * as REF (== 0) or ALT.  Allele numbers accumulate modulo 2^32 (the reference's int
 * accumulation as built: "4294967296" counts as REF).  A byte other than a digit, '/', '|'
 * or '.' makes the reference loop forever (its cursor never advances): outside the parity
 * domain, skipped here. */
static void ac_parse(const char *g, const char *e, int *ref, int *alt) {
    *ref = *alt = 0;
    while (g < e) {
        while (g < e && (*g == '/' || *g == '|')) g++;
        if (g >= e) break;
        if (*g == '.') { g++; continue; }
        uint32_t a = 0;
        int dig = 0;
        while (g < e && *g >= '0' && *g <= '9') { a = a * 10u + (uint32_t)(*g - '0'); dig = 1; g++; }
        if (dig) { if (a == 0) ++*ref; else ++*alt; }
        else g++;  /* (the reference hangs here) */
    }
}
static const char *ac_find(const char *p, const char *end, char c) {
    const char *q = (const char *)memchr(p, c, (size_t)(end - p));
    return q ? q : end;
}
/* writeInt (ThreadBuffer::writeInt :110-129) */
static void ac_int(ob_t *o, int v) {
    if (v == 0) { ob_putc(o, '0'); return; }
    char t[12];
    int k = 0;
    long long x = v;
    if (x < 0) { ob_putc(o, '-'); x = -x; }
    while (x > 0) { t[k++] = (char)('0' + x % 10); x /= 10; }
    while (k > 0) ob_putc(o, t[--k]);
}
typedef struct {
    size_t *idx;       /* selected sample indices (sampleIndices) */
    size_t m;
    sv_t *suf;         /* per output slot: sample name (the '\t' is appended on output) */
    size_t nsuf;
} ac_sel;
enum { AC_TEXT = 0, AC_AGG = 1, AC_BIN = 2 };
/* the five-field prefix "CHROM\tPOS\tID\tREF\tALT\t" (extractField x5, :577-601) and the
 * sample start (skipFields(4), :604) */
static size_t ac_prefix(const char *ls, const char *le, char *pre, const char **sp) {
    const char *p = ls;
    size_t k = 0;
    for (int f = 0; f < 5; f++) {
        const char *s = p;
        p = ac_find(p, le, '\t');
        memcpy(pre + k, s, (size_t)(p - s));
        k += (size_t)(p - s);
        pre[k++] = '\t';
        if (p < le) p++;
    }
    for (int i = 0; i < 4 && p < le; i++) {
        p = ac_find(p, le, '\t');
        if (p < le) p++;
    }
    *sp = p;
    return k;
}
/* processChunk, :550-642 (the default file path, countAllelesMmapMT): every selected sample
 * gets a row; a sample past the line's last tab counts 0 / 0; the counts pass through int8_t */
static void ac_line_mt(const char *ls, const char *le, const ac_sel *S, ob_t *o) {
    char *pre = (char *)malloc((size_t)(le - ls) + 8);
    const char *p;
    size_t pl = ac_prefix(ls, le, pre, &p);
    size_t ns = 0, cap = 64;
    const char **st = (const char **)malloc(cap * sizeof *st);
    st[ns++] = p;  /* findAllSampleStarts :528-544 */
    while (p < le) {
        p = ac_find(p, le, '\t');
        if (p < le) {
            p++;
            if (ns == cap) { cap *= 2; st = (const char **)realloc(st, cap * sizeof *st); }
            st[ns++] = p;
        }
    }
    for (size_t i = 0; i < S->m; i++) {
        size_t id = S->idx[i];
        int r = 0, a = 0;
        if (id < ns) {
            const char *g = st[id], *nt = id + 1 < ns ? st[id + 1] - 1 : le;
            ac_parse(g, ac_find(g, nt, ':'), &r, &a);
        }
        ob_put(o, pre, pl);
        ob_put(o, S->suf[i].p, S->suf[i].n);
        ob_putc(o, '\t');
        ac_int(o, (int8_t)r);
        ob_putc(o, '\t');
        ac_int(o, (int8_t)a);
        ob_putc(o, '\n');
    }
    free(st);
    free(pre);
}
/* countAllelesUnified :1371-1465 / countAllelesStream :1188-1246: the selected samples in
 * order, the cursor only moving forward (an index below the previous one re-reads the
 * cursor's sample), stopping at the first one past the line */
static void ac_line_seq(const char *ls, const char *le, const ac_sel *S, int kind, ob_t *o) {
    char *pre = (char *)malloc((size_t)(le - ls) + 8);
    const char *p;
    size_t pl = ac_prefix(ls, le, pre, &p);
    long long tr = 0, ta = 0;
    int cnt = 0;
    size_t si = 0;
    const char *s = p;
    for (size_t i = 0; i < S->m; i++) {
        size_t id = S->idx[i];
        while (si < id && s < le) {
            s = ac_find(s, le, '\t');
            if (s < le) s++;
            si++;
        }
        if (s >= le) break;
        const char *ge = ac_find(s, le, ':'), *tp = ac_find(s, le, '\t');
        if (tp < ge) ge = tp;
        int r, a;
        ac_parse(s, ge, &r, &a);
        if (kind == AC_TEXT) {
            ob_put(o, pre, pl);
            ob_put(o, S->suf[i].p, S->suf[i].n);
            ob_putc(o, '\t');
            ac_int(o, r);
            ob_putc(o, '\t');
            ac_int(o, a);
            ob_putc(o, '\n');
        } else if (kind == AC_AGG) {
            tr += r;
            ta += a;
            cnt++;
        } else {
            ob_putc(o, (char)(int8_t)r);
            ob_putc(o, (char)(int8_t)a);
        }
    }
    if (kind == AC_AGG) {
        ob_put(o, pre, pl);
        ob_printf(o, "%lld\t%lld\t%d\n", tr, ta, cnt);
    }
    free(pre);
}
static const char kAcHdr[] = "CHROM\tPOS\tID\tREF\tALT\tSample\tRef_Count\tAlt_Count\n";
/* the #CHROM line's sample names (fields after the 9th tab), appended to names */
static void ac_names(const char *ls, const char *le, sv_t **names, size_t *nn) {
    const char *hp = ls;
    for (int i = 0; i < 9 && hp < le; i++) {
        hp = ac_find(hp, le, '\t');
        if (hp < le) hp++;
    }
    while (hp < le) {
        const char *s = hp;
        hp = ac_find(hp, le, '\t');
        *names = (sv_t *)realloc(*names, (*nn + 1) * sizeof(sv_t));
        (*names)[(*nn)++] = sv(s, (size_t)(hp - s));
        if (hp < le) hp++;
    }
}
typedef struct {
    char **samples;
    size_t ns;
    const char *input;
    int quiet, threads, limit, gzip, kind;
} ac_args;
/* sampleMap lookups (:843-855): the last sample of a duplicated name wins */
static int ac_select(const sv_t *names, size_t nn, const ac_args *A, size_t **idx, size_t *m, ob_t *err) {
    *m = 0;
    *idx = (size_t *)malloc((A->ns ? A->ns : nn) * sizeof(size_t) + 8);
    if (A->ns) {
        for (size_t k = 0; k < A->ns; k++) {
            long hit = -1;
            for (size_t i = 0; i < nn; i++)
                if (sv_eqs(names[i], A->samples[k])) hit = (long)i;
            if (hit < 0) {
                ob_printf(err, "Error: Sample '%s' not found\n", A->samples[k]);
                return -1;
            }
            (*idx)[(*m)++] = (size_t)hit;
        }
    } else
        for (size_t i = 0; i < nn; i++) (*idx)[(*m)++] = i;
    return 0;
}
static int ac_hw_threads(void) {
    long k = sysconf(_SC_NPROCESSORS_ONLN);
    return k > 0 ? (int)k : 0;
}
/* the header scan of the file paths (:802-839 / :1284-1307): '#' lines up to the first
 * other line (an empty line included); names from every "#CHROM" line */
static const char *ac_file_header(const char *d, size_t n, sv_t **names, size_t *nn) {
    const char *p = d, *end = d + n;
    while (p < end) {
        const char *le = ac_find(p, end, '\n');
        if (*p != '#') return p;
        if (le - p >= 6 && memcmp(p, "#CHROM", 6) == 0) ac_names(p, le, names, nn);
        p = le;
        if (p < end) p++;
    }
    return NULL;
}
/* countAllelesMmapMT :786-950 */
static int ac_mmap_mt(const ac_args *A, ob_t *out, ob_t *err) {
    char *d;
    size_t n;
    if (read_file(A->input, &d, &n) < 0) { ob_printf(err, "Error: Cannot open file: %s\n", A->input); return 1; }
    if (n == 0) { free(d); ob_puts(err, "Error: Empty file\n"); return 1; }
    sv_t *names = NULL;
    size_t nn = 0, *idx = NULL, m = 0;
    const char *ds = ac_file_header(d, n, &names, &nn);
    int rc = 0;
    if (nn == 0) { ob_puts(err, "Error: No samples found in VCF\n"); rc = 1; goto done; }
    if (!ds) { ob_puts(err, "Error: No data lines found\n"); rc = 1; goto done; }
    if (ac_select(names, nn, A, &idx, &m, err) < 0) { rc = 1; goto done; }
    {
        int nt = A->threads;
        if (nt <= 0) { nt = ac_hw_threads(); if (nt <= 0) nt = 4; }
        size_t dsz = (size_t)(d + n - ds);
        if (dsz < 10u * 1024 * 1024) nt = 1;
        else if (dsz < 100u * 1024 * 1024 && nt > 4) nt = 4;
        if (!A->quiet) ob_printf(err, "Info: Using %d threads\n", nt);
        sv_t *suf = (sv_t *)malloc((m + 1) * sizeof(sv_t));
        for (size_t i = 0; i < m; i++) suf[i] = names[idx[i]];
        ac_sel S = {idx, m, suf, m};
        ob_puts(out, kAcHdr);
        const char *p = ds, *end = d + n;
        while (p < end) {  /* chunks cut at line ends give the lines of one sequential pass */
            const char *le = ac_find(p, end, '\n');
            if (p < le && *p != '#') ac_line_mt(p, le, &S, out);
            p = le;
            if (p < end) p++;
        }
        free(suf);
    }
done:
    free(idx);
    free(names);
    free(d);
    return rc;
}
/* gzdopen(dup(fd), "wb6") + gzwrite + gzclose (GzipWriter :431-514): one deflate stream,
 * level 6, gzip wrapper, default header */
static void ac_gzip(const ob_t *in, ob_t *out) {
    z_stream z;
    memset(&z, 0, sizeof z);
    deflateInit2(&z, 6, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY);
    z.next_in = (Bytef *)(in->p ? in->p : "");
    z.avail_in = (uInt)in->n;
    int r;
    do {
        ob_reserve(out, 1 << 16);
        z.next_out = (Bytef *)(out->p + out->n);
        z.avail_out = 1 << 16;
        r = deflate(&z, Z_FINISH);
        out->n += (1 << 16) - z.avail_out;
    } while (r != Z_STREAM_END);
    deflateEnd(&z);
}
/* countAllelesUnified :1266-1468 (aggregate, binary, gzip or --limit-samples) */
static int ac_unified(const ac_args *A, ob_t *out, ob_t *err) {
    char *d;
    size_t n;
    if (read_file(A->input, &d, &n) < 0) { ob_printf(err, "Error: Cannot open file: %s\n", A->input); return 1; }
    if (n == 0) { free(d); ob_puts(err, "Error: Empty file\n"); return 1; }
    sv_t *names = NULL;
    size_t nn = 0, *idx = NULL, m = 0;
    const char *ds = ac_file_header(d, n, &names, &nn);
    int rc = 0;
    if (nn == 0) { ob_puts(err, "Error: No samples found in VCF\n"); rc = 1; goto done; }
    if (ac_select(names, nn, A, &idx, &m, err) < 0) { rc = 1; goto done; }
    if (A->limit > 0 && m > (size_t)A->limit) {
        m = (size_t)A->limit;
        if (!A->quiet) ob_printf(err, "Info: Limiting to first %d samples\n", A->limit);
    }
    {
        sv_t *suf = (sv_t *)malloc((m + 1) * sizeof(sv_t));
        for (size_t i = 0; i < m; i++) suf[i] = names[idx[i]];
        ac_sel S = {idx, m, suf, m};
        ob_t o = {0};
        if (A->kind == AC_TEXT) ob_puts(&o, kAcHdr);
        else if (A->kind == AC_AGG) ob_puts(&o, "CHROM\tPOS\tID\tREF\tALT\tTotal_Ref\tTotal_Alt\tSample_Count\n");
        else {  /* BinaryHeader :327-332 (packed, little-endian) */
            unsigned char h[20] = {'V', 'C', 'A', 'C', 1, 0, 0, 0};
            uint32_t ns = (uint32_t)m;
            memcpy(h + 8, &ns, 4);
            ob_put(&o, (const char *)h, 20);
        }
        const char *p = ds ? ds : d + n, *end = d + n;
        while (p < end) {
            const char *le = ac_find(p, end, '\n');
            if (p < le && *p != '#') ac_line_seq(p, le, &S, A->kind, &o);
            p = le;
            if (p < end) p++;
        }
        if (A->gzip) ac_gzip(&o, out);
        else ob_put(out, o.p, o.n);
        free(o.p);
        free(suf);
    }
done:
    free(idx);
    free(names);
    free(d);
    return rc;
}
/* countAllelesStream :1122-1260 (text rows only; every "#CHROM" line appends its names, and
 * re-appends the selection; the suffix list grows by the whole selection each time) */
static int ac_stream(const ac_args *A, const char *d, size_t n, ob_t *out, ob_t *err) {
    sv_t *names = NULL, *suf = NULL;
    size_t nn = 0, m = 0, nsuf = 0, *idx = NULL;
    int found = 0, rc = -1;
    ob_t pend = {0};
    ob_puts(&pend, kAcHdr);
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        if (le == ls) continue;
        if (*ls == '#') {
            if (starts_chrom(ls, (size_t)(le - ls))) {
                ac_names(ls, le, &names, &nn);
                size_t *add = NULL, k = 0;
                if (ac_select(names, nn, A, &add, &k, err) < 0) { free(add); rc = 1; break; }
                idx = (size_t *)realloc(idx, (m + k + 1) * sizeof(size_t));
                memcpy(idx + m, add, k * sizeof(size_t));
                m += k;
                free(add);
                suf = (sv_t *)realloc(suf, (nsuf + m + 1) * sizeof(sv_t));
                for (size_t i = 0; i < m; i++) suf[nsuf++] = names[idx[i]];
                found = 1;
            }
            continue;
        }
        if (!found) { ob_puts(err, "Error: No #CHROM header found before data\n"); rc = 1; break; }
        ac_sel S = {idx, m, suf, nsuf};
        ac_line_seq(ls, le, &S, AC_TEXT, &pend);
        if (pend.n > 64u * 1024 * 1024) { ob_put(out, pend.p, pend.n); pend.n = 0; }
    }
    if (rc < 0) {
        ob_put(out, pend.p, pend.n);
        rc = found ? 0 : 1;
    }
    free(pend.p);
    free(names);
    free(suf);
    free(idx);
    return rc;
}
static void ac_help(ob_t *o) {  /* printHelp :400-426 */
    ob_puts(o,
        "VCFX_allele_counter - Count reference and alternate alleles per sample\n\n"
        "Usage: VCFX_allele_counter [OPTIONS] [FILE]\n\n"
        "Options:\n"
        "  -i, --input FILE      Input VCF file (uses mmap for best performance)\n"
        "  -t, --threads N       Number of threads (default: auto-detect CPU cores)\n"
        "  -s, --samples STR     Space-separated list of sample names to include\n"
        "  -l, --limit-samples N Limit to first N samples (useful for large cohorts)\n"
        "  -a, --aggregate       Output per-variant aggregates instead of per-sample\n"
        "  -z, --gzip            Compress output with gzip (~10x smaller)\n"
        "  -b, --binary          Output binary format (compact, for machine consumption)\n"
        "  -q, --quiet           Suppress informational messages\n"
        "  -h, --help            Display this help message\n"
        "  -v, --version         Display version information\n\n"
        "Examples:\n"
        "  VCFX_allele_counter -i input.vcf > counts.tsv              # Default per-sample\n"
        "  VCFX_allele_counter -a -i input.vcf > aggregate.tsv        # Per-variant aggregates\n"
        "  VCFX_allele_counter -z -i input.vcf > counts.tsv.gz        # Gzip compressed\n"
        "  VCFX_allele_counter -l 100 -i input.vcf > counts.tsv       # First 100 samples\n"
        "  VCFX_allele_counter -b -i input.vcf > counts.bin           # Binary format\n"
        "  VCFX_allele_counter -t 8 -i input.vcf > counts.tsv         # 8 threads\n\n"
        "Output formats:\n"
        "  Default:    CHROM  POS  ID  REF  ALT  Sample  Ref_Count  Alt_Count\n"
        "  Aggregate:  CHROM  POS  ID  REF  ALT  Total_Ref  Total_Alt  Sample_Count\n"
        "  Binary:     Compact binary with header (use -b flag)\n");
}
/* main :1473-1536 over parseArguments :352-395 */
static int ac_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    ac_args A;
    memset(&A, 0, sizeof A);
    char **toks = NULL;
    size_t nt = 0;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if ((!strcmp(a, "--samples") || !strcmp(a, "-s")) && i + 1 < argc) {
            const char *s = argv[++i];  /* split on ' ', each trimmed of " \t\n\r" */
            size_t L = strlen(s), st = 0;
            for (size_t k = 0; k <= L; k++) {
                if (k == L || s[k] == ' ') {
                    if (k > st || (k == L && st < L)) {
                        size_t b = st, e = k;
                        while (b < e && strchr(" \t\n\r", s[b])) b++;
                        while (e > b && strchr(" \t\n\r", s[e - 1])) e--;
                        if (b == e) { b = st; e = k; }  /* all whitespace: left as is */
                        toks = (char **)realloc(toks, (nt + 1) * sizeof(char *));
                        toks[nt++] = strndup(s + b, e - b);
                    }
                    st = k + 1;
                }
            }
        } else if (!strcmp(a, "--input") || !strcmp(a, "-i")) {
            if (i + 1 < argc) A.input = argv[++i];
        } else if (!strcmp(a, "--threads") || !strcmp(a, "-t")) {
            if (i + 1 < argc) A.threads = atoi(argv[++i]);
        } else if (!strcmp(a, "--limit-samples") || !strcmp(a, "-l")) {
            if (i + 1 < argc) A.limit = atoi(argv[++i]);
        } else if (!strcmp(a, "--gzip") || !strcmp(a, "-z")) A.gzip = 1;
        else if (!strcmp(a, "--aggregate") || !strcmp(a, "-a")) A.kind = AC_AGG;
        else if (!strcmp(a, "--binary") || !strcmp(a, "-b")) A.kind = AC_BIN;
        else if (!strcmp(a, "--quiet") || !strcmp(a, "-q")) A.quiet = 1;
        else if (!strcmp(a, "--help") || !strcmp(a, "-h")) {
            ac_help(out);
            for (size_t k = 0; k < nt; k++) free(toks[k]);
            free(toks);
            return 0;
        } else if (a[0] != '-' && !A.input) A.input = a;
    }
    A.samples = toks;
    A.ns = nt;
    int rc;
    for (int i = 1; i < argc; i++)
        if (!strcmp(argv[i], "--version") || !strcmp(argv[i], "-v")) {
            ob_puts(out, "VCFX_allele_counter 2.0 (multi-threaded)\n");
            rc = 0;
            goto end;
        }
    if (!A.quiet) {
        if (nt) {
            ob_puts(err, "Info: Counting alleles for samples:");
            for (size_t k = 0; k < nt; k++) ob_printf(err, " %s", toks[k]);
            ob_puts(err, "\n");
        } else if (A.limit > 0) ob_printf(err, "Info: Counting alleles for first %d samples\n", A.limit);
        else ob_puts(err, "Info: Counting alleles for ALL samples\n");
        if (A.kind == AC_AGG) ob_puts(err, "Info: Output mode: aggregate (per-variant summaries)\n");
        else if (A.kind == AC_BIN) ob_puts(err, "Info: Output mode: binary\n");
        if (A.gzip) ob_puts(err, "Info: Output compression: gzip\n");
    }
    if (A.input) {
        if (!A.quiet) ob_printf(err, "Info: Using mmap mode for file: %s\n", A.input);
        if (A.kind != AC_TEXT || A.gzip || A.limit > 0) rc = ac_unified(&A, out, err);
        else rc = ac_mmap_mt(&A, out, err);
    } else {
        if (!A.quiet) ob_puts(err, "Info: Using stdin streaming mode (single-threaded)\n");
        rc = ac_stream(&A, in, inn, out, err);
    }
end:
    for (size_t k = 0; k < nt; k++) free(toks[k]);
    free(toks);
    return rc;
}

/* ==================================================================================== */
/* VCFX_missing_detector                                           */
/* ==================================================================================== */
/* findTabSIMD :180-191 (first '\t'; '\n' never lies inside a line) */
static const char *md_tab(const char *p, const char *end) {
    while (p < end && *p != '\t' && *p != '\n') p++;
    return p;
}
/* skipToField :277-283 */
static const char *md_skip(const char *p, const char *end, int n) {
    for (int i = 0; i < n && p < end; i++) {
        p = md_tab(p, end);
        if (p < end) p++;
    }
    return p;
}
/* hasMissingGenotypeInSamples :290-336: a '.' of a sample's first ':' sub-field that starts
 * or ends it or touches a '/' or '|' */
static int md_missing(const char *sp, const char *le) {
    if (!memchr(sp, '.', (size_t)(le - sp))) return 0;
    const char *p = sp;
    while (p < le) {
        const char *se = md_tab(p, le), *ge = p;
        while (ge < se && *ge != ':') ge++;
        for (const char *g = p; g < ge; g++)
            if (*g == '.') {
                int prev = g == p || g[-1] == '/' || g[-1] == '|';
                int next = g + 1 >= ge || g[1] == '/' || g[1] == '|';
                if (prev || next) return 1;
            }
        if (se >= le) break;
        p = se + 1;
    }
    return 0;
}
/* the flagged record: INFO (field 7) becomes "MISSING_GENOTYPES=1" when "." or empty, else
 * gains ";MISSING_GENOTYPES=1" (no ';' doubled); the rest verbatim up to le, then '\n'
 * (processMmapZeroCopy :545-576 / detectMissingGenotypes :892-909) */
static void md_flag(const char *ls, const char *le, ob_t *o) {
    const char *is = md_skip(ls, le, 7), *ie = md_tab(is, le);
    ob_put(o, ls, (size_t)(is - ls));
    if (ie == is || (ie - is == 1 && *is == '.')) ob_puts(o, "MISSING_GENOTYPES=1");
    else {
        ob_put(o, is, (size_t)(ie - is));
        if (ie[-1] != ';') ob_putc(o, ';');
        ob_puts(o, "MISSING_GENOTYPES=1");
    }
    ob_put(o, ie, (size_t)(le - ie));
    ob_putc(o, '\n');
}
/* std::ostream << double (precision 6, defaultfloat == %g) */
static void md_stats(ob_t *err, size_t total, size_t miss, const char *tail) {
    double pct = total > 0 ? (100.0 * (double)miss / (double)total) : 0.0;
    ob_printf(err, "Processed %zu variants, %zu with missing genotypes (%g%%)%s\n", total, miss, pct, tail);
}
/* processMmapZeroCopy :450-589 (the file path run() takes, :975-990) */
static int md_mmap(const char *path, int quiet, ob_t *out, ob_t *err) {
    char *d;
    size_t n;
    if (read_file(path, &d, &n) < 0) { ob_printf(err, "Error: Cannot open file: %s\n", path); return 1; }
    if (!quiet) ob_printf(err, "Processing %s (%zu MB)\n", path, n / (1024 * 1024));
    const char *p = d, *end = d + n;
    /* sampleColumnsHaveAnyDots :371-445: the leading '#' lines skipped, then every line that
     * ends in '\n' (the last line without one is not scanned), '#' and empty lines included */
    while (p < end && *p == '#') {
        p = ac_find(p, end, '\n');
        if (p < end) p++;
    }
    size_t lines = 0;
    int dot = 0;
    while (p < end && !dot) {
        const char *le = ac_find(p, end, '\n');
        if (le >= end) break;
        lines++;
        const char *sp = md_skip(p, le, 9);
        if (sp < le && memchr(sp, '.', (size_t)(le - sp))) dot = 1;
        p = le + 1;
    }
    if (!dot) {
        if (!quiet) ob_puts(err, "Fast path: No '.' in sample columns (scan complete)\n");
        ob_put(out, d, n);
        if (!quiet) ob_printf(err, "Processed %zu variants, 0 with missing genotypes (0%%)\n", lines);
        free(d);
        return 0;
    }
    size_t total = 0, miss = 0;
    p = d;
    while (p < end) {
        const char *ls = p, *le = ac_find(p, end, '\n');
        const char *next = le < end ? le + 1 : end, *adj = le;
        if (adj > ls && adj[-1] == '\r') adj--;
        if (adj == ls || *ls == '#') { ob_put(out, ls, (size_t)(next - ls)); p = next; continue; }
        total++;
        const char *sp = md_skip(ls, adj, 9);
        if (sp >= adj || !md_missing(sp, adj)) ob_put(out, ls, (size_t)(next - ls));
        else { miss++; md_flag(ls, adj, out); }
        p = next;
    }
    if (!quiet) md_stats(err, total, miss, "");
    free(d);
    return 0;
}
/* detectMissingGenotypes :860-911 (getline: no '\r' strip, every line ends in '\n') */
static void md_stdin(const char *d, size_t n, ob_t *out) {
    lines_t it = {d, d + n};
    const char *ls, *le;
    while (next_line(&it, &ls, &le)) {
        if (le == ls) { ob_putc(out, '\n'); continue; }
        const char *sp = *ls == '#' ? le : md_skip(ls, le, 9);
        if (sp >= le || !md_missing(sp, le)) { ob_put(out, ls, (size_t)(le - ls)); ob_putc(out, '\n'); }
        else md_flag(ls, le, out);
    }
}
static void md_help(ob_t *o) {  /* displayHelp :916-938 */
    ob_puts(o,
        "VCFX_missing_detector v2.0 - Extreme-performance missing genotype detector\n\n"
        "Usage:\n"
        "  VCFX_missing_detector [OPTIONS] [input.vcf]\n"
        "  VCFX_missing_detector [OPTIONS] < input.vcf > flagged.vcf\n\n"
        "Options:\n"
        "  -i, --input FILE   Input VCF file (uses memory-mapping for best performance)\n"
        "  -t, --threads N    Number of threads (default: auto)\n"
        "  -q, --quiet        Suppress informational messages\n"
        "  -h, --help         Display this help message and exit\n"
        "  -v, --version      Show program version and exit\n\n"
        "Description:\n"
        "  Detects variants with missing sample genotypes and flags them\n"
        "  with 'MISSING_GENOTYPES=1' in the INFO field.\n\n"
        "Performance:\n"
        "  - Memory-mapped I/O: Use -i flag for extreme speed\n"
        "  - SIMD-accelerated '.' character search (AVX2/SSE2/NEON)\n"
        "  - Multi-threaded chunk processing\n"
        "  - Zero-copy output for lines without missing genotypes\n\n"
        "Example:\n"
        "  VCFX_missing_detector -i input.vcf > flagged.vcf\n"
        "  VCFX_missing_detector < input.vcf > flagged.vcf\n");
}
/* run :943-997 */
static int md_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    const char *input = NULL;
    int quiet = 0;
    static struct option lo[] = {{"input", required_argument, NULL, 'i'},
                                 {"threads", required_argument, NULL, 't'},
                                 {"quiet", no_argument, NULL, 'q'},
                                 {"help", no_argument, NULL, 'h'},
                                 {"version", no_argument, NULL, 'v'},
                                 {NULL, 0, NULL, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    int opt, rc = -1;
    while (rc < 0 && (opt = getopt_long(argc, argv, "i:t:qhv", lo, NULL)) != -1) {
        switch (opt) {
            case 'i': input = optarg; break;
            case 't': break;  /* the scan's thread count: no effect on the output */
            case 'q': quiet = 1; break;
            case 'h': md_help(out); rc = 0; break;
            case 'v': ob_puts(out, "VCFX_missing_detector v2.0\n"); rc = 0; break;
            default: md_help(out); rc = 1; break;
        }
    }
    errcap_end(&ec, err);
    if (rc >= 0) return rc;
    if (!input && optind < argc) input = argv[optind];
    if (input) return md_mmap(input, quiet, out, err);
    md_stdin(in, inn, out);
    return 0;
}

/* ==================================================================================== */
/* VCFX_haplotype_phaser (consecutive-variant r^2 on the LD coding)     */
/* ==================================================================================== */
/* parseGenotypeFast, VCFX_haplotype_phaser.cpp:312-357: the allele sum as int8_t, -1 missing */
static int ph_gt(const char *g, size_t n) {
    if (n == 0) return -1;
    if (n == 3 && (g[1] == '/' || g[1] == '|')) {
        if (g[0] == '.' || g[2] == '.') return -1;
        if (g[0] >= '0' && g[0] <= '9' && g[2] >= '0' && g[2] <= '9') return (int8_t)((g[0] - '0') + (g[2] - '0'));
    }
    size_t k = 0;
    while (k < n && g[k] != '/' && g[k] != '|') k++;
    if (k == n) return -1;
    const char *a1 = g, *a2 = g + k + 1;
    size_t n1 = k, n2 = n - k - 1;
    if (!n1 || !n2 || a1[0] == '.' || a2[0] == '.') return -1;
    uint32_t i1 = 0, i2 = 0;  /* (int accumulation; wraps as built) */
    for (size_t j = 0; j < n1; j++) {
        if (a1[j] < '0' || a1[j] > '9') return -1;
        i1 = i1 * 10u + (uint32_t)(a1[j] - '0');
    }
    for (size_t j = 0; j < n2; j++) {
        if (a2[j] < '0' || a2[j] > '9') return -1;
        i2 = i2 * 10u + (uint32_t)(a2[j] - '0');
    }
    return (int8_t)(i1 + i2);
}
/* findGTIndex :289-307 */
static int ph_gt_index(const char *f, size_t n) {
    size_t st = 0;
    int idx = 0;
    for (size_t p = 0; p <= n; p++)
        if (p == n || f[p] == ':') {
            if (p - st == 2 && f[st] == 'G' && f[st + 1] == 'T') return idx;
            idx++;
            st = p + 1;
        }
    return -1;
}
/* extractNthField :265-284 */
static sv_t ph_nth(const char *s, size_t n, int k) {
    size_t st = 0;
    int idx = 0;
    for (size_t p = 0; p <= n; p++)
        if (p == n || s[p] == ':') {
            if (idx == k) return sv(s + st, p - st);
            idx++;
            st = p + 1;
        }
    return sv(s, 0);
}
/* calculateLDFast :366-470 (both builds: integer sums, then the same fp64 sequence) */
void oracle_ph_ld(const int8_t *a, const int8_t *b, size_t n, double *r, double *r2) {
    long long sx = 0, sy = 0, sxy = 0, sx2 = 0, sy2 = 0;
    int vn = 0;
    for (size_t i = 0; i < n; i++) {
        int x = a[i], y = b[i];
        if (x < 0 || y < 0) continue;
        vn++;
        sx += x; sy += y; sxy += x * y; sx2 += x * x; sy2 += y * y;
    }
    *r = *r2 = 0.0;
    if (vn == 0) return;
    double mx = (double)sx / vn, my = (double)sy / vn;
    double cov = ((double)sxy / vn) - (mx * my);
    double vx = ((double)sx2 / vn) - (mx * mx), vy = ((double)sy2 / vn) - (my * my);
    if (vx <= 0.0 || vy <= 0.0) return;
    *r = cov / (sqrt(vx) * sqrt(vy));
    *r2 = *r * *r;
}
typedef struct {
    sv_t chrom;
    int pos;
    size_t ns;
    int8_t *g;
} ph_var;
enum { PH_OK = 0, PH_FEW = 1, PH_POS = 2, PH_NOGT = 3 };
/* the record parse shared by the four paths: fields split on every tab, >= 10 fields, POS all
 * digits (empty = 0), GT index of FORMAT, a genotype per field from the 10th */
static int ph_parse(const char *ls, const char *le, ph_var *v) {
    size_t nf = 1;
    for (const char *p = ls; p < le; p++) nf += *p == '\t';
    if (nf < 10) return PH_FEW;
    const char *f[10];
    const char *p = ls;
    for (int k = 0; k < 10; k++) {
        f[k] = p;
        if (k < 9) p = (const char *)memchr(p, '\t', (size_t)(le - p)) + 1;
    }
    uint32_t pos = 0;
    for (const char *q = f[1]; q < f[2] - 1; q++) {
        if (*q < '0' || *q > '9') return PH_POS;
        pos = pos * 10u + (uint32_t)(*q - '0');
    }
    int gi = ph_gt_index(f[8], (size_t)(f[9] - 1 - f[8]));
    if (gi < 0) return PH_NOGT;
    v->chrom = sv(ls, (size_t)(f[1] - 1 - ls));
    v->pos = (int)pos;
    v->ns = nf - 9;
    v->g = (int8_t *)malloc(v->ns + 1);
    const char *s = f[9];
    for (size_t k = 0; k < v->ns; k++) {
        const char *e = (const char *)memchr(s, '\t', (size_t)(le - s));
        if (!e) e = le;
        sv_t gt = ph_nth(s, (size_t)(e - s), gi);
        v->g[k] = (int8_t)ph_gt(gt.p, gt.n);
        s = e + 1;
    }
    return PH_OK;
}
static void ph_entry(ob_t *o, int idx, const ph_var *v) {
    ob_printf(o, "%d:(", idx);
    ob_put(o, v->chrom.p, v->chrom.n);
    ob_printf(o, ":%d)", v->pos);
}
/* the block decision of groupVariants :1275-1322 / the streaming loops for variant b after a */
static int ph_join(const ph_var *a, const ph_var *b, double thr) {
    double r, r2;
    oracle_ph_ld(a->g, b->g, a->ns < b->ns ? a->ns : b->ns, &r, &r2);
    if (sv_eqs(b->chrom, "1")) return r2 >= thr && r > 0;
    return r2 >= thr;
}
/* phaseHaplotypesMmap :607-751 (stdin_mode 0) / phaseHaplotypes :971-1081 (1); streaming:
 * phaseHaplotypesMmapStreaming :757-965 / phaseHaplotypesStreaming :1086-1259 (a window
 * of `win` variants, CircularVariantBuffer :153-203 restated over variant numbers) */
static void ph_run(const char *d, size_t n, int stdin_mode, int streaming, double thr, size_t win, int quiet,
                   ob_t *out, ob_t *err) {
    lines_t it = {d, d + n};
    const char *ls, *le;
    int found = 0, marker = 0, blockno = 0;
    ph_var *vs = NULL;
    size_t nv = 0, capv = 0;
    /* streaming: the circular buffer of variant numbers */
    size_t cap = win + 1, head = 0, cnt = 0;
    size_t *ring = streaming ? (size_t *)malloc((cap ? cap : 1) * sizeof(size_t)) : NULL;
    sv_t cur = sv("", 0);
    while (next_line(&it, &ls, &le)) {
        if (stdin_mode && le == ls) continue;
        if (le > ls && le[-1] == '\r') le--;
        if (!stdin_mode && le == ls) continue;
        char c0 = le > ls ? *ls : '\0';
        if (c0 == '#') {
            if (starts_chrom(ls, (size_t)(le - ls))) found = 1;
            ob_put(out, ls, (size_t)(le - ls));
            ob_putc(out, '\n');
            continue;
        }
        if (!found) {
            if (!stdin_mode) {
                if (!quiet) ob_puts(err, "Warning: VCF data line before #CHROM\n");
                continue;
            }
            if (!quiet) ob_puts(err, "Error: no #CHROM line found.\n");
            goto done;
        }
        if (streaming && !marker) {
            ob_puts(out, "#HAPLOTYPE_BLOCKS_START (streaming)\n");
            marker = 1;
        }
        ph_var v;
        int st = ph_parse(ls, le, &v);
        if (st == PH_FEW) { if (!quiet) ob_puts(err, "Warning: skipping line with <10 fields\n"); continue; }
        if (st == PH_POS) { if (!quiet) ob_puts(err, "Warning: invalid pos => skip\n"); continue; }
        if (st == PH_NOGT) {
            if (!quiet && !streaming) ob_puts(err, stdin_mode ? "Warning: no GT field\n" : "Warning: no GT field found\n");
            continue;
        }
        if (nv == capv) { capv = capv ? 2 * capv : 64; vs = (ph_var *)realloc(vs, capv * sizeof *vs); }
        vs[nv++] = v;
        if (!streaming) continue;
        size_t vi = nv - 1;
#define PH_AT(i) ring[(head + (i)) % cap]
#define PH_BLOCK(k)                                                      \
    do {                                                                 \
        ob_printf(out, "Block %d: ", ++blockno);                         \
        for (size_t j = 0; j < (k); j++) {                               \
            ph_entry(out, (int)PH_AT(j), &vs[PH_AT(j)]);                 \
            if (j + 1 < (k)) ob_puts(out, ", ");                         \
        }                                                                \
        ob_putc(out, '\n');                                              \
    } while (0)
#define PH_PUSH(x)                                                       \
    do {                                                                 \
        ring[(head + cnt) % cap] = (x);                                  \
        if (cnt < cap) cnt++;                                            \
        else head = (head + 1) % cap;                                    \
    } while (0)
        if (cnt == 0) {
            PH_PUSH(vi);
            cur = v.chrom;
            continue;
        }
        if (!(cur.n == v.chrom.n && memcmp(cur.p, v.chrom.p, cur.n) == 0)) {
            PH_BLOCK(cnt);
            head = cnt = 0;
            PH_PUSH(vi);
            cur = v.chrom;
            continue;
        }
        if (ph_join(&vs[ring[(head + cnt - 1) % cap]], &v, thr)) {
            PH_PUSH(vi);
            if (cnt > win) {
                size_t ev = cnt - win;
                PH_BLOCK(ev);
                for (size_t j = 0; j < ev; j++) if (cnt) { head = (head + 1) % cap; cnt--; }
            }
        } else {
            PH_BLOCK(cnt);
            head = cnt = 0;
            PH_PUSH(vi);
        }
    }
    if (streaming) {
        if (cnt) PH_BLOCK(cnt);
        if (marker) ob_puts(out, "#HAPLOTYPE_BLOCKS_END\n");
        goto done;
    }
    if (nv == 0) {
        if (!quiet) ob_puts(err, "Error: no variant data found.\n");
        goto done;
    }
    ob_puts(out, "#HAPLOTYPE_BLOCKS_START\n");
    for (size_t i = 0; i < nv; i++) {
        int start = i == 0 || !sv_eq(vs[i].chrom, vs[i - 1].chrom.p, vs[i - 1].chrom.n) || !ph_join(&vs[i - 1], &vs[i], thr);
        if (start) {
            if (i) ob_putc(out, '\n');
            ob_printf(out, "Block %d: ", ++blockno);
        } else ob_puts(out, ", ");
        ph_entry(out, (int)i, &vs[i]);
    }
    ob_puts(out, "\n#HAPLOTYPE_BLOCKS_END\n");
done:
#undef PH_AT
#undef PH_BLOCK
#undef PH_PUSH
    for (size_t i = 0; i < nv; i++) free(vs[i].g);
    free(vs);
    free(ring);
}
static void ph_help(ob_t *o) {  /* displayHelp :571-601 */
    ob_puts(o,
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
        "  VCFX_haplotype_phaser --streaming -w 500 -i large.vcf\n");
}
/* std::stod / std::stoul: no conversion or ERANGE -> the error path */
static int ph_stod(const char *s, double *v) {
    char *e;
    errno = 0;
    *v = strtod(s, &e);
    return e != s && errno != ERANGE;
}
static int ph_stoul(const char *s, unsigned long *v) {
    char *e;
    errno = 0;
    *v = strtoul(s, &e, 10);
    return e != s && errno != ERANGE;
}
/* main :1336-1342 (handle_common_flags) + run :478-569 */
static int ph_main(int argc, char **argv, const char *in, size_t inn, ob_t *out, ob_t *err) {
    if (common_flags(argc, argv, "VCFX_haplotype_phaser", ph_help, out)) return 0;
    double thr = 0.8;
    unsigned long win = 1000;
    int streaming = 0, quiet = 0, help = 0;
    const char *input = NULL;
    static struct option lo[] = {{"help", no_argument, NULL, 'h'},      {"ld-threshold", required_argument, NULL, 'l'},
                                 {"streaming", no_argument, NULL, 's'}, {"window", required_argument, NULL, 'w'},
                                 {"input", required_argument, NULL, 'i'}, {"quiet", no_argument, NULL, 'q'},
                                 {NULL, 0, NULL, 0}};
    optind = 0;
    errcap_t ec;
    errcap_begin(&ec);
    int opt, rc = -1;
    while (rc < 0 && (opt = getopt_long(argc, argv, "hl:sw:i:q", lo, NULL)) != -1) {
        switch (opt) {
            case 'h': help = 1; break;
            case 'l':
                if (!ph_stod(optarg, &thr)) {
                    errcap_end(&ec, err);
                    ob_puts(err, "Error: invalid LD threshold.\n");
                    ph_help(out);
                    return 1;
                }
                break;
            case 's': streaming = 1; break;
            case 'w':
                if (!ph_stoul(optarg, &win)) {
                    errcap_end(&ec, err);
                    ob_puts(err, "Error: invalid window size.\n");
                    ph_help(out);
                    return 1;
                }
                break;
            case 'i': input = optarg; break;
            case 'q': quiet = 1; break;
            default: help = 1;
        }
    }
    errcap_end(&ec, err);
    if (!input && optind < argc) input = argv[optind];
    if (help) { ph_help(out); return 0; }
    if (thr < 0.0 || thr > 1.0) {
        ob_puts(err, "Error: invalid LD threshold\n");
        ph_help(out);
        return 1;
    }
    if (input && strcmp(input, "-") != 0) {
        char *d;
        size_t n;
        if (read_file(input, &d, &n) < 0) {
            ob_printf(err, "Error: Cannot open file: %s\n", input);
            return 0;
        }
        if (n) ph_run(d, n, 0, streaming, thr, (size_t)win, quiet, out, err);
        free(d);
    } else
        ph_run(in, inn, 1, streaming, thr, (size_t)win, quiet, out, err);
    return 0;
}

int oracle_main(const char *tool, int argc, char **argv, const char *in, size_t inn, oracle_result *res) {
    ob_t out = {0}, err = {0};
    int rc;
    const char *t = strrchr(tool, '/');
    t = t ? t + 1 : tool;
    if (strcmp(t, "VCFX_allele_freq_calc") == 0) rc = af_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_variant_counter") == 0) rc = vc_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_genotype_query") == 0) rc = gq_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_record_filter") == 0) rc = rf_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_ld_calculator") == 0) rc = ld_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_nonref_filter") == 0) rc = nr_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_hwe_tester") == 0) rc = hwe_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_dosage_calculator") == 0) rc = dose_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_allele_counter") == 0) rc = ac_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_missing_detector") == 0) rc = md_main(argc, argv, in, inn, &out, &err);
    else if (strcmp(t, "VCFX_haplotype_phaser") == 0) rc = ph_main(argc, argv, in, inn, &out, &err);
    else return -1;
    res->out = out.p ? out.p : (char *)calloc(1, 1);
    res->out_len = out.n;
    res->err = err.p ? err.p : (char *)calloc(1, 1);
    res->err_len = err.n;
    res->rc = rc;
    return 0;
}
void oracle_result_free(oracle_result *r) {
    free(r->out);
    free(r->err);
    r->out = r->err = NULL;
}
