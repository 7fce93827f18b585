/*
 * vcfx_synth.c -- deterministic synthetic VCF generator.
 *
 * Produces chr21-like VCFs: CHROM=21, POS strictly increasing from 9,411,239 with gap
 * U[1,180], ID=rs<k>, single-base REF/ALT (~1% multi-allelic "A,C"), QUAL=100,
 * FILTER=PASS (97%) / LowQual, INFO '.' (chr21-like, ~10.05 KB/record at 2,504 samples)
 * or annotated "AF=..;DP=..", FORMAT=GT, phased a|b genotypes with a skewed site
 * frequency spectrum.  Options: missing rate, haplotype-block mode (LD structure),
 * an "irregular" fraction of records that exercise the general GT path (GT:DP, mixed
 * phasing, multi-digit alleles, haploid, DP:GT), and CRLF line endings.
 *
 * Every random draw is a counter-based hash (splitmix64) of (seed, record, stream), so
 * records can be generated in parallel and the bytes are identical on any host.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint64_t seed;
    int64_t n_records;
    int32_t n_samples;
    int32_t info_mode;       /* 0: INFO='.'  1: AF=..;DP=.. */
    double missing_rate;     /* per-sample probability of ".|." */
    int32_t hap_blocks;      /* 1: founder-haplotype blocks (LD structure) */
    double irregular_rate;   /* fraction of records in a general-path shape */
    int32_t crlf;            /* 1: "\r\n" line endings */
    int32_t format_mode;     /* 0: FORMAT=GT; 1: the regular records as GT:AD:DP ("a|b:x,y:x+y") */
} vcfx_synth_opts;

static inline uint64_t smix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static inline uint64_t rnd(uint64_t seed, uint64_t rec, uint64_t stream) {
    return smix(seed ^ smix(rec * 0x100000001B3ull + stream * 0xD6E8FEB86659FD93ull));
}
static inline double u01(uint64_t r) { return (double)(r >> 11) * (1.0 / 9007199254740992.0); }

static const char BASES[4] = {'A', 'C', 'G', 'T'};
#define START_POS 9411239ll

/* per-record header fields, computed sequentially for POS (cheap) */
typedef struct {
    int64_t pos;
    uint8_t ref, alt, multi, lowqual, irregular;
    double p;      /* alt allele frequency */
} rec_meta;

static void meta_for(const vcfx_synth_opts *o, int64_t k, int64_t pos, rec_meta *m) {
    uint64_t r0 = rnd(o->seed, (uint64_t)k, 1);
    m->pos = pos;
    m->ref = (uint8_t)(r0 & 3);
    m->alt = (uint8_t)((m->ref + 1 + ((r0 >> 2) % 3)) & 3);
    m->multi = ((r0 >> 8) % 100) == 0;
    m->lowqual = ((r0 >> 16) % 100) < 3;
    double u = u01(rnd(o->seed, (uint64_t)k, 2));
    double p = 0.5 * u * u * u * u * u * u;  /* skewed SFS: most sites rare */
    if (p < 1.0 / (2.0 * (o->n_samples > 0 ? o->n_samples : 1))) p = 1.0 / (2.0 * (o->n_samples > 0 ? o->n_samples : 1));
    m->p = p;
    m->irregular = o->irregular_rate > 0.0 && u01(rnd(o->seed, (uint64_t)k, 3)) < o->irregular_rate;
}

static size_t put_int(char *b, int64_t v) {
    char t[24];
    int i = 0;
    if (v == 0) { b[0] = '0'; return 1; }
    int neg = v < 0;
    uint64_t u = neg ? (uint64_t)(-v) : (uint64_t)v;
    while (u) { t[i++] = (char)('0' + u % 10); u /= 10; }
    size_t n = 0;
    if (neg) b[n++] = '-';
    while (i) b[n++] = t[--i];
    return n;
}

/* genotype allele for haplotype h (0/1) of sample s at record k */
static inline int allele_of(const vcfx_synth_opts *o, int64_t k, const rec_meta *m, int s, int h) {
    uint64_t r;
    if (o->hap_blocks) {
        /* 100 founders; a sample haplotype copies a founder chosen per 64-record block.
         * Founder f carries the ALT allele at site k iff its per-block key is below the
         * site's frequency, so the carrier sets of a block's sites are nested (strong LD
         * between sites of similar frequency); 0.5% copying error */
        int64_t blk = k / 64;
        int f = (int)(rnd(o->seed, (uint64_t)blk, 1000 + (uint64_t)(2 * s + h)) % 100);
        double key = u01(rnd(o->seed, (uint64_t)blk, 5000 + (uint64_t)f));
        int a = key < (m->p < 0.05 ? 0.05 + m->p : m->p);
        if (u01(rnd(o->seed, (uint64_t)k, 9000000 + (uint64_t)(2 * s + h))) < 0.005) a ^= 1;
        return a;
    }
    r = rnd(o->seed, (uint64_t)k, 100 + (uint64_t)(2 * s + h));
    int a = u01(r) < m->p;
    if (a && m->multi && (r & 1)) a = 2;
    return a;
}

/* write (or, if b==NULL, measure) record k; returns bytes */
static size_t emit_record(const vcfx_synth_opts *o, int64_t k, const rec_meta *m, char *b) {
    char tmp[256];
    char *w = b ? b : tmp;
    size_t n = 0;
#define PUT(c) do { if (b) w[n] = (c); n++; } while (0)
#define PUTS(s, l) do { if (b) memcpy(w + n, (s), (l)); n += (l); } while (0)
    char nb[32];
    size_t l;
    PUTS("21\t", 3);
    l = put_int(nb, m->pos); PUTS(nb, l); PUT('\t');
    PUTS("rs", 2); l = put_int(nb, k + 1); PUTS(nb, l); PUT('\t');
    PUT(BASES[m->ref]); PUT('\t');
    PUT(BASES[m->alt]);
    if (m->multi) { PUT(','); PUT(BASES[(m->alt + 1) & 3] == BASES[m->ref] ? BASES[(m->alt + 2) & 3] : BASES[(m->alt + 1) & 3]); }
    PUTS("\t100\t", 5);
    if (m->lowqual) PUTS("LowQual", 7); else PUTS("PASS", 4);
    PUT('\t');
    if (o->info_mode == 1) {
        /* AF with 4 decimals of p (exactly representable text), DP in [10, 5000) */
        int64_t afq = (int64_t)(m->p * 10000.0 + 0.5);
        PUTS("AF=0.", 5);
        nb[0] = (char)('0' + (afq / 1000) % 10); nb[1] = (char)('0' + (afq / 100) % 10);
        nb[2] = (char)('0' + (afq / 10) % 10); nb[3] = (char)('0' + afq % 10);
        PUTS(nb, 4);
        PUTS(";DP=", 4);
        l = put_int(nb, 10 + (int64_t)(rnd(o->seed, (uint64_t)k, 4) % 4990)); PUTS(nb, l);
    } else {
        PUT('.');
    }
    int shape = 0;
    if (m->irregular) shape = 1 + (int)(rnd(o->seed, (uint64_t)k, 6) % 5);
    const int fmt3 = o->format_mode == 1 && shape == 0;
    if (!b && shape == 0 && !fmt3) {
        /* regular record: "\tGT" + N x "\ta|b" (missing ".|." has the same width) */
        n += 3 + 4 * (size_t)o->n_samples + (o->crlf ? 2 : 1);
        return n;
    }
    if (shape == 1) PUTS("\tGT:DP", 6);
    else if (shape == 5) PUTS("\tDP:GT", 6);
    else if (fmt3) PUTS("\tGT:AD:DP", 9);
    else PUTS("\tGT", 3);
    for (int s = 0; s < o->n_samples; s++) {
        PUT('\t');
        int a0 = allele_of(o, k, m, s, 0), a1 = allele_of(o, k, m, s, 1);
        int miss = o->missing_rate > 0.0 && u01(rnd(o->seed, (uint64_t)k, 20000000 + (uint64_t)s)) < o->missing_rate;
        uint64_t rs = shape ? rnd(o->seed, (uint64_t)k, 30000000 + (uint64_t)s) : 0;
        if (shape == 5) { l = put_int(nb, (int64_t)(rs % 60)); PUTS(nb, l); PUT(':'); }
        if (miss) { PUT('.'); PUT(shape == 2 && (rs & 1) ? '/' : '|'); PUT('.'); }
        else if (shape == 4 && (rs % 7) == 0) { PUT((char)('0' + a0)); }                       /* haploid */
        else if (shape == 3 && (rs % 11) == 0) { PUTS("10", 2); PUT('|'); PUT((char)('0' + a1)); } /* multi-digit */
        else {
            PUT((char)('0' + a0));
            PUT(shape == 2 && (rs & 1) ? '/' : '|');
            PUT((char)('0' + a1));
        }
        if (shape == 1) { PUT(':'); l = put_int(nb, (int64_t)(rs % 60)); PUTS(nb, l); }
        if (fmt3) {  /* AD (two read depths < 31) and DP = their sum */
            const uint64_t r3 = rnd(o->seed, (uint64_t)k, 40000000 + (uint64_t)s);
            const int64_t d0 = (int64_t)(r3 % 31), d1 = (int64_t)((r3 >> 8) % 31);
            PUT(':'); l = put_int(nb, d0); PUTS(nb, l); PUT(','); l = put_int(nb, d1); PUTS(nb, l);
            PUT(':'); l = put_int(nb, d0 + d1); PUTS(nb, l);
        }
    }
    if (o->crlf) PUT('\r');
    PUT('\n');
#undef PUT
#undef PUTS
    return n;
}

static size_t emit_header(const vcfx_synth_opts *o, char *b) {
    size_t n = 0;
    char line[64];
#define PUTS(s) do { size_t _l = strlen(s); if (b) memcpy(b + n, (s), _l); n += _l; } while (0)
    const char *eol = o->crlf ? "\r\n" : "\n";
    PUTS("##fileformat=VCFv4.1"); PUTS(eol);
    PUTS("##source=vcfx_amd.synth"); PUTS(eol);
    PUTS("##contig=<ID=21,length=48129895>"); PUTS(eol);
    if (o->info_mode == 1) {
        PUTS("##INFO=<ID=AF,Number=A,Type=Float,Description=\"Allele Frequency\">"); PUTS(eol);
        PUTS("##INFO=<ID=DP,Number=1,Type=Integer,Description=\"Total Depth\">"); PUTS(eol);
    }
    PUTS("##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">"); PUTS(eol);
    PUTS("##FORMAT=<ID=DP,Number=1,Type=Integer,Description=\"Read Depth\">"); PUTS(eol);
    if (o->format_mode == 1) { PUTS("##FORMAT=<ID=AD,Number=R,Type=Integer,Description=\"Allelic depths\">"); PUTS(eol); }
    PUTS("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT");
    for (int s = 0; s < o->n_samples; s++) {
        snprintf(line, sizeof line, "\tS%05d", s + 1);
        PUTS(line);
    }
    PUTS(eol);
#undef PUTS
    return n;
}

typedef struct {
    const vcfx_synth_opts *o;
    const rec_meta *meta;
    const size_t *off;
    char *buf;
    int64_t r0, r1;
} job_t;

static void *fill_job(void *arg) {
    job_t *j = (job_t *)arg;
    for (int64_t k = j->r0; k < j->r1; k++) emit_record(j->o, k, &j->meta[k], j->buf + j->off[k]);
    return NULL;
}

static rec_meta *build_meta(const vcfx_synth_opts *o) {
    rec_meta *meta = (rec_meta *)malloc(sizeof(rec_meta) * (size_t)(o->n_records > 0 ? o->n_records : 1));
    int64_t pos = START_POS;
    for (int64_t k = 0; k < o->n_records; k++) {
        if (k) pos += 1 + (int64_t)(rnd(o->seed, (uint64_t)k, 0) % 180);
        meta_for(o, k, pos, &meta[k]);
    }
    return meta;
}

/* total size in bytes of the VCF described by o */
size_t vcfx_synth_size(const vcfx_synth_opts *o) {
    rec_meta *meta = build_meta(o);
    size_t n = emit_header(o, NULL);
    for (int64_t k = 0; k < o->n_records; k++) n += emit_record(o, k, &meta[k], NULL);
    free(meta);
    return n;
}

/* fill buf (capacity cap) with the VCF; returns bytes written or 0 if cap too small.
 * rec_off (optional, n_records+1 entries) receives each record's byte offset. */
size_t vcfx_synth_fill(const vcfx_synth_opts *o, char *buf, size_t cap, int nthreads, uint64_t *rec_off) {
    rec_meta *meta = build_meta(o);
    size_t *off = (size_t *)malloc(sizeof(size_t) * (size_t)(o->n_records + 1));
    size_t n = emit_header(o, NULL);
    for (int64_t k = 0; k < o->n_records; k++) { off[k] = n; n += emit_record(o, k, &meta[k], NULL); }
    off[o->n_records] = n;
    if (n > cap) { free(meta); free(off); return 0; }
    emit_header(o, buf);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    job_t jobs[64];
    int64_t per = (o->n_records + nthreads - 1) / nthreads;
    int started = 0;
    for (int t = 0; t < nthreads; t++) {
        int64_t r0 = t * per, r1 = r0 + per;
        if (r0 >= o->n_records) break;
        if (r1 > o->n_records) r1 = o->n_records;
        jobs[t] = (job_t){o, meta, off, buf, r0, r1};
        pthread_create(&th[t], NULL, fill_job, &jobs[t]);
        started++;
    }
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    if (rec_off)
        for (int64_t k = 0; k <= o->n_records; k++) rec_off[k] = off[k];
    free(meta);
    free(off);
    return n;
}

#ifdef VCFX_SYNTH_MAIN
/* vcfx_synth OUT.vcf N_RECORDS N_SAMPLES [seed] [info_mode] [missing_rate] [hap_blocks]
 *            [irregular_rate] [crlf] */
int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: vcfx_synth OUT N_RECORDS N_SAMPLES [seed info_mode missing hap irregular crlf]\n");
        return 2;
    }
    vcfx_synth_opts o = {20251226ull, atoll(argv[2]), atoi(argv[3]), 0, 0.0, 0, 0.0, 0, 0};
    if (argc > 4) o.seed = strtoull(argv[4], NULL, 10);
    if (argc > 5) o.info_mode = atoi(argv[5]);
    if (argc > 6) o.missing_rate = atof(argv[6]);
    if (argc > 7) o.hap_blocks = atoi(argv[7]);
    if (argc > 8) o.irregular_rate = atof(argv[8]);
    if (argc > 9) o.crlf = atoi(argv[9]);
    if (argc > 10) o.format_mode = atoi(argv[10]);
    size_t n = vcfx_synth_size(&o);
    char *buf = (char *)malloc(n);
    vcfx_synth_fill(&o, buf, n, 8, NULL);
    FILE *f = strcmp(argv[1], "-") == 0 ? stdout : fopen(argv[1], "wb");
    if (!f) { perror("open"); return 1; }
    fwrite(buf, 1, n, f);
    if (f != stdout) fclose(f);
    free(buf);
    return 0;
}
#endif
