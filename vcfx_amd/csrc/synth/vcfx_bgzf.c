/*
 * vcfx_bgzf.c -- BGZF writer for test and bench inputs (the .vcf.gz form of a synthetic VCF).
 *
 * BGZF (SAM/BAM spec §4.1): a series of gzip members, each holding at most 64 KiB of input,
 * whose FEXTRA field carries the subfield 'B','C' (SLEN 2) = member size - 1, ended by the
 * standard 28-byte empty member.  Blocks are compressed on several threads and written in
 * order.  --plain writes one ordinary gzip member instead (the sequential-inflate case).
 *
 *   vcfx_bgzf IN OUT [threads] [level] [--plain]
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>
#include <zlib.h>

#define BLOCK_IN 65280u   /* input bytes per block, as bgzip */
#define BLOCK_MAX 65536u  /* a member never exceeds this */

typedef struct {
    const uint8_t *in;
    size_t n, nblocks;
    uint8_t *out;      /* nblocks * BLOCK_MAX */
    uint32_t *osize;
    int level, T, id;
} job;

static const uint8_t EOF_BLOCK[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                                      0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

static void put32(uint8_t *p, uint32_t v) { p[0] = v; p[1] = v >> 8; p[2] = v >> 16; p[3] = v >> 24; }

static void *worker(void *arg) {
    job *j = (job *)arg;
    for (size_t b = j->id; b < j->nblocks; b += j->T) {
        const uint8_t *src = j->in + b * BLOCK_IN;
        const size_t len = b * BLOCK_IN + BLOCK_IN <= j->n ? BLOCK_IN : j->n - b * BLOCK_IN;
        uint8_t *dst = j->out + b * (size_t)BLOCK_MAX;
        z_stream z;
        memset(&z, 0, sizeof z);
        if (deflateInit2(&z, j->level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) exit(3);
        z.next_in = (Bytef *)src;
        z.avail_in = (uInt)len;
        z.next_out = dst + 18;
        z.avail_out = BLOCK_MAX - 26;
        if (deflate(&z, Z_FINISH) != Z_STREAM_END) {
            fprintf(stderr, "vcfx_bgzf: block %zu does not fit\n", b);
            exit(3);
        }
        const size_t clen = (BLOCK_MAX - 26) - z.avail_out;
        deflateEnd(&z);
        const uint8_t hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0, 0, 0};
        memcpy(dst, hdr, 18);
        const uint32_t total = (uint32_t)(18 + clen + 8);
        dst[16] = (uint8_t)((total - 1) & 0xff);
        dst[17] = (uint8_t)((total - 1) >> 8);
        put32(dst + 18 + clen, (uint32_t)crc32(crc32(0L, Z_NULL, 0), src, (uInt)len));
        put32(dst + 18 + clen + 4, (uint32_t)len);
        j->osize[b] = total;
    }
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: vcfx_bgzf IN OUT [threads] [level] [--plain]\n");
        return 2;
    }
    int T = argc > 3 ? atoi(argv[3]) : 8, level = argc > 4 ? atoi(argv[4]) : 1;
    int plain = argc > 5 && strcmp(argv[5], "--plain") == 0;
    if (T < 1) T = 1;
    int fd = open(argv[1], O_RDONLY);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) < 0) { perror("open"); return 1; }
    const size_t n = (size_t)st.st_size;
    const uint8_t *in = n ? (const uint8_t *)mmap(NULL, n, PROT_READ, MAP_PRIVATE, fd, 0) : (const uint8_t *)"";
    FILE *f = fopen(argv[2], "wb");
    if (!f) { perror("out"); return 1; }
    if (plain) {
        gzFile g = gzdopen(dup(fileno(f)), "wb1");
        for (size_t o = 0; o < n; o += 1u << 30) gzwrite(g, in + o, (unsigned)(n - o < (1u << 30) ? n - o : (1u << 30)));
        gzclose(g);
        fclose(f);
        return 0;
    }
    const size_t nb = (n + BLOCK_IN - 1) / BLOCK_IN;
    uint8_t *out = (uint8_t *)malloc(nb ? nb * (size_t)BLOCK_MAX : 1);
    uint32_t *osize = (uint32_t *)calloc(nb + 1, 4);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * T);
    job *js = (job *)malloc(sizeof(job) * T);
    for (int t = 0; t < T; t++) {
        js[t] = (job){in, n, nb, out, osize, level, T, t};
        pthread_create(&th[t], NULL, worker, &js[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    for (size_t b = 0; b < nb; b++) fwrite(out + b * (size_t)BLOCK_MAX, 1, osize[b], f);
    fwrite(EOF_BLOCK, 1, sizeof EOF_BLOCK, f);
    fclose(f);
    return 0;
}
