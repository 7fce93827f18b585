/* pipe_drain.c -- the pipe-ingest ceiling (measurement tool, build/bin/vcfx_drain): reads all
 * of stdin the way the drop-ins' device-only stdin path does (pipe buffer raised to 1 MiB with
 * F_SETPIPE_SZ, reads of up to 32 MiB into one reused buffer) and discards it; prints
 * "<bytes> <seconds> <GB/s>" on stderr.  `cat F | vcfx_drain` is the rate no stdin reader on
 * the box can beat, the denominator of bench.py's e2e.process_stdin_pipe. */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

int main(int argc, char **argv) {
    /* optional: vcfx_drain BYTES NBUF -- reads rotate over NBUF buffers of BYTES (a staging
     * ring's cache footprint); default one 32 MiB buffer */
    const size_t kBuf = argc > 1 ? (size_t)strtoull(argv[1], NULL, 10) : (size_t)32 << 20;
    const int nbuf = argc > 2 ? atoi(argv[2]) : 1;
    if (!kBuf || nbuf < 1) return 2;
    char *all = malloc(kBuf * (size_t)nbuf);
    if (!all) return 1;
    for (size_t i = 0; i < kBuf * (size_t)nbuf; i += 4096) all[i] = 0;
    int cur = 0;
    if (fcntl(0, F_GETPIPE_SZ) > 0) (void)fcntl(0, F_SETPIPE_SZ, 1 << 20);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    unsigned long long n = 0;
    for (;;) {
        char *b = all + (size_t)cur * kBuf;
        size_t got = 0;
        ssize_t k = 0;
        while (got < kBuf) {  /* fill the buffer, as the staging ring's reader does */
            k = read(0, b + got, kBuf - got);
            if (k < 0 && errno == EINTR) continue;
            if (k <= 0) break;
            got += (size_t)k;
        }
        n += got;
        cur = (cur + 1) % nbuf;
        if (k <= 0) break;
        continue;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    fprintf(stderr, "%llu %.4f %.2f\n", n, s, s > 0 ? (double)n / s / 1e9 : 0.0);
    free(all);
    return 0;
}
