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

int main(void) {
    const size_t kBuf = (size_t)32 << 20;
    char *b = malloc(kBuf);
    if (!b) return 1;
    if (fcntl(0, F_GETPIPE_SZ) > 0) (void)fcntl(0, F_SETPIPE_SZ, 1 << 20);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    unsigned long long n = 0;
    for (;;) {
        ssize_t k = read(0, b, kBuf);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) break;
        n += (unsigned long long)k;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    fprintf(stderr, "%llu %.4f %.2f\n", n, s, s > 0 ? (double)n / s / 1e9 : 0.0);
    free(b);
    return 0;
}
