/* oracle_cli.c -- `vcfx_oracle <tool> [args...]` runs the C restatement of <tool> as a
 * process (stdin -> stdout/stderr/exit code).  TEST INFRASTRUCTURE ONLY. */
#include "vcfx_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: vcfx_oracle <VCFX_tool> [args...]\n"); return 2; }
    size_t cap = 1 << 20, n = 0;
    char *in = malloc(cap);
    if (!isatty(0)) {
        for (;;) {
            if (n == cap) { cap *= 2; in = realloc(in, cap); }
            ssize_t k = read(0, in + n, cap - n);
            if (k <= 0) break;
            n += (size_t)k;
        }
    }
    oracle_result r;
    if (oracle_main(argv[1], argc - 1, argv + 1, in, n, &r) != 0) { fprintf(stderr, "unknown tool\n"); return 2; }
    fwrite(r.out, 1, r.out_len, stdout);
    fflush(stdout);
    fwrite(r.err, 1, r.err_len, stderr);
    int rc = r.rc;
    oracle_result_free(&r);
    free(in);
    return rc;
}
