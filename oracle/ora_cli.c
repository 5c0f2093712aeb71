/* ora_cli -- command-line driver of the oracle restatement (test infrastructure / CPU "port" baseline).
 * usage: ora_cli precompress IN OUT [chunksize recomp sizediff shortcut tol brute]
 *        ora_cli reconstruct IN OUT
 * Prints one JSON line with phase timings. */
#define _POSIX_C_SOURCE 199309L
#include "atz_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }
static uint8_t *slurp(const char *p, uint64_t *n) {
    FILE *f = fopen(p, "rb"); if (!f) return NULL;
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t *b = (uint8_t *)malloc(sz ? sz : 1);
    if (fread(b, 1, sz, f) != (size_t)sz) { fclose(f); free(b); return NULL; }
    fclose(f); *n = (uint64_t)sz; return b;
}
int main(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s precompress|reconstruct IN OUT [...]\n", argv[0]); return 2; }
    uint64_t n; uint8_t *in = slurp(argv[2], &n);
    if (!in) { fprintf(stderr, "cannot read %s\n", argv[2]); return 2; }
    uint8_t *out = NULL; uint64_t on = 0;
    if (!strcmp(argv[1], "precompress")) {
        ora_opts_t o = {128, 128, 512, 2, 524288, 0};
        if (argc > 4) o.chunksize = strtoull(argv[4], 0, 10);
        if (argc > 5) o.recomp_tresh = strtoull(argv[5], 0, 10);
        if (argc > 6) o.sizediff_tresh = strtoull(argv[6], 0, 10);
        if (argc > 7) o.shortcut_len = strtoull(argv[7], 0, 10);
        if (argc > 8) o.mismatch_tol = strtoull(argv[8], 0, 10);
        if (argc > 9) o.brute_window = atoi(argv[9]);
        ora_result_t res;
        double t0 = now();
        int r = ora_scan(in, n, o.chunksize, &res);
        double t1 = now();
        if (!r) r = ora_sweep(in, n, &o, &res);
        double t2 = now();
        if (!r) r = ora_write_atz(in, n, &res, &out, &on);
        double t3 = now();
        if (r) { fprintf(stderr, "precompress failed: %d\n", r); return 1; }
        uint64_t nrec = 0; for (uint64_t s = 0; s < res.n_streams; s++) nrec += res.streams[s].recomp;
        printf("{\"streams\": %llu, \"recomp\": %llu, \"trials\": %llu, \"bailed\": %llu, \"hazard\": %llu, "
               "\"scan_s\": %.6f, \"sweep_s\": %.6f, \"write_s\": %.6f, \"bytes\": %llu}\n",
               (unsigned long long)res.n_streams, (unsigned long long)nrec, (unsigned long long)res.n_trials,
               (unsigned long long)res.n_shortcut_bailed, (unsigned long long)res.n_hazard,
               t1 - t0, t2 - t1, t3 - t2, (unsigned long long)n);
        ora_result_free(&res);
    } else {
        int r = ora_reconstruct(in, n, &out, &on);
        if (r) { fprintf(stderr, "reconstruct failed: %d\n", r); return 1; }
    }
    FILE *f = fopen(argv[3], "wb");
    if (!f || fwrite(out, 1, on, f) != on) { fprintf(stderr, "write failed\n"); return 1; }
    fclose(f);
    return 0;
}
