/*
 * atz_oracle.h -- CPU restatement of the AntiZ hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X product in antiz_amd/.  It restates, in plain C,
 *   - zlib 1.2.8 deflate (vendored by the reference, `includes, tools, stuff/zlib test/zlib128/`)
 *     for level 0..9, windowBits 9..15, memLevel 1..9, Z_DEFAULT_STRATEGY, one-shot Z_FINISH;
 *   - zlib 1.2.8 inflate acceptance/consumption semantics as the reference's scanner sees them;
 *   - the reference's chunked magic-byte scan (main.cpp:149-249, 392-420), its recompression
 *     parameter sweep (main.cpp:421-763), the ATZ1 writer (main.cpp:764-834) and the
 *     reconstructor (main.cpp:862-1064).
 * It is pinned against the REAL reference built by oracle/build_ref.sh (oracle/_ref/).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 */
#ifndef ATZ_ORACLE_H
#define ATZ_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- deflate (zlib 1.2.8 deflate.c / trees.c restated) ---- */
uint64_t ora_deflate_bound(uint64_t n, int wbits, int memlevel);
/* returns 0 ok, -1 bad params, -2 out_cap too small; *flags bit0 = pending-overlay hazard seen */
int ora_deflate(const uint8_t *in, uint64_t n, int level, int wbits, int memlevel,
                uint8_t *out, uint64_t out_cap, uint64_t *out_len, int *flags);

/* ---- inflate (zlib 1.2.8 inflate.c / inffast.c / inftrees.c semantics) ---- */
enum { ORA_INF_END = 0, ORA_INF_ERROR = 1, ORA_INF_NEED_INPUT = 2 };
/* Decode a zlib stream from in[0..n).  out may be NULL (lengths only).
 * *consumed: bytes zlib would have taken from next_in when it stopped (total_in),
 * *produced: total_out.  Return ORA_INF_*. */
int ora_inflate(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                uint64_t *consumed, uint64_t *produced);
uint32_t ora_adler32(uint32_t adler, const uint8_t *buf, uint64_t len);

/* ---- pipeline ---- */
typedef struct {
    uint64_t recomp_tresh, sizediff_tresh, shortcut_len, mismatch_tol; /* uint_fast16_t == 64-bit */
    uint64_t chunksize;
    int brute_window;
} ora_opts_t;

typedef struct {            /* ATZdata::streamOffset (ATZData.h:42-77), flattened */
    uint64_t offset;
    int32_t  type;
    uint8_t  clevel, window, memlevel, recomp;
    uint64_t comp_len, infl_len, ident;
    int64_t  first_diff;
    uint64_t n_diff;        /* diffs live in the caller-visible arrays of ora_result_t */
    uint64_t diff_index;    /* index of this stream's first diff in the flat arrays */
    uint64_t n_trials;      /* trials actually evaluated (diagnostic) */
} ora_stream_t;

typedef struct {
    ora_stream_t *streams; uint64_t n_streams;
    uint64_t *diff_off; uint8_t *diff_val; uint64_t n_diffs;
    uint64_t n_trials, n_shortcut_bailed, n_hazard;
} ora_result_t;

/* Phase 1: chunked scan; fills streams[] (offset,type,comp_len,infl_len).  Returns 0 or <0. */
int ora_scan(const uint8_t *file, uint64_t n, uint64_t chunksize, ora_result_t *res);
/* Phase 3: parameter sweep over res->streams (as produced by ora_scan). */
int ora_sweep(const uint8_t *file, uint64_t n, const ora_opts_t *o, ora_result_t *res);
/* Phase 4: ATZ1 bytes.  *atz is malloc'd (free with ora_free). */
int ora_write_atz(const uint8_t *file, uint64_t n, const ora_result_t *res, uint8_t **atz, uint64_t *atz_len);
/* Whole precompress (Phase1+3+4). */
int ora_precompress(const uint8_t *file, uint64_t n, const ora_opts_t *o, uint8_t **atz,
                    uint64_t *atz_len, ora_result_t *res_out /* may be NULL */);
/* Reconstruct (-r). 0 ok, <0 invalid file. */
int ora_reconstruct(const uint8_t *atz, uint64_t n, uint8_t **out, uint64_t *out_len);
void ora_result_free(ora_result_t *res);
void ora_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
