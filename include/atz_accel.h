/*
 * atz_accel.h -- C ABI of libatz_accel.so, the MI355X (gfx950) replacement for AntiZ's codec boundary.
 *
 * The reference talks to zlib directly (ZlibWrapper.h:25-100 for the scanner, raw zlib calls in
 * main.cpp for the sweep, the writer and the reconstructor).  Those calls are per stream and per
 * trial; this ABI is per FILE: one call runs a whole phase on the GPU.  Plain pointers and sizes,
 * no C++ or torch types, negative error codes, no exceptions.  Library-owned arrays are released
 * with atz_free().  One context per process and per GPU; not shared across threads.
 *
 * Reference interface each entry point replaces (file:line in /root/reference):
 *   atz_scan        ATZcreator::searchInfile + ZBuffSearcher + ZlibInflator   main.cpp:392-420, 149-249;
 *                   ZlibWrapper.h:58-82 (inflateReset/inflate(Z_SYNC_FLUSH)/continuePrev/refillInput)
 *   atz_sweep       findDeflateParams_ALL .. testDeflateParams + doInflate     main.cpp:421-763
 *                   (deflateInit2/deflateBound/deflate(Z_FINISH)x2/deflateEnd, inflate(Z_FINISH))
 *   atz_precompress Phase1 + Phase3 + Phase4 (writeATZfile, main.cpp:764-834)  main.cpp:1216-1221
 *   atz_reconstruct ATZreconstructor::reconstructATZ + doDeflate               main.cpp:869-1003
 *   atz_deflate     one deflateInit2/deflate(Z_FINISH)/deflateEnd              main.cpp:976-1003
 *   atz_shard_*     the precompress of one file split over several GPUs (new: the reference is
 *                   single-threaded)
 */
#ifndef ATZ_ACCEL_H
#define ATZ_ACCEL_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct atz_ctx atz_ctx_t;

/* ATZdata::programOptions (ATZData.h:7-35).  The thresholds are uint_fast16_t in the reference,
 * i.e. 64-bit on x86-64 glibc; they are uint64_t here so the unsigned wrap of main.cpp:649 is kept. */
typedef struct {
    uint64_t recomp_tresh;    /* default 128 */
    uint64_t sizediff_tresh;  /* default 128 */
    uint64_t shortcut_len;    /* default 512 */
    uint64_t mismatch_tol;    /* default 2 */
    uint64_t chunksize;       /* default 524288 */
    int32_t  brute_window;    /* default 0 */
    int32_t  device;          /* HIP device ordinal (-1: current) */
} atz_opts_t;

/* ATZdata::streamOffset after Phase 1 (ATZData.h:46-58). */
typedef struct {
    uint64_t offset;
    uint64_t comp_len;   /* streamLength */
    uint64_t infl_len;   /* inflatedLength */
    int32_t  type;       /* offsetType 0..23 */
    uint32_t flags;      /* bit0: recorded through a chunk-boundary continuation; bit1: the first block is
                            dynamic and codes matches but none of length 3-5 (a Z_FILTERED-like stream: the
                            multi-GPU split's cost hint, not part of the reference's record); bits 2-5:
                            the memLevel (1-9) whose lit_bufsize - 1 symbols the first block holds when
                            more blocks follow, else 0 (a sweep hint, likewise not the reference's) */
} atz_cand_t;

/* ATZdata::streamOffset after Phase 3. */
typedef struct {
    uint8_t  clevel, window, memlevel, recomp;
    uint32_t n_trials;       /* trials evaluated (diagnostic) */
    uint64_t ident;          /* identBytes */
    int64_t  first_diff;     /* firstDiffByte (-1: none) */
    uint64_t n_diff;         /* diffByteOffsets.size() (written only for recomp streams) */
    uint64_t diff_index;     /* first entry of this stream in the diff arrays */
} atz_result_t;

typedef struct {
    uint64_t file_bytes, n_streams, n_recomp, n_trials, n_trials_shortcut, n_rounds, atz_bytes;
    uint64_t n_candidates, n_continuations, n_hazard;
    double scan_ms, sweep_ms, write_ms, total_ms;       /* device-synchronised wall times */
    /* per-kernel device time (HIP events on the library's stream) and algorithmic bytes */
    double k_trial_ms, k_inflate_ms, k_chains_ms, k_other_ms;
    uint64_t k_trial_launches, k_inflate_launches, k_chains_launches;
    uint64_t k_trial_alg_bytes, k_inflate_alg_bytes, k_chains_alg_bytes;
    uint64_t trial_parsed_bytes;                         /* inflated bytes the trials actually parsed */
    double k_match_ms;                                   /* match-table kernel (longest_match per position) */
    uint64_t k_match_launches, k_match_positions;
    uint64_t n_trials_rerun;                             /* trials run again after extending their match table */
    uint64_t n_fast_fallbacks;                           /* fast-level steps that walked a chain in the parse */
    uint64_t trial_cyc_total, trial_cyc_tree, trial_cyc_emit, trial_blocks;  /* shader clocks summed over trials */
    uint64_t trial_cyc_heap, trial_cyc_fallback, trial_symbols;   /* heap: ATZ_STEP_CLOCKS builds only */
    uint64_t n_trials_speculative;                       /* trials run ahead of a stream's stop and discarded */
    uint64_t n_reinflated;                               /* recorded streams inflated again (scan output not kept) */
    uint64_t n_inflate_retries;                          /* inflates rerun with the 32 KiB history ring */
    uint64_t n_trials_replayed;                          /* trials that replayed a saved symbol sequence */
    uint64_t n_replay_checked;                           /* replays offered under a match-table check (passed or not) */
    uint64_t n_trials_duplicate;                         /* replays whose output equals their saver's: not launched */
    uint64_t n_fast_restarts;                            /* fast-level exact walks that changed the parse path */
    /* device memory the library held in this process (every context's buffers): the peak during the call,
       and what stays allocated after it (kept for the next call's reuse) */
    uint64_t dev_bytes_peak, dev_bytes_held;
    uint64_t n_trials_skipped;                           /* speculative trials ended by an earlier trial's stop */
} atz_stats_t;

enum {
    ATZ_OK = 0,
    ATZ_E_ARG = -1,          /* bad argument */
    ATZ_E_NODEV = -2,        /* no HIP device / kernels not loadable */
    ATZ_E_HIP = -3,          /* HIP runtime error */
    ATZ_E_NOMEM = -4,        /* device or host allocation failed */
    ATZ_E_REF_ABORT = -5,    /* the reference would abort() here (e.g. main.cpp:450-452, 663-665) */
    ATZ_E_REF_UB = -6,       /* the reference has undefined behaviour on this input (documented) */
    ATZ_E_FORMAT = -7,       /* invalid ATZ file (main.cpp:1018-1025) */
    ATZ_E_INTERNAL = -8
};

int  atz_open(atz_ctx_t **ctx, const atz_opts_t *opts);
void atz_close(atz_ctx_t *ctx);
const char *atz_strerror(int err);
void atz_free(void *p);
void atz_default_opts(atz_opts_t *opts);

/* Phase 1: the reference's chunked scan.  *out (atz_free) receives *n records in scan order. */
int atz_scan(atz_ctx_t *ctx, const uint8_t *file, uint64_t len, atz_cand_t **out, uint64_t *n);

/* Phase 3 on the streams of the LAST atz_scan of this context (cands must be that array).  Returns
 * ATZ_E_ARG unless atz_scan was the previous call on ctx (any other call replaces its records); the
 * scanned host buffer need not stay alive (atz_scan keeps what the sweep needs: the file on the
 * device, each stream's Adler-32 trailer).  One atz_sweep per atz_scan.
 * res[n] is caller-allocated.  *diff_off / *diff_val (atz_free) hold n_diffs delta-encoded entries. */
int atz_sweep(atz_ctx_t *ctx, const atz_cand_t *cands, uint64_t n, atz_result_t *res,
              uint64_t **diff_off, uint8_t **diff_val, uint64_t *n_diffs);

/* Whole precompress of a host buffer: *atz (atz_free) receives the ATZ1 bytes. */
int atz_precompress(atz_ctx_t *ctx, const uint8_t *file, uint64_t len, uint8_t **atz, uint64_t *atz_len,
                    atz_stats_t *stats);

/* Benchmark entry: the input is already resident in HBM (d_file, a device pointer allocated by the
 * caller with >= 4096 bytes of slack after len) and a host copy is given for host-side bookkeeping.
 * The ATZ1 bytes are assembled in device memory; *d_atz (device pointer, owned by ctx, valid until
 * the next call) and *atz_len receive them. */
int atz_precompress_device(atz_ctx_t *ctx, const uint8_t *d_file, const uint8_t *h_file, uint64_t len,
                           const uint8_t **d_atz, uint64_t *atz_len, atz_stats_t *stats);

/* -r: rebuild the original from ATZ1 bytes. *out (atz_free). */
int atz_reconstruct(atz_ctx_t *ctx, const uint8_t *atz, uint64_t len, uint8_t **out, uint64_t *out_len);

/* -r with the ATZ1 bytes resident in HBM (d_atz, >= 4096 bytes of slack; h_atz: host copy for the
 * descriptors): *d_out (device, owned by ctx, valid until the next call) receives *out_len bytes. */
int atz_reconstruct_device(atz_ctx_t *ctx, const uint8_t *d_atz, const uint8_t *h_atz, uint64_t len,
                           const uint8_t **d_out, uint64_t *out_len);

/* One zlib-1.2.8-exact deflate (level 0..9, windowBits 9..15, memLevel 1..9, default strategy). */
int atz_deflate(atz_ctx_t *ctx, const uint8_t *in, uint64_t in_len, int clevel, int window, int memlevel,
                uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* Batch of independent one-shot deflates of ranges of a host buffer; params[i] = (clevel<<16)|(window<<8)|memlevel.
 * Output i is written at out + out_offs[i] (capacity out_caps[i]); out_lens[i] receives its length. */
int atz_deflate_batch(atz_ctx_t *ctx, const uint8_t *buf, uint64_t len, const uint64_t *offs, const uint64_t *lens,
                      const uint32_t *params, uint64_t n, uint8_t *out, const uint64_t *out_offs,
                      const uint64_t *out_caps, uint64_t *out_lens);

/* Batch of independent one-shot inflates of the given ranges of a host buffer (parity/debug):
 * status[i] in {0 end, 1 error, 2 need input}, consumed[i] = zlib total_in, produced[i] = total_out. */
int atz_inflate_batch(atz_ctx_t *ctx, const uint8_t *buf, uint64_t len, const uint64_t *offs,
                      const uint64_t *lens, uint64_t n, uint32_t *status, uint64_t *consumed, uint64_t *produced);

/* ---- Multi-GPU precompress of ONE file -----------------------------------------
 * One process, context and GPU per rank; every rank holds the whole file in HBM (d_file, >= 4096
 * bytes of slack) and a host copy.  Replaces the same Phase 1 + 3 + 4 as atz_precompress, split
 * where the ranks exchange data (the caller does the exchanges, e.g. torch.distributed over RCCL):
 *   1. atz_shard_scan: inflates the scan candidates of this rank's chunk range -> *blob (atz_free).
 *      Exchange: all-gather every rank's blob.
 *   2. atz_shard_sweep: replays the whole file's greedy scan (main.cpp:205-246) from all blobs, then
 *      sweeps (main.cpp:421-763) and writes the ATZ1 descriptors + payloads (writeStreamdesc,
 *      main.cpp:805-831) of the records its chunk range produced: *piece_len bytes, kept in the
 *      context.  *recomp_flags (atz_free) = one byte per such record.
 *      Exchange: all-gather piece lengths, recomp counts and flags; gather the pieces to rank 0.
 *   3. atz_shard_piece: device copy of this rank's piece to d_dst (rank 0: d_atz + 28 + the pieces
 *      of the ranks before it).
 *   4. rank 0, atz_shard_assemble: header + residue (writeATZfile, main.cpp:764-801) around the
 *      pieces in d_atz (capacity cap); flags = every rank's, in rank order.
 * The ATZ1 bytes are identical to atz_precompress of the same file on one GPU. */
int atz_shard_scan(atz_ctx_t *ctx, const uint8_t *d_file, const uint8_t *h_file, uint64_t len, int rank, int world,
                   uint8_t **blob, uint64_t *blob_len);
int atz_shard_sweep(atz_ctx_t *ctx, const uint8_t *d_file, const uint8_t *h_file, uint64_t len,
                    const uint8_t *const *blobs, const uint64_t *blob_lens, int world, uint64_t *piece_len,
                    uint8_t **recomp_flags, uint64_t *n_flags, uint64_t *n_recomp, atz_stats_t *stats);
int atz_shard_piece(atz_ctx_t *ctx, uint8_t *d_dst);
int atz_shard_assemble(atz_ctx_t *ctx, const uint8_t *d_file, uint64_t len, const uint8_t *recomp_flags,
                       uint64_t n_flags, uint64_t n_recomp, uint64_t pieces_len, uint8_t *d_atz, uint64_t cap,
                       uint64_t *atz_len);

/* zlib-1.2.8 deflate bound for the parameters (deflateBound, Z/deflate.c:566-621). */
uint64_t atz_deflate_bound(uint64_t n, int window, int memlevel);

#ifdef __cplusplus
}
#endif
#endif
