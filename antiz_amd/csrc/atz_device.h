// atz_device.h -- structures shared by the HIP kernels and the host orchestration (libatz_accel).
// All kernels target gfx950 (CDNA4): wave64, 160 KiB LDS per CU.
#pragma once
#include <stdint.h>

#ifndef ATZ_INF_CLOCKS
#define ATZ_INF_CLOCKS 0   // 1: per-job clocks and symbol counts in InfRes (diagnostics builds)
#endif

namespace atz {

// ---- inflate (k_inflate) -------------------------------------------------------------------
// One job = one zlib stream candidate: decode in[in_off, in_off+in_len) with zlib 1.2.8 acceptance
// semantics (ZlibWrapper.h:58-82 as driven by main.cpp:205-246; restated in oracle/ora_inflate.c).
struct InfJob {
  uint64_t in_off;   // byte offset into the input base buffer
  uint64_t in_len;   // bytes offered (the rest of the reference's chunk buffer)
  uint64_t out_off;  // byte offset into the output base buffer, or NO_OUT to discard output
  uint64_t out_cap;  // output capacity (ignored when NO_OUT)
};
static constexpr uint64_t NO_OUT = ~0ull;
static constexpr uint64_t ARENA_OUT = ~1ull;   // output into the arena: a slot of out_cap bytes claimed at first flush
static constexpr uint64_t ARENA_NONE = ~0ull;

enum : uint32_t { INF_END = 0, INF_ERROR = 1, INF_NEED = 2, INF_RETRY = 3 };   // RETRY: rerun with the 32 KiB ring

// InfRes.err bit 31: the first block is dynamic and codes matches, none of length 3-5 (a cost hint
// for the multi-GPU split); bits 27-30: the memLevel (1-9) whose lit_bufsize - 1 symbols the first
// block holds when more blocks follow, else 0 (the sweep builds whole match tables for that memLevel's
// trials); the low bits are the failing check's code
static constexpr uint32_t INF_HINT_NOSHORT = 1u << 31;
static constexpr uint32_t INF_HINT_MLEV_SHIFT = 27;

struct InfRes {
  uint32_t status;    // INF_*
  uint32_t err;       // diagnostic code of the failing check | INF_HINT_NOSHORT
  uint64_t consumed;  // zlib total_in at the stop
  uint64_t produced;  // zlib total_out at the stop
  uint64_t arena_off; // ARENA_OUT jobs: offset of the output slot (ARENA_NONE: none / incomplete)
#if ATZ_INF_CLOCKS   // diagnostics builds only (the scan copies one InfRes per candidate back)
  uint64_t cyc, nlit, nmatch;  // shader clocks, literals, matches
  uint64_t cyc_copy, cyc_flush; // clocks in match copies (incl. the stage write before) / ring flushes
  uint64_t nfar, cyc_far;       // matches whose source lies beyond the LDS ring (read from HBM), their clocks
  uint64_t nblk, cyc_hdr, nlong; // blocks, clocks in block headers + table builds, fast-loop codes > 6 bits
#endif
};

// ---- deflate trial (k_trial) ---------------------------------------------------------------
struct Trial {
  uint32_t stream;   // index into the stream table
  uint8_t clevel, window, memlevel, mode;  // mode bit0: full output needed (no early exits)
  uint64_t best_ident;  // best ident of this stream before this round (for the can't-beat exit)
  uint64_t out_off;     // scratch output offset for this trial (bytes)
  uint64_t out_cap;     // scratch output capacity (bytes)
  uint64_t sym_off;     // symbol-buffer offset (uint32 units), capacity 1 << (memlevel + 6)
  uint64_t chain_off;   // hash buckets of (stream, memlevel) (uint32 units, k_buckets); unused for level 0
  uint64_t r_off;       // match table of this trial (uint2 units, indexed by absolute position)
  uint64_t x_lim;       // match-table entries exist for positions < x_lim (else the trial stops: TR_NEED_R)
  // symbol replay: mode bit2 = this trial saves its whole symbol sequence at rp_syms (bit5: and its
  // match table at rp_tab); bit3 = this trial replays the rp_nsym symbols saved there (rp_flags bit1:
  // the last one is deflate_slow's end-of-input pending literal) instead of parsing -- with bit4 only
  // if its own match table equals the one saved at rp_tab (else it parses)
  uint64_t rp_syms;     // absolute device address (u32 symbols)
  uint64_t rp_tab;      // absolute device address (uint2 match-table entries)
  uint32_t rp_nsym, rp_flags;
  // speculative rounds: the trial's place among its stream's trials of the round (0: the first); a trial
  // whose stream an earlier one of the round has already stopped ends at once (SweepArgs::stopj)
  uint32_t spec_j, pad2_;
};

// ---- match tables (k_match) ----------------------------------------------------------------
// longest_match (Z/deflate.c:1148-1289) evaluated for every position p of a stream, one lane per
// position, for one (level, window) on the (stream, memLevel) chains:
//   slow levels: .x = result with the full chain budget, .y = with budget >> 2 (prev_length >= good)
//   fast levels: .x = full-budget result, .y = p - (lowest chain node the walk visited), hash slot
// result = len:9 | dist:15 (0 = no match longer than MIN_MATCH-1); see k_match for the packing.
struct MatchJob {
  uint64_t infl_off, n;   // stream bytes
  uint64_t chain_off;     // u32 units (hash buckets)
  uint64_t r_off;         // uint2 units
  uint64_t p0, p1;        // positions [p0, p1)
  uint32_t level, window;
  uint32_t fast, memlevel;
};

struct StreamDev {
  uint64_t orig_off;   // offset of the original compressed bytes in the file buffer
  uint64_t infl_off;   // offset of the inflated bytes in the inflated buffer
  uint64_t comp_len;   // C_s
  uint64_t infl_len;   // I_s
};

struct TrialRes {
  uint32_t state;       // TR_* below
  uint32_t flags;       // bit0 overlay hazard, bit1 shortcut applied
  uint64_t out_len;     // deflate total_out (when state == TR_FULL)
  uint64_t ident;       // positional equal bytes over min(out_len, C_s) (TR_FULL) / shortcut ident
  uint64_t symbols;     // diagnostic: symbols tallied
  uint64_t parsed;      // input positions consumed when the trial stopped
  uint64_t fallbacks;   // fast levels: steps that walked the chain because a skipped position was on it
                        // (low 32 bits), of which walks whose result changed the parse path (high 32)
  uint64_t cyc_total, cyc_tree, cyc_emit, blocks;   // diagnostics: shader clocks in the trial / tree
                                                    // construction / block emission, blocks flushed
  uint64_t cyc_heap, cyc_fallback;                  // tree heap steps (ATZ_STEP_CLOCKS) / fast-level exact walks
  uint64_t cyc_scan, cyc_send;                      // scan_tree / send_tree (ATZ_STEP_CLOCKS)
  uint64_t cyc_sec[4];                              // parse window phases: refill / steps / path / tally (ATZ_STEP_CLOCKS)
  uint32_t saved_syms;  // mode bit2: symbols saved at rp_syms
  uint32_t saved_flags; // bit0: the whole input was parsed (the sequence is complete), bit1: end-of-input
                        // literal, bit2: the trial replayed a saved sequence
  uint32_t reads_max;   // slow parses: (longest prev_length a lazy read improved) << 16 | longest length read
  uint32_t rt0, rt1;    // diagnostics: s_memrealtime (100 MHz) at the trial's start and end, low 32 bits
  uint32_t pad_;
};
enum : uint32_t {
  TR_FULL = 0,        // full output produced and compared: ident valid
  TR_SHORTCUT = 1,    // bailed at the shortcut (ident < shortcut_len - recomp_tresh)
  TR_SIZEDIFF = 2,    // |out - C_s| > sizediff_tresh: no compare
  TR_CANT_BEAT = 3,   // stopped: cannot exceed best_ident (result irrelevant to the sweep)
  TR_OVERFLOW = 4,    // output capacity exceeded (host treats as reference abort)
  TR_NEED_R = 5,      // parse reached x_lim: extend the match table and run the trial again
  TR_SKIPPED = 6,     // an earlier trial of its stream in the round stops the stream: never walked
};

struct SweepOpts {
  uint64_t recomp_tresh, sizediff_tresh, shortcut_len, mismatch_tol;
};

// Inclusive prefix sum over the 64 lanes of a wave (every lane active), on DPP: a Hillis-Steele scan
// inside each row of 16 lanes (row_shr 1, 2, 4, 8), then the rows' totals carried by row_bcast:15
// (into rows 1 and 3) and row_bcast:31 (into rows 2 and 3).  Six VALU adds; no LDS-crossbar
// permutes, unlike a __shfl_up ladder.  A lane whose DPP source is outside its row (or whose row is
// masked off) adds the `old` operand, 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15, rows 1 and 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31, rows 2 and 3
  return (uint32_t)x;
}

}  // namespace atz
