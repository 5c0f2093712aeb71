// atz_device.h -- structures shared by the HIP kernels and the host orchestration (libatz_accel).
// All kernels target gfx950 (CDNA4): wave64, 160 KiB LDS per CU.
#pragma once
#include <stdint.h>

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

enum : uint32_t { INF_END = 0, INF_ERROR = 1, INF_NEED = 2 };

struct InfRes {
  uint32_t status;    // INF_*
  uint32_t err;       // diagnostic code of the failing check
  uint64_t consumed;  // zlib total_in at the stop
  uint64_t produced;  // zlib total_out at the stop
};

// ---- deflate trial (k_trial) ---------------------------------------------------------------
struct Trial {
  uint32_t stream;   // index into the stream table
  uint8_t clevel, window, memlevel, mode;  // mode bit0: full output needed (no early exits)
  uint64_t best_ident;  // best ident of this stream before this round (for the can't-beat exit)
  uint64_t out_off;     // scratch output offset for this trial (bytes)
  uint64_t out_cap;     // scratch output capacity (bytes)
  uint64_t sym_off;     // symbol-buffer offset (uint32 units), capacity 1 << (memlevel + 6)
  uint64_t chain_off;   // chain-link table of (stream, memlevel) (uint16 units); unused for level 0
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
};
enum : uint32_t {
  TR_FULL = 0,        // full output produced and compared: ident valid
  TR_SHORTCUT = 1,    // bailed at the shortcut (ident < shortcut_len - recomp_tresh)
  TR_SIZEDIFF = 2,    // |out - C_s| > sizediff_tresh: no compare
  TR_CANT_BEAT = 3,   // stopped: cannot exceed best_ident (result irrelevant to the sweep)
  TR_OVERFLOW = 4,    // output capacity exceeded (host treats as reference abort)
};

struct SweepOpts {
  uint64_t recomp_tresh, sizediff_tresh, shortcut_len, mismatch_tol;
};

}  // namespace atz
