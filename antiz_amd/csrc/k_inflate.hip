// k_inflate.hip -- zlib stream scan + inflate on CDNA4 (gfx950).
//
// k_find_headers: one pass over the input in HBM marking the 24 RFC 1950 headers the reference
//   recognises (ZBuffSearcher::parseOffsetType, main.cpp:168-203); coalesced 16-byte loads,
//   ballot compaction.
// k_inflate: one wavefront per candidate/stream.  The Huffman decode is lane-parallel: lane l
//   (1..15) holds the canonical first-code/count/offset of code length l, a 15-bit bit-reversed
//   peek is tested by all 15 lanes at once and the lowest hitting lane (ballot + ffs) is the code
//   length -- no table build per block beyond a ballot-ranked symbol sort.  Match copies are spread
//   over lanes; the 32 KiB history ring lives in LDS; Adler-32 is folded into the lane-parallel
//   ring flush.  Input consumption (total_in) reproduces zlib 1.2.8 exactly: NEEDBITS semantics,
//   error positions, table quirks (see oracle/ora_inflate.c for the restatement it is tested against).
#include <hip/hip_runtime.h>
#include "atz_device.h"

namespace atz {

// History: the last RING output bytes live in an LDS ring per wave.  RING = 32 KiB holds the whole
// deflate window.  A smaller ring (INF_RING_SMALL) raises occupancy from 4 to 16 waves per CU (measured on C4: k_inflate 396 -> 154 ms; a 16 KiB ring at 8 waves/CU: 257 ms) (the
// decode is a serial per-stream chain, so resident waves are the throughput); a match reaching further
// back than the ring reads the bytes from the job's output in HBM, which the ring flushes every RING/2
// bytes.  A job that has no such output left (no slot, or its slot overflowed) stops with INF_RETRY and
// the host runs it again with the 32 KiB ring.
static constexpr uint32_t INF_RING_FULL = 32768;
#ifndef INF_RING_SMALL_BYTES
#define INF_RING_SMALL_BYTES 4096   // C4 k_inflate (A/B): 8 KiB x 4 waves 137 ms, 4 KiB x 5 126 ms, x 6 121 ms, x 8 127 ms
#endif
static constexpr uint32_t INF_RING_SMALL = INF_RING_SMALL_BYTES;
// >= 2 KiB: a far source (dist > RING) ends >= RING - 258 bytes back, which must lie below the
// unflushed tail (< RING/2 + 258 + 64 bytes), i.e. RING/2 >= 580
static_assert(INF_RING_SMALL >= 2048 && (INF_RING_SMALL & (INF_RING_SMALL - 1)) == 0,
              "small ring: a power of two >= 2 KiB");
#ifndef INF_SMALL_WAVES
#define INF_SMALL_WAVES 6   // waves per SIMD the small-ring decoder is register-bounded for (8 KiB ring: 3 -> 183 ms, 4 -> 154 ms)
#endif
#ifndef ATZ_INF_LITRUN
#define ATZ_INF_LITRUN 1   // fast path: short-code literals in their own tight loop
#endif
// The first block's symbol count (the sweep's memLevel hint): bytes produced - sum(length - 1) over its
// matches.  The decode loop is bound by the CU's one scalar unit, so the per-match add goes to the VALU:
// 2 (default) a v_add3 into a VGPR, 1 an SGPR add, 0 no hint.  C4 A/B (gpurun_out/pre_f, 2 runs each):
// k_inflate 75.6 ms with 2, 82.1 with 1, 75.9 with 0.
#ifndef ATZ_INF_MLS
#define ATZ_INF_MLS 2
#endif
#if ATZ_INF_MLS == 2
#define MLS_ADD(len) asm volatile("v_add3_u32 %0, %0, %1, -1" : "+v"(mls) : "s"(len))
#define MLS_GET() ((uint32_t)__builtin_amdgcn_readfirstlane((int)mls))
#elif ATZ_INF_MLS == 1
#define MLS_ADD(len) (mls += (len) - 1u)
#define MLS_GET() mls
#else
#define MLS_ADD(len) ((void)0)
#define MLS_GET() 0x7fffffffu
#endif
#ifndef ATZ_INF_CLOCKS
#define ATZ_INF_CLOCKS 0                       // 1: per-job clocks and symbol counts in InfRes
#endif

__device__ __constant__ uint16_t c_hdr_flg[6][4] = {
    {0x15, 0x53, 0x91, 0xcf}, {0x11, 0x4f, 0x8d, 0xcb}, {0x0d, 0x4b, 0x89, 0xc7},
    {0x09, 0x47, 0x85, 0xc3}, {0x05, 0x43, 0x81, 0xde}, {0x01, 0x5e, 0x9c, 0xda}};

__device__ inline int header_type(uint32_t b0, uint32_t b1) {
  // parseOffsetType: CMF in {0x28,0x38,...,0x78}, FLG one of four per CMF.
  if ((b0 & 0x0f) != 8) return -1;
  int ci = (int)(b0 >> 4) - 2;
  if (ci < 0 || ci > 5) return -1;
  int fl = (int)(b1 >> 6);
  return c_hdr_flg[ci][fl] == b1 ? ci * 4 + fl : -1;
}

// Marks every file position p in [0, n-1) whose byte pair is a recognised header.
// out[k] = p (unsorted); *count = number found (capped at cap).
__global__ __launch_bounds__(256) void k_find_headers(const uint8_t* __restrict__ f, uint64_t n,
                                                      uint64_t* __restrict__ out,
                                                      unsigned long long* __restrict__ count,
                                                      uint64_t cap) {
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 16;
  // the loop bound is wave-uniform so the shuffles below always see all 64 lanes
  for (uint64_t wb = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * 16; wb < n; wb += stride) {
    const uint64_t base = wb + lane * 16;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (base + 16 <= n) v = *reinterpret_cast<const uint4*>(f + base);
    uint8_t b[17];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t w = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
      b[4 * k + 0] = w & 0xff; b[4 * k + 1] = (w >> 8) & 0xff;
      b[4 * k + 2] = (w >> 16) & 0xff; b[4 * k + 3] = w >> 24;
    }
    if (base + 16 > n) {
      for (int k = 0; k < 16; k++) b[k] = base + k < n ? f[base + k] : 0;
    }
    b[16] = base + 16 < n ? f[base + 16] : 0;
    uint32_t hits = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (base + k + 1 < n && header_type(b[k], b[k + 1]) >= 0) hits |= 1u << k;
    }
    // wave compaction: one atomic per wave
    uint32_t c = __popc(hits);
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t t = __shfl_up(incl, d, 64);
      if ((int)lane >= d) incl += t;
    }
    uint32_t total = __shfl(incl, 63, 64);
    unsigned long long wbase = 0;
    if (lane == 63 && total) wbase = atomicAdd(count, (unsigned long long)total);
    wbase = __shfl(wbase, 63, 64);
    uint64_t o = wbase + (incl - c);
    while (hits) {
      int k = __ffs(hits) - 1;
      hits &= hits - 1;
      if (o < cap) out[o] = base + k;
      o++;
    }
  }
}

// Ordered variant: block b owns the contiguous segment [b*seg, (b+1)*seg) (seg a multiple of 4 KiB)
// and walks it 4 KiB at a time, lane l testing the 16 pairs starting at l*16.  count mode writes the
// block's total to cnt[b]; write mode writes (position << 5 | header type) in file order from base[b]
// on (block-wide exclusive prefix per step), so the list needs no sort.
__global__ __launch_bounds__(256) void k_headers_ordered(const uint8_t* __restrict__ f, uint64_t n, uint64_t seg,
                                                         uint32_t* __restrict__ cnt, const uint64_t* __restrict__ base,
                                                         uint64_t* __restrict__ out, int write) {
  __shared__ uint32_t wsum[4];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t s0 = (uint64_t)blockIdx.x * seg;
  const uint64_t s1 = s0 + seg < n ? s0 + seg : n;
  uint64_t o = write ? base[blockIdx.x] : 0;
  uint32_t total = 0;
  for (uint64_t sb = s0; sb < s1; sb += 4096) {
    const uint64_t p = sb + (uint64_t)t * 16;
    uint32_t hits = 0;
    if (p < s1) {
      uint8_t b[17];
      if (p + 17 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(f + p);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t x = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
          b[4 * k] = x & 0xff; b[4 * k + 1] = (x >> 8) & 0xff; b[4 * k + 2] = (x >> 16) & 0xff; b[4 * k + 3] = x >> 24;
        }
        b[16] = f[p + 16];
      } else {
        for (int k = 0; k < 17; k++) b[k] = p + k < n ? f[p + k] : 0;
      }
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (p + k < s1 && p + k + 1 < n && header_type(b[k], b[k + 1]) >= 0) hits |= 1u << k;
    }
    const uint32_t c = __popc(hits);
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if ((int)lane >= d) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t before = 0, step = 0;
    for (uint32_t k = 0; k < 4; k++) { const uint32_t v = wsum[k]; if (k < w) before += v; step += v; }
    __syncthreads();
    if (write) {
      uint64_t q = o + before + incl - c;
      while (hits) {
        const int k = __ffs(hits) - 1;
        hits &= hits - 1;
        out[q++] = ((p + k) << 5) | (uint64_t)header_type(f[p + k], f[p + k + 1]);   // position << 5 | type
      }
    }
    o += step;
    total += step;
  }
  if (!write && t == 0) cnt[blockIdx.x] = total;
}

// ---------------------------------------------------------------------------------------------
// k_inflate: one wavefront per job, everything inlined into the kernel so the decoder state stays
// in (wave-uniform) SGPRs -- a by-reference state struct crossing a call would live in scratch.
//
// Per-symbol cost is what bounds this kernel (a serial bit-stream decode per stream), so the hot
// loop is shaped for a short dependency chain and no memory wait per symbol:
//  * input: a 256-byte window, one dword per lane, loaded when the previous one is used up; the
//    refill reads one dword with readlane;
//  * decode: canonical compare in lanes 1..15 + ballot/ff1 + two readlanes (index, 16-bit packed
//    symbol table in 3 VGPRs);
//  * literals go to a VGPR stage (one byte per lane, v_cndmask on lane == count) that reaches the LDS history
//    ring with one ds_write_b8 per 64 literals or before a match copy;
//  * while >= 64 input bits remain every field of the next symbol is available, so the fast loop
//    drops zlib's per-field NEEDBITS checks; the last 8 bytes go through the careful path that
//    reproduces 1.2.8's exact total_in at NEED / ERROR (oracle/ora_inflate.c).

__device__ __forceinline__ uint32_t iuni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// RFC 1951 length / distance tables in closed form (an indexed __constant__ table compiles to a
// global load per symbol).
__device__ __forceinline__ uint32_t len_extra(uint32_t s) { return (s < 8 || s == 28) ? 0u : (s - 4) >> 2; }
__device__ __forceinline__ uint32_t len_base(uint32_t s) {
  return s < 8 ? 3 + s : s == 28 ? 258u : ((4 + (s & 3)) << len_extra(s)) + 3;
}
__device__ __forceinline__ uint32_t dist_extra(uint32_t d) { return d < 2 ? 0u : (d >> 1) - 1; }
__device__ __forceinline__ uint32_t dist_base(uint32_t d) { return d < 2 ? d + 1 : ((2 + (d & 1)) << dist_extra(d)) + 1; }
// code-length code order {16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15}, 5 bits each
__device__ __forceinline__ uint32_t cl_order(uint32_t i) {
  return (uint32_t)((i < 12 ? (0x22caa324e804a30ull >> (5 * i)) : (0x3c2e1346cull >> (5 * (i - 12)))) & 31);
}

// Fast-loop entries (the roots' lanes hold them for codes of <= 6 bits): literal/length symbol s
// with code length L is s << 4 | L for literals and end-of-block (< 4096 for literals), and a length
// symbol adds its extra-bit count (bits 13-15) and base - 3 (bits 16-23); a distance symbol d is
// L | extra bits << 4 | base << 8.  A length or distance is then base + one bit-field extract, and
// its code and extra bits are consumed together.
__device__ __forceinline__ uint32_t lit_entry(uint32_t s, uint32_t L) {
  if (s <= 256) return (s << 4) | L;
  const uint32_t ls = s - 257;
  return (s << 4) | L | (len_extra(ls) << 13) | ((len_base(ls) - 3u) << 16);
}
__device__ __forceinline__ uint32_t dist_entry(uint32_t d, uint32_t L) {
  return L | (dist_extra(d) << 4) | (dist_base(d) << 8);
}
__device__ __forceinline__ uint32_t ubfe(uint32_t x, uint32_t o, uint32_t w) { return __builtin_amdgcn_ubfe(x, o, w); }

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int d = 32; d >= 1; d >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, d, 64);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// Canonical Huffman code of one table: lane l (1..15) holds first-code / count of length l and
// ofm = offs - first (offs = index of its first symbol in the sorted list); the sorted symbols are
// 16-bit packed in three VGPRs (entry e in dword e >> 1: lane (e >> 1) & 63, register e >> 7) and
// read with v_readlane at a wave-uniform index -- no memory access per decoded symbol.
// root: lane p (the next 6 stream bits, first bit in bit 0) holds (symbol << 4) | length for the
// code of length <= 6 that p starts with, 0 if p starts a longer (or no) code.
struct Huff {
  uint32_t first, count, ofm;
  uint32_t t0, t1, t2;
  uint32_t root;
  int max;
  __device__ __forceinline__ uint32_t sym(uint32_t e) const {
    const uint32_t d = e >> 1;
    uint32_t w;
    if (d < 64) w = rl(t0, d);
    else if (d < 128) w = rl(t1, d - 64);
    else w = rl(t2, d - 128);
    return (w >> ((e & 1) << 4)) & 0xffffu;
  }
};

enum { R_OK = 0, R_ERR = -1, R_NEED = -2, R_RETRY = -3 };

template <uint32_t RING>
struct InfShared {
  uint8_t ring[RING];
  uint16_t lens[320];
  uint16_t sort[384];
};

template <uint32_t RING>
__global__ __launch_bounds__(64, RING == INF_RING_FULL ? 1 : INF_SMALL_WAVES) void k_inflate(const uint8_t* __restrict__ in_base, uint8_t* __restrict__ out_base,
                                               const InfJob* __restrict__ jobs, InfRes* __restrict__ res,
                                               uint32_t njobs, uint8_t* __restrict__ arena,
                                               unsigned long long* __restrict__ arena_used, uint64_t arena_cap) {
  constexpr uint32_t RMASK = RING - 1;
  constexpr uint32_t FLUSH_AT = RING / 2;   // unflushed bytes stay <= FLUSH_AT + 258 + 64 < RING
  // WIDE: in the small ring, stage writes and match copies store all 64 lanes (no exec mask); the
  // lanes past the data put garbage into the next < 64 slots, i.e. over bytes more than RING - 64
  // back.  Those are long flushed, and a match reaching them is a far copy (dist > RING - 64), read
  // from the HBM output.  The slots get their real bytes before anything reads them.  The 32 KiB
  // ring holds the whole window, so it keeps the masks.
  __shared__ InfShared<RING> sh;
  const int lane = threadIdx.x;
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const InfJob job = jobs[j];
  const uint64_t t_start = ATZ_INF_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t nlit = 0, nmatch = 0, cyc_copy = 0, cyc_flush = 0, nfar = 0, cyc_far = 0, nblk = 0, cyc_hdr = 0, nlong = 0;
  uint8_t* const ring = sh.ring;
  uint16_t* const lens = sh.lens;
  // per-lane shift of the canonical compare: lane l in 1..15 looks at the first l stream bits
  const uint32_t lsh = (lane >= 1 && lane <= 15) ? (uint32_t)(15 - lane) : 31u;
  const uint32_t laneb = (uint32_t)lane + 4033u;   // the literal run: lane nst is the one where nb + 1 == laneb
  // RFC 1951 base / extra bits per length symbol (lane = symbol - 257) and distance symbol
  const uint32_t lentab = lane < 29 ? (len_base((uint32_t)lane) << 4) | len_extra((uint32_t)lane) : 0u;
  const uint32_t disttab = lane < 30 ? (dist_base((uint32_t)lane) << 4) | dist_extra((uint32_t)lane) : 0u;

  // ---- bit reader: 256-byte windows of the job's bytes, one dword per lane: `cur` is being read,
  // `nxt` (the following 256 bytes) is in flight
  const uint8_t* p0 = in_base + job.in_off;
  const uintptr_t ap = reinterpret_cast<uintptr_t>(p0);
  const uint64_t skip = ap & 3;
  // global address space explicitly: a flat load would also count in lgkmcnt and make every LDS
  // wait drain the input loads
  const __attribute__((address_space(1))) uint32_t* const abase =
      (const __attribute__((address_space(1))) uint32_t*)(ap - skip);
  const uint64_t skip_bits = 8 * skip;
  const uint64_t limit = 8 * (skip + job.in_len);   // bit limit (aligned coordinates)
  uint64_t pos = 0, bb = 0, wcur = 0;   // wcur: dword index of the window in `cur`
  uint32_t bc = 0, rk = 0;
  uint32_t cur = 0;
  // Bits past `limit` are never consumed (every consumption is preceded by a bounds check or by
  // the fast loop's 64-bit margin), and a canonical code found within the available bits is the
  // true code whatever follows (prefix-free), so windows are loaded unmasked.  The input buffers
  // carry >= 4 KiB of slack for the <= 256-byte over-read.
  // One dword into the bit buffer (bc <= 32 on entry).  The next 256-byte window is loaded when
  // the current one is used up: one load latency per 256 input bytes (~2 % of the decode) and no
  // in-flight load crossing the loop's register copies (a copy of an in-flight load waits for it).
  auto refill1 = [&]() __attribute__((always_inline)) {
    const uint32_t w = rl(cur, rk);
    bb |= (uint64_t)w << bc;
    bc += 32;
    if (++rk == 64) {
      wcur += 64;
      cur = abase[wcur + lane];
      rk = 0;
    }
  };
  auto refill = [&]() __attribute__((always_inline)) { while (bc <= 32) refill1(); };
  auto seek = [&](uint64_t apos) __attribute__((always_inline)) {
    const uint64_t dw = apos >> 5;
    wcur = dw & ~63ull;
    cur = abase[wcur + lane];
    rk = (uint32_t)(dw & 63);
    bb = 0; bc = 0;
    pos = apos & ~31ull;
    refill1();
    const uint32_t d = (uint32_t)(apos & 31);
    bb >>= d; bc -= d; pos += d;
    refill();
  };
  auto peek = [&](uint32_t k) __attribute__((always_inline)) -> uint32_t { return (uint32_t)(bb & ((k >= 32) ? 0xffffffffull : ((1ull << k) - 1))); };
  auto drop = [&](uint32_t k) __attribute__((always_inline)) { bb >>= k; bc -= k; pos += k; if (bc <= 32) refill(); };
  auto has = [&](uint64_t k) __attribute__((always_inline)) -> bool { return pos + k <= limit; };

  // ---- output: LDS history ring, flushed to HBM (if kept) and folded into Adler-32 every 16 KiB
  // output: to out_base + out_off, nowhere (NO_OUT), or to an arena slot of out_cap bytes claimed
  // at the first flush (ARENA_OUT: scan candidates keep their output if they turn out to be streams)
  const bool to_arena = job.out_off == ARENA_OUT;
  uint8_t* out = (job.out_off == NO_OUT || to_arena) ? nullptr : out_base + job.out_off;
  uint64_t arena_off = ARENA_NONE;
  bool arena_tried = false;
  const uint64_t out_cap = job.out_cap;
  uint64_t prod = 0, flushed = 0;   // prod: bytes in the ring (the stage's nst literals follow)
  uint32_t ad_a = 1, ad_b = 0;
  int overflow = 0;
  // literal stage: output byte prod + l in lane l (l < nst)
  // literal stage: lane l holds (output byte prod + l) << 4 in its low 12 bits (l < nst); the root
  // entries go in unshifted (symbol << 4 | length), so staging a literal is VALU work only
  uint32_t stg = 0, nst = 0;
  auto flush = [&](bool final) __attribute__((always_inline)) {
    const uint64_t n = prod - flushed;
    if (!n) return;
    const uint64_t tf0 = ATZ_INF_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
    if (to_arena && !arena_tried) {
      arena_tried = true;
      const uint64_t want = final ? ((prod + 255) & ~255ull) : out_cap;
      unsigned long long o = 0;
      if (lane == 0) o = atomicAdd(arena_used, (unsigned long long)want);
      // broadcast with readfirstlane, not a shuffle: the slot (and `out`) must be provably
      // wave-uniform, or every branch on `out` -- the far-copy check in the hot loop -- makes the
      // decoder state divergent (VGPRs + exec-mask bookkeeping on every symbol)
      o = ((uint64_t)iuni((uint32_t)(o >> 32)) << 32) | iuni((uint32_t)o);
      if (o + want <= arena_cap && (final || prod <= out_cap)) { arena_off = o; out = arena + o; }
    }
    uint64_t S = 0, W = 0;
#pragma unroll 4
    for (uint64_t k = lane; k < n; k += 64) {
      const uint32_t x = ring[(flushed + k) & RMASK];
      S += x;
      W += (n - k) * x;
      if (out && flushed + k < out_cap) out[flushed + k] = (uint8_t)x;
    }
    S = wave_sum_u64(S);
    W = wave_sum_u64(W);
    uint64_t a = ad_a, b = ad_b;
    b = (b + (n % 65521) * a + W) % 65521;
    a = (a + S) % 65521;
    ad_a = iuni((uint32_t)a); ad_b = iuni((uint32_t)b);
    if (out && prod > out_cap) {
      overflow = to_arena ? 0 : 1;   // an arena slot that overflows is just dropped
      if (to_arena) { arena_off = ARENA_NONE; out = nullptr; }
    }
    flushed = prod;
    if (ATZ_INF_CLOCKS) cyc_flush += __builtin_amdgcn_s_memtime() - tf0;
  };
  auto stage_flush = [&]() __attribute__((always_inline)) {
    if (nst) {
      if (RING < INF_RING_FULL || (uint32_t)lane < nst) ring[(prod + lane) & RMASK] = (uint8_t)(stg >> 4);   // (see WIDE)
      prod += nst;
      nst = 0;
      if (prod - flushed >= FLUSH_AT) flush(false);
    }
  };
  auto put_lit = [&](uint32_t s) __attribute__((always_inline)) {
    stg = ((uint32_t)lane == nst) ? (s << 4) : stg;
    nst++;
    if (ATZ_INF_CLOCKS) nlit++;
    if (nst == 64) stage_flush();
  };
  // copy `len` bytes from `dist` back (dist <= prod) to prod; the stage must be empty.  False: the
  // source is beyond the ring and no HBM copy of it exists (R_RETRY).  The caller advances prod and
  // checks the flush threshold.
  auto copy_at = [&](uint32_t len, uint32_t dist) __attribute__((always_inline)) -> bool {
    if (ATZ_INF_CLOCKS) nmatch++;
    if (RING < INF_RING_FULL && dist > RING - 64) {
      // Far source: [prod - dist, prod - dist + len) ends at least RING - 258 bytes back, so it was
      // flushed (unflushed bytes < RING/2 + 322) -- if this job's output still exists.  dist > RING
      // > len, so the copy does not overlap itself.  The flush's stores are drained first and the
      // loads are agent-coherent (L1 bypassed: a line may have been cached before it was complete).
      const uint64_t src = prod - dist;
      const uint64_t valid = flushed < out_cap ? flushed : out_cap;
      if (!out || src + len > valid) return false;
      const uint64_t tf0 = ATZ_INF_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
      __builtin_amdgcn_s_waitcnt(0);
      for (uint32_t i0 = 0; i0 < len; i0 += 64) {
        const uint32_t i = i0 + lane;
        if (i < len) {
          const uint8_t v = __hip_atomic_load(out + src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ring[(prod + i) & RMASK] = v;
        }
      }
      if (ATZ_INF_CLOCKS) { nfar++; cyc_far += __builtin_amdgcn_s_memtime() - tf0; }
    } else {
      // overlapping (dist < len): the source repeats with period dist.  i % dist in float: i < 320
      // and dist <= 258, so (i + 0.5) / dist stays >= 0.5 / 258 away from an integer, far above
      // the error of v_rcp_f32 (checked exhaustively, with the reciprocal 2 ulp off either way)
      const uint32_t base = (uint32_t)prod - dist;
      const bool ovl = dist < len;
      for (uint32_t i0 = 0; i0 < len; i0 += 64) {
        const uint32_t i = i0 + lane;
        uint32_t k = i;
        if (ovl) k = i - (uint32_t)(((float)i + 0.5f) * __builtin_amdgcn_rcpf((float)dist)) * dist;
        uint8_t v = 0;
        if (RING < INF_RING_FULL || i < len) v = ring[(base + k) & RMASK];
        __builtin_amdgcn_wave_barrier();
        if (RING < INF_RING_FULL || i < len) ring[((uint32_t)prod + i) & RMASK] = v;   // (see WIDE)
      }
    }
    return true;
  };
  auto copy = [&](uint32_t len, uint32_t dist) __attribute__((always_inline)) -> bool {
    if (!copy_at(len, dist)) return false;
    prod += len;
    if (prod - flushed >= FLUSH_AT) flush(false);
    return true;
  };

  // inflate_table acceptance (Z/inftrees.c:32-141); type 0 CODES, 1 LENS, 2 DISTS. Returns 0 / -1.
  // pre: lane l (1..15) of `given` holds the number of length-l codes when have_cnt (the dynamic
  // header counts them while decoding the lengths), else the count pass runs here
  auto build = [&](Huff& h, const uint16_t* ln, int n, int type, bool have_cnt, uint32_t given) __attribute__((always_inline)) -> int {
    uint32_t cnt = given;
    if (!have_cnt) {
      cnt = 0;
      for (int g = 0; g < n; g += 64) {
        const int i = g + lane;
        const uint32_t len = i < n ? ln[i] : 0;
        for (int l = 1; l <= 15; l++) {
          const uint32_t c = __popcll(__ballot(len == (uint32_t)l));
          if (lane == l) cnt += c;
        }
      }
    }
    // zlib's sequential pass over the lengths (inftrees.c: left, offs[], next code), lane-parallel:
    // with w_l = count_l << (15 - l), the first code of length l is (sum over i < l of w_i) >> (15 - l),
    // and "left" goes negative at some length exactly when the Kraft sum W = sum of w_l exceeds 2^15
    // (the partial sums only grow); the code is incomplete when W < 2^15.  Two DPP scans.
    const uint32_t cl = (lane >= 1 && lane <= 15) ? cnt : 0u;
    const uint64_t nz = __ballot(cl != 0);
    const int max = nz ? 63 - __clzll((long long)nz) : 0;
    const uint32_t wl = cl << ((15 - lane) & 15);
    const uint32_t wi = wave_incl_scan(wl), ci = wave_incl_scan(cl);
    const uint32_t W = rl(wi, 15);
    const uint32_t my_first = (lane >= 1 && lane <= 15) ? (wi - wl) >> (15 - lane) : 0u;
    const uint32_t my_offs = ci - cl;
    h.max = max;
    h.root = 0;
    if (max == 0) { h.count = 0; h.first = 0; h.ofm = 0; return 0; }
    if (W > 32768u) return -1;
    if (W < 32768u && (type == 0 || max != 1)) return -1;
    h.first = my_first; h.count = (lane >= 1 && lane <= 15) ? cnt : 0; h.ofm = my_offs - my_first;
    // ballot-ranked counting sort into LDS, then into the packed VGPR table
    uint32_t run = my_offs;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint64_t present = __ballot(lane >= 1 && lane <= 15 && cnt != 0);   // lengths that occur
    for (int g = 0; g < n; g += 64) {
      const int i = g + lane;
      const uint32_t len = i < n ? ln[i] : 0;
      for (uint64_t pm = present; pm; pm &= pm - 1) {
        const int l = __ffsll((unsigned long long)pm) - 1;
        const uint64_t m = __ballot(len == (uint32_t)l);
        if (!m) continue;
        const uint32_t base = rl(run, l);
        if (len == (uint32_t)l) sh.sort[base + __popcll(m & lt)] = (uint16_t)i;
        if (lane == l) run += __popcll(m);
      }
    }
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sh.sort);
    h.t0 = sw[lane];
    h.t1 = n > 128 ? sw[64 + lane] : 0;
    h.t2 = n > 256 ? sw[128 + lane] : 0;
    // 6-bit root: lane p resolves the code of length <= 6 its stream bits start with, as a fast-loop
    // entry (LENS, DISTS; the fixed distance symbols 30-31 stay 0, so the fast loop hands them to
    // the careful path) or symbol << 4 | length (CODES)
    {
      const uint32_t rp = __builtin_bitreverse32((uint32_t)lane) >> 26;
      uint32_t sv = 0, lf = 0;
      const int lm = max < 6 ? max : 6;
      for (int l = 1; l <= lm; l++) {
        const uint32_t f = rl(h.first, l), k = rl(h.count, l), o = rl(h.ofm, l);
        const uint32_t c = rp >> (6 - l);
        if (lf == 0 && (c - f) < k) { sv = sh.sort[o + c]; lf = (uint32_t)l; }
      }
      uint32_t e = 0;
      if (lf) e = type == 1 ? lit_entry(sv, lf) : type == 2 ? (sv < 30 ? dist_entry(sv, lf) : 0u) : ((sv << 4) | lf);
      h.root = e;
    }
    return 0;
  };

  // Careful decode: >= 0 symbol, -1 invalid code, -2 need more input.  need = the bit position
  // zlib would have required when it stops here.
  auto decode = [&](const Huff& h, bool cl_quirk, uint64_t& need) __attribute__((always_inline)) -> int {
    if (h.max == 0) {
      need = pos + 1;
      if (!has(1)) return -2;
      drop(1);
      return cl_quirk ? 0 : -1;
    }
    const uint32_t v = __builtin_bitreverse32((uint32_t)bb) >> 17;   // first stream bit at bit 14
    const uint32_t c = v >> lsh;
    const uint64_t m = __ballot((c - h.first) < h.count);
    if (!m) {  // only incomplete codes have unused patterns: zlib's invalid entry has 1 bit
      need = pos + 1;
      if (!has(1)) return -2;
      drop(1);
      return -1;
    }
    const uint32_t L = (uint32_t)__ffsll((unsigned long long)m) - 1;
    need = pos + L;
    if (!has(L)) return -2;
    const uint32_t idx = rl(c + h.ofm, L);
    drop(L);
    return (int)h.sym(idx);
  };

  uint64_t errneed = 0;
  uint32_t errcode = 0;
  uint32_t hint = 0;   // INF_HINT_NOSHORT (see the dynamic header below) | INF_HINT_MLEV
  // sum of (length - 1) over the block's matches: symbols = bytes - mls.  ATZ_INF_MLS 2 keeps it in a
  // VGPR (one VALU add per match; the decode loop is bound by the CU's scalar issue), 1 in an SGPR
  uint32_t mls = 0;
#define NEEDB(k) do { if (!has(k)) return R_NEED; } while (0)
#define FAIL(code, needpos) do { errneed = (needpos); errcode = (code); return R_ERR; } while (0)

  auto codes = [&](const Huff& lh, const Huff& dh) __attribute__((always_inline)) -> int {
    uint64_t need;
    bool redo = false;   // the careful path decodes the next symbol (the fast loop gave it back)
    for (;;) {
      if (!redo && pos + 64 <= limit) {
        // ---- fast loop: while >= 64 input bits remain at a symbol's start every field of it is
        // buffered-or-refillable (<= 48 bits), so no NEEDBITS checks.  Bits consumed here are
        // counted in `used` (32-bit) and folded into pos when the loop leaves.
        const uint64_t pos0 = pos;
        const uint64_t rr64 = limit - 64 - pos;
        const uint32_t rem = rr64 > 0x7fffffffull ? 0x7fffffffu : (uint32_t)rr64;
        uint32_t used = 0;
        int rc = 1;   // 1: careful path next, R_OK / R_RETRY: return
        while (used <= rem) {
          if (bc <= 32) refill1();
          uint32_t e = rl(lh.root, (uint32_t)bb & 63);
#if ATZ_INF_LITRUN
          // literal run: root-table literals (codes of <= 6 bits: e in [1, 4095]) go straight into
          // the stage in a loop with one back edge; anything else takes the general path below
          // The end-of-fast-path test (used <= rem: >= 64 input bits left) is made at each refill
          // only: after a passing test the buffer holds bits up to at most 64 past it, all before
          // the input limit, and the run decodes only buffered bits (bc > 32 at every lookup).
          // The run never flushes: it leaves when the stage is full (the flush, a large inlined
          // block, stays outside the loop, so the loop body is straight-line scalar code).
          if (e - 1u < 4095u) {
            // One back edge and a 4-instruction exit test: nb = nst + 4032 (compared with
            // laneb, it reaches 4096 when the stage is full) and the end-of-fast-region stop
            // (tested at refills only: after a passing test every buffered bit lies before the input
            // limit) sets bit 16, so "short literal, stage not full, no stop" is max(e - 1, nb) < 4096
            // (a root entry has a length >= 1, so e - 1 < 4096 means e in [1, 4095]).  ub = used + bc
            // changes only at refills.
            uint32_t nb = nst + 4032u, ub = used + bc;
            do {
              const uint32_t L = e & 15;
              bb >>= L; bc -= L;
              nb++;
              stg = (laneb == nb) ? e : stg;
              if (ATZ_INF_CLOCKS) nlit++;
              if (bc <= 32) {
                if (ub - bc > rem) nb |= 0x10000u;
                refill1();
                ub += 32;
              }
              e = rl(lh.root, (uint32_t)bb & 63);
            } while (((e - 1u) > nb ? (e - 1u) : nb) < 4096u);
            nst = (nb & 0xffffu) - 4032u;
            used = ub - bc;
            if (nst == 64) stage_flush();
            if (used > rem) break;   // rc == 1: the careful path resumes at this symbol
            if (e - 1u < 4095u) continue;   // the stage was full: back to the run (bc > 32 here)
          }
#endif
          // Anything unusual -- an invalid code, a fixed-code length/distance symbol 286-287 / 30-31,
          // a distance beyond the output -- leaves the fast loop at the symbol's start (`sym0`) and
          // is decoded once more by the careful path, which reports it with zlib's exact error
          // position.  So the fast loop has three exits: careful path next, end of block, retry.
          const uint32_t sym0 = used;
          if (e == 0) {   // code longer than 6 bits (or invalid): canonical compare
            if (ATZ_INF_CLOCKS) nlong++;
            const uint32_t v = __builtin_bitreverse32((uint32_t)bb) >> 17;
            const uint32_t c = v >> lsh;
            const uint64_t m = __ballot((c - lh.first) < lh.count);
            if (!m) { redo = true; break; }
            const uint32_t Lc = (uint32_t)__ffsll((unsigned long long)m) - 1;
            const uint32_t sc = lh.sym(rl(c + lh.ofm, Lc));
            if (sc >= 286) { redo = true; break; }   // fixed codes 286/287
            e = lit_entry(sc, Lc);
          }
          const uint32_t L = e & 15;
          if (e < 4096u) { bb >>= L; bc -= L; used += L; put_lit(e >> 4); continue; }   // (the stage is never left full)
          if (((e >> 4) & 511u) == 256u) { bb >>= L; bc -= L; used += L; rc = R_OK; break; }
          const uint32_t le = (e >> 13) & 7u;
          const uint32_t len = (e >> 16) + 3u + ubfe((uint32_t)bb, L, le);
          bb >>= L + le; bc -= L + le; used += L + le;
          if (bc <= 32) refill1();
          uint32_t d = rl(dh.root, (uint32_t)bb & 63);
          if (d == 0) {   // (an empty distance code has an all-zero root and no lengths: m == 0)
            const uint32_t v = __builtin_bitreverse32((uint32_t)bb) >> 17;
            const uint32_t c = v >> lsh;
            const uint64_t m = __ballot((c - dh.first) < dh.count);
            if (!m) { used = sym0; redo = true; break; }
            const uint32_t Lc = (uint32_t)__ffsll((unsigned long long)m) - 1;
            const uint32_t dc = dh.sym(rl(c + dh.ofm, Lc));
            if (dc >= 30) { used = sym0; redo = true; break; }   // fixed distance 30/31
            d = dist_entry(dc, Lc);
          }
          const uint32_t L2 = d & 15, de = (d >> 4) & 15u;
          const uint32_t dist = (d >> 8) + ubfe((uint32_t)bb, L2, de);
          bb >>= L2 + de; bc -= L2 + de; used += L2 + de;
          const uint64_t tc0 = ATZ_INF_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
          // the stage goes to the ring, the match is copied after it, one flush test for both
          // (unflushed bytes stay < FLUSH_AT + 64 + 258)
          if (nst) {
            if (RING < INF_RING_FULL || (uint32_t)lane < nst) ring[(prod + lane) & RMASK] = (uint8_t)(stg >> 4);
            prod += nst;
            nst = 0;
          }
          if ((uint64_t)dist > prod) { used = sym0; redo = true; break; }   // too far back
          MLS_ADD(len);
          if (!copy_at(len, dist)) { rc = R_RETRY; break; }
          prod += len;
          if (prod - flushed >= FLUSH_AT) flush(false);
          if (ATZ_INF_CLOCKS) cyc_copy += __builtin_amdgcn_s_memtime() - tc0;
        }
        pos = pos0 + used;
        if (redo) seek(pos);   // the bit buffer is past the symbol the careful path decodes again
        else if (bc <= 32) refill();
        if (rc != 1) return rc;
        continue;
      }
      // ---- careful path (the last 8 input bytes, and one symbol the fast loop gave back):
      // zlib's NEEDBITS points and error positions exactly
      redo = false;
      if (bc <= 32) refill();
      int sym = decode(lh, false, need);
      if (sym == -2) return R_NEED;
      if (sym == -1) FAIL(10, need);
      if (sym < 256) { put_lit((uint32_t)sym); continue; }
      if (sym == 256) return R_OK;
      sym -= 257;
      if (sym >= 29) FAIL(11, need);                       // fixed codes 286/287
      const uint32_t le = len_extra((uint32_t)sym);
      NEEDB(le);
      const uint32_t len = len_base((uint32_t)sym) + peek(le);
      drop(le);
      const int ds = decode(dh, false, need);
      if (ds == -2) return R_NEED;
      if (ds == -1) FAIL(12, need);
      if (ds >= 30) FAIL(13, need);                        // fixed distance 30/31
      const uint32_t de = dist_extra((uint32_t)ds);
      NEEDB(de);
      const uint32_t dist = dist_base((uint32_t)ds) + peek(de);
      drop(de);
      stage_flush();
      if ((uint64_t)dist > prod) FAIL(14, pos);            // invalid distance too far back
      MLS_ADD(len);
      if (!copy(len, dist)) return R_RETRY;
    }
  };

  auto body = [&]() __attribute__((always_inline)) -> int {
    // HEAD (Z/inflate.c:640-685): wrap=1, wbits=15
    NEEDB(16);
    const uint32_t cmf = peek(8);
    const uint32_t flg = (peek(16) >> 8) & 0xff;
    if (((cmf << 8) + flg) % 31) FAIL(1, pos + 16);
    if ((cmf & 15) != 8) FAIL(2, pos + 16);
    if ((cmf >> 4) + 8 > 15) FAIL(3, pos + 16);
    drop(16);
    if (flg & 0x20) { NEEDB(32); FAIL(4, pos + 32); }      // preset dictionary: not a stream end
    int last;
    Huff lh, dh;
    uint32_t nblk_seen = 0;
    do {
      const uint64_t th0 = ATZ_INF_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
      if (ATZ_INF_CLOCKS) nblk++;
      NEEDB(3);
      last = (int)peek(1);
      const uint32_t type = (peek(3) >> 1) & 3;
      drop(3);
      if (type == 0) {                                      // STORED
        const uint32_t al = (uint32_t)((8 - (pos & 7)) & 7);
        drop(al);
        NEEDB(32);
        const uint32_t len = peek(16);
        const uint32_t nlen = (peek(32) >> 16) & 0xffff;
        if (len != (~nlen & 0xffff)) FAIL(5, pos + 32);
        drop(32);
        stage_flush();
        // copy `len` bytes straight from the input (byte aligned now)
        const uint64_t avail = (limit - pos) >> 3;
        const uint64_t take = len < avail ? len : avail;
        const __attribute__((address_space(1))) uint8_t* src =
            (const __attribute__((address_space(1))) uint8_t*)(ap - skip) + (pos >> 3);
        uint64_t done = 0;
        while (done < take) {
          uint64_t step = take - done;
          if (step > FLUSH_AT) step = FLUSH_AT;   // after a flush (which empties the ring) a step always fits
          const uint64_t room = RING - (prod - flushed);
          if (step > room) { flush(false); continue; }
          for (uint64_t k = lane; k < step; k += 64) ring[(prod + k) & RMASK] = src[done + k];
          prod += step;
          done += step;
          if (prod - flushed >= FLUSH_AT) flush(false);
        }
        seek(pos + 8 * take);
        if (take < len) return R_NEED;
      } else if (type == 1) {                               // FIXED
        for (int i = lane; i < 288; i += 64) lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
        build(lh, lens, 288, 1, false, 0);
        for (int i = lane; i < 32; i += 64) lens[i] = 5;
        build(dh, lens, 32, 2, false, 0);
      } else if (type == 2) {                               // DYNAMIC (Z/inflate.c:908-1013)
        NEEDB(14);
        const uint32_t nlen = peek(5) + 257;
        const uint32_t ndist = ((peek(10) >> 5) & 31) + 1;
        const uint32_t ncode = ((peek(14) >> 10) & 15) + 4;
        if (nlen > 286 || ndist > 30) FAIL(6, pos + 14);
        drop(14);
        for (int i = lane; i < 320; i += 64) lens[i] = 0;
        for (uint32_t i = 0; i < ncode; i++) {
          NEEDB(3);
          const uint32_t v = peek(3);
          drop(3);
          if (lane == 0) lens[cl_order(i)] = (uint16_t)v;
        }
        Huff chh;
        if (build(chh, lens, 19, 0, false, 0)) FAIL(7, pos);
        uint32_t have = 0;
        const uint32_t total = nlen + ndist;
        uint64_t need;
        for (int i = lane; i < 320; i += 64) lens[i] = 0;
        uint32_t prevlen = 0;
        // per-length counts for the two builds, kept while the lengths are decoded: lane l counts
        // the literal/length codes of length l, lane 16 + l the distance codes (a run may cross
        // from one table into the other)
        uint32_t lcnt = 0;
        auto count = [&](uint32_t len, uint32_t n) __attribute__((always_inline)) {
          if (len == 0) return;
          const uint32_t nl = have < nlen ? (n < nlen - have ? n : nlen - have) : 0u;
          lcnt += ((uint32_t)lane == len) ? nl : 0u;
          lcnt += ((uint32_t)lane == len + 16) ? n - nl : 0u;
        };
        // Fast loop: the whole length sequence lies before the input limit (at most 7 + 7 bits per
        // length), so no NEEDBITS tests.  Codes of <= 6 bits come from the root lane; a 7-bit code,
        // an invalid pattern or an invalid repeat leaves the rest to the careful loop below, which
        // reports errors at zlib's exact positions.
        if (pos + 14ull * total + 64 <= limit) {
          while (have < total) {
            if (bc <= 32) refill1();
            const uint32_t e = rl(chh.root, (uint32_t)bb & 63);
            if (e == 0) break;
            const uint32_t L = e & 15, sym = e >> 4;
            if (sym < 16) {
              bb >>= L; bc -= L; pos += L;
              if (lane == 0) lens[have] = (uint16_t)sym;
              count(sym, 1);
              prevlen = sym;
              have++;
              continue;
            }
            const uint32_t eb = sym == 16 ? 2u : sym == 17 ? 3u : 7u;
            const uint32_t x = (uint32_t)(bb >> L) & ((1u << eb) - 1);
            const uint32_t copyn = (sym == 18 ? 11u : 3u) + x;
            if ((sym == 16 && have == 0) || have + copyn > total) break;
            const uint32_t len = sym == 16 ? prevlen : 0u;
            bb >>= L + eb; bc -= L + eb; pos += L + eb;
            for (uint32_t k = lane; k < copyn; k += 64) lens[have + k] = (uint16_t)len;
            count(len, copyn);
            prevlen = len;
            have += copyn;
          }
        }
        while (have < total) {
          const int sym = decode(chh, true, need);
          if (sym == -2) return R_NEED;
          if (sym < 16) { if (lane == 0) lens[have] = (uint16_t)sym; count((uint32_t)sym, 1); prevlen = (uint32_t)sym; have++; continue; }
          uint32_t copyn, len = 0, eb;
          if (sym == 16) eb = 2; else if (sym == 17) eb = 3; else eb = 7;
          NEEDB(eb);
          if (sym == 16) {
            if (have == 0) FAIL(8, pos + eb);
            len = prevlen;
            copyn = 3 + peek(2);
          } else if (sym == 17) {
            copyn = 3 + peek(3);
          } else {
            copyn = 11 + peek(7);
          }
          drop(eb);
          if (have + copyn > total) FAIL(8, pos);
          for (uint32_t k = lane; k < copyn; k += 64) lens[have + k] = (uint16_t)len;
          count(len, copyn);
          prevlen = len;
          have += copyn;
        }
        if (iuni(lens[256]) == 0) FAIL(9, pos);
        if (nblk_seen == 0) {
          // Cost hint for the multi-GPU split, part of no output: the first block codes matches, but
          // none of length 3-5 (symbols 257-259).  zlib's Z_FILTERED strategy drops those
          // (Z/deflate.c:1774-1782), and no entry of the reference's trial lists uses it, so such a
          // stream usually runs its whole list.
          const uint32_t v = (uint32_t)lane < nlen - 257u ? (uint32_t)lens[257 + lane] : 0u;
          const uint64_t m = __ballot(v != 0);
          if (m != 0 && (m & 7u) == 0) hint = INF_HINT_NOSHORT;
        }
        const uint32_t dcnt = __shfl_down(lcnt, 16, 64);   // lane l: distance codes of length l
        if (build(lh, lens, (int)nlen, 1, true, lcnt)) FAIL(9, pos);
        if (build(dh, lens + nlen, (int)ndist, 2, true, dcnt)) FAIL(9, pos);
      } else {
        FAIL(15, pos);                                      // invalid block type
      }
      if (ATZ_INF_CLOCKS) cyc_hdr += __builtin_amdgcn_s_memtime() - th0;
      nblk_seen++;
      if (type != 0) {   // one (inlined) decode loop for fixed and dynamic blocks
        const uint64_t b0 = prod + nst;
        mls = 0;
        const int rr = codes(lh, dh);
        if (rr != R_OK) return rr;
        if (nblk_seen == 1 && !last) {
          // Sweep hint, part of no output: zlib flushes a block when its symbol buffer is full
          // (_tr_tally, Z/trees.c:1050, Z/deflate.h:328-338), so a first block that is not the last holds exactly
          // lit_bufsize - 1 = 2^(memLevel + 6) - 1 symbols
          const uint64_t syms = prod + nst - b0 - MLS_GET();
          if (syms >= 127 && syms <= 32767 && ((syms + 1) & syms) == 0)
            hint |= (uint32_t)(__builtin_ctzll(syms + 1) - 6) << INF_HINT_MLEV_SHIFT;
        }
      }
    } while (!last);
    // CHECK (Z/inflate.c:1174-1195)
    const uint32_t al = (uint32_t)((8 - (pos & 7)) & 7);
    drop(al);
    NEEDB(32);
    const uint32_t t = peek(32);
    const uint32_t want = ((t & 0xff) << 24) | ((t & 0xff00) << 8) | ((t >> 8) & 0xff00) | (t >> 24);
    drop(32);
    stage_flush();
    flush(true);
    const uint32_t adler = (ad_b << 16) | ad_a;
    if (want != adler) FAIL(16, pos);
    return R_OK;
  };
#undef NEEDB
#undef FAIL

  seek(8 * skip);
  const int rr = body();
  prod += nst;   // literals still in the stage (their ring bytes are never read again)
  InfRes o;
  o.arena_off = (rr == R_OK && to_arena) ? arena_off : ARENA_NONE;
  o.produced = prod;
  o.err = errcode | hint;
  if (rr == R_RETRY) {
    o.status = INF_RETRY;
    o.consumed = 0;
    o.arena_off = ARENA_NONE;
  } else if (rr == R_OK && !overflow) {
    o.status = INF_END;
    o.consumed = (pos - skip_bits) >> 3;
  } else if (rr == R_NEED) {
    o.status = INF_NEED;
    o.consumed = job.in_len;
  } else {
    o.status = INF_ERROR;
    if (overflow) o.err = 17;
    const uint64_t need = errneed > skip_bits ? errneed - skip_bits : 0;
    const uint64_t cons = (need + 7) >> 3;
    o.consumed = cons > job.in_len ? job.in_len : cons;
  }
#if ATZ_INF_CLOCKS
  o.cyc = __builtin_amdgcn_s_memtime() - t_start;
  o.nlit = nlit; o.nmatch = nmatch; o.cyc_copy = cyc_copy; o.cyc_flush = cyc_flush;
  o.nfar = nfar; o.cyc_far = cyc_far;
  o.nblk = nblk; o.cyc_hdr = cyc_hdr; o.nlong = nlong;
#else
  (void)t_start; (void)nlit; (void)nmatch; (void)cyc_copy; (void)cyc_flush; (void)nfar; (void)cyc_far;
  (void)nblk; (void)cyc_hdr; (void)nlong;
#endif
  if (lane == 0) res[j] = o;
}

}  // namespace atz
