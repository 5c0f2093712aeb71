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

static constexpr uint32_t RING = 32768;        // history ring per wave (LDS)
static constexpr uint32_t RMASK = RING - 1;
static constexpr uint32_t FLUSH_AT = 16384;    // flush ring to HBM / Adler every 16 KiB

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

// ---------------------------------------------------------------------------------------------
// k_inflate: one wavefront per job, everything inlined into the kernel so the decoder state stays
// in (wave-uniform) SGPRs -- a by-reference state struct crossing a call would live in scratch.

__device__ __forceinline__ uint32_t iuni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

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

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int d = 32; d >= 1; d >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, d, 64);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// Canonical Huffman code of one table: lane l (1..15) holds first-code/count/offset of length l;
// the sorted symbols live in VGPRs (entry e in lane e & 63, register e >> 6) and are read with
// v_readlane at a wave-uniform index -- no memory access per decoded symbol.
struct Huff {
  uint32_t first, count, offs;
  uint32_t s0, s1, s2, s3, s4;
  int max;
  __device__ __forceinline__ uint32_t sym(uint32_t e) const {
    uint32_t v;
    switch (e >> 6) {
      case 0: v = s0; break;
      case 1: v = s1; break;
      case 2: v = s2; break;
      case 3: v = s3; break;
      default: v = s4; break;
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(e & 63));
  }
};

enum { R_OK = 0, R_ERR = -1, R_NEED = -2 };

struct InfShared {
  uint8_t ring[RING];
  uint16_t lens[320];
  uint16_t sort[320];
};

__global__ __launch_bounds__(64) void k_inflate(const uint8_t* __restrict__ in_base, uint8_t* __restrict__ out_base,
                                               const InfJob* __restrict__ jobs, InfRes* __restrict__ res,
                                               uint32_t njobs, uint8_t* __restrict__ arena,
                                               unsigned long long* __restrict__ arena_used, uint64_t arena_cap) {
  __shared__ InfShared sh;
  const int lane = threadIdx.x;
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const InfJob job = jobs[j];
  uint8_t* const ring = sh.ring;
  uint16_t* const lens = sh.lens;

  // ---- bit reader over the job's bytes: 256-byte windows staged in lane VGPRs, next one in flight
  const uint8_t* p0 = in_base + job.in_off;
  const uintptr_t ap = reinterpret_cast<uintptr_t>(p0);
  const uint64_t skip = ap & 3;
  // global address space explicitly: a flat load would also count in lgkmcnt and make every LDS
  // wait drain the input prefetch
  const __attribute__((address_space(1))) uint32_t* const abase =
      (const __attribute__((address_space(1))) uint32_t*)(ap - skip);
  const uint64_t skip_bits = 8 * skip;
  const uint64_t limit = 8 * (skip + job.in_len);   // bit limit (aligned coordinates)
  uint64_t pos = 0, bb = 0, next_dw = 0, wbase = 1ull << 62;
  uint32_t bc = 0, cw = 0, nw = 0;
  // Bits past `limit` are never consumed (every consumption is preceded by has()), and a canonical
  // code found within the available bits is the true code whatever follows (prefix-free), so
  // the window is loaded unmasked -- the load stays asynchronous until its first readlane.  The
  // input buffers carry >= 4 KiB of slack for the <= 512-byte over-read.
  auto load_dw = [&](uint64_t dw) __attribute__((always_inline)) -> uint32_t { return abase[dw]; };
  auto refill = [&]() __attribute__((always_inline)) {
    while (bc <= 32) {
      const uint64_t k = next_dw;
      if (k - wbase >= 64) {
        if (k - wbase < 128) { cw = nw; wbase += 64; }
        else { wbase = k & ~63ull; cw = load_dw(wbase + lane); }
        nw = load_dw(wbase + 64 + lane);
      }
      const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)cw, (int)(k - wbase));
      bb |= (uint64_t)w << bc;
      bc += 32;
      next_dw = k + 1;
    }
  };
  auto seek = [&](uint64_t apos) __attribute__((always_inline)) {
    bb = 0; bc = 0;
    next_dw = apos >> 5;
    pos = apos & ~31ull;
    refill();
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
  uint64_t prod = 0, flushed = 0;
  uint32_t ad_a = 1, ad_b = 0;
  int overflow = 0;
  auto flush = [&](bool final) __attribute__((always_inline)) {
    const uint64_t n = prod - flushed;
    if (!n) return;
    if (to_arena && !arena_tried) {
      arena_tried = true;
      const uint64_t want = final ? ((prod + 255) & ~255ull) : out_cap;
      unsigned long long o = 0;
      if (lane == 0) o = atomicAdd(arena_used, (unsigned long long)want);
      o = __shfl(o, 0, 64);
      if (o + want <= arena_cap && (final || prod <= out_cap)) { arena_off = o; out = arena + o; }
    }
    uint64_t S = 0, W = 0;
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
  };

  // inflate_table acceptance (Z/inftrees.c:32-141); type 0 CODES, 1 LENS, 2 DISTS. Returns 0 / -1.
  auto build = [&](Huff& h, const uint16_t* ln, int n, int type) __attribute__((always_inline)) -> int {
    uint32_t cnt = 0;
    for (int g = 0; g < n; g += 64) {
      const int i = g + lane;
      const uint32_t len = i < n ? ln[i] : 0;
      for (int l = 1; l <= 15; l++) {
        const uint32_t c = __popcll(__ballot(len == (uint32_t)l));
        if (lane == l) cnt += c;
      }
    }
    int max = 0, left = 1, bad = 0;
    uint32_t code = 0, offs = 0, my_first = 0, my_offs = 0;
    for (int l = 1; l <= 15; l++) {
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cnt, l);
      if (c) max = l;
      left <<= 1;
      left -= (int)c;
      if (left < 0) bad = 1;
      if (lane == l) { my_first = code; my_offs = offs; }
      code = (code + c) << 1;
      offs += c;
    }
    h.max = max;
    if (max == 0) { h.count = 0; h.first = 0; h.offs = 0; return 0; }
    if (bad) return -1;
    if (left > 0 && (type == 0 || max != 1)) return -1;
    h.first = my_first; h.count = (lane >= 1 && lane <= 15) ? cnt : 0; h.offs = my_offs;
    // ballot-ranked counting sort into LDS, then into the VGPR table
    uint32_t run = my_offs;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int g = 0; g < n; g += 64) {
      const int i = g + lane;
      const uint32_t len = i < n ? ln[i] : 0;
      for (int l = 1; l <= 15; l++) {
        const uint64_t m = __ballot(len == (uint32_t)l);
        if (!m) continue;
        const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)run, l);
        if (len == (uint32_t)l) sh.sort[base + __popcll(m & lt)] = (uint16_t)i;
        if (lane == l) run += __popcll(m);
      }
    }
    h.s0 = sh.sort[lane];
    h.s1 = n > 64 ? sh.sort[64 + lane] : 0;
    h.s2 = n > 128 ? sh.sort[128 + lane] : 0;
    h.s3 = n > 192 ? sh.sort[192 + lane] : 0;
    h.s4 = n > 256 && lane < 64 ? sh.sort[256 + lane] : 0;
    return 0;
  };

  // Decode one symbol: >= 0 symbol, -1 invalid code, -2 need more input.  need = the bit position
  // zlib would have required when it stops here.
  auto decode = [&](const Huff& h, bool cl_quirk, uint64_t& need) __attribute__((always_inline)) -> int {
    if (h.max == 0) {
      need = pos + 1;
      if (!has(1)) return -2;
      drop(1);
      return cl_quirk ? 0 : -1;
    }
    const uint32_t v = __builtin_bitreverse32((uint32_t)bb) >> 17;   // first stream bit at bit 14
    const uint32_t c = v >> (15 - (lane & 15));
    const bool hit = lane >= 1 && lane <= 15 && (c - h.first) < h.count;
    const uint64_t m = __ballot(hit);
    if (!m) {  // only incomplete codes have unused patterns: zlib's invalid entry has 1 bit
      need = pos + 1;
      if (!has(1)) return -2;
      drop(1);
      return -1;
    }
    const uint32_t L = (uint32_t)__ffsll((unsigned long long)m) - 1;
    need = pos + L;
    if (!has(L)) return -2;
    const uint32_t idx = (uint32_t)__builtin_amdgcn_readlane((int)(h.offs + (c - h.first)), (int)L);
    drop(L);
    return (int)h.sym(idx);
  };

  uint64_t errneed = 0;
  uint32_t errcode = 0;
#define NEEDB(k) do { if (!has(k)) return R_NEED; } while (0)
#define FAIL(code, needpos) do { errneed = (needpos); errcode = (code); return R_ERR; } while (0)

  auto codes = [&](const Huff& lh, const Huff& dh) __attribute__((always_inline)) -> int {
    uint64_t need;
    for (;;) {
      int sym = decode(lh, false, need);
      if (sym == -2) return R_NEED;
      if (sym == -1) FAIL(10, need);
      if (sym < 256) {
        if (lane == 0) ring[prod & RMASK] = (uint8_t)sym;
        prod++;
        if (prod - flushed >= FLUSH_AT) flush(false);
        continue;
      }
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
      if ((uint64_t)dist > prod) FAIL(14, pos);            // invalid distance too far back
      // copy: read the whole source first (a period of `dist` repeats for overlapping copies)
      for (uint32_t i0 = 0; i0 < len; i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint32_t src = dist >= len ? i : i % dist;
        uint8_t v = 0;
        if (i < len) v = ring[(prod - dist + src) & RMASK];
        __builtin_amdgcn_wave_barrier();
        if (i < len) ring[(prod + i) & RMASK] = v;
      }
      prod += len;
      if (prod - flushed >= FLUSH_AT) flush(false);
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
    do {
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
        // copy `len` bytes straight from the input (byte aligned now)
        const uint64_t avail = (limit - pos) >> 3;
        const uint64_t take = len < avail ? len : avail;
        const __attribute__((address_space(1))) uint8_t* src =
            (const __attribute__((address_space(1))) uint8_t*)(ap - skip) + (pos >> 3);
        uint64_t done = 0;
        while (done < take) {
          uint64_t step = take - done;
          if (step > 4096) step = 4096;
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
        Huff lh, dh;
        build(lh, lens, 288, 1);
        for (int i = lane; i < 32; i += 64) lens[i] = 5;
        build(dh, lens, 32, 2);
        const int rr = codes(lh, dh);
        if (rr != R_OK) return rr;
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
        if (build(chh, lens, 19, 0)) FAIL(7, pos);
        uint32_t have = 0;
        const uint32_t total = nlen + ndist;
        uint64_t need;
        for (int i = lane; i < 320; i += 64) lens[i] = 0;
        uint32_t prevlen = 0;
        while (have < total) {
          const int sym = decode(chh, true, need);
          if (sym == -2) return R_NEED;
          if (sym < 16) { if (lane == 0) lens[have] = (uint16_t)sym; prevlen = (uint32_t)sym; have++; continue; }
          uint32_t copy, len = 0, eb;
          if (sym == 16) eb = 2; else if (sym == 17) eb = 3; else eb = 7;
          NEEDB(eb);
          if (sym == 16) {
            if (have == 0) FAIL(8, pos + eb);
            len = prevlen;
            copy = 3 + peek(2);
          } else if (sym == 17) {
            copy = 3 + peek(3);
          } else {
            copy = 11 + peek(7);
          }
          drop(eb);
          if (have + copy > total) FAIL(8, pos);
          for (uint32_t k = lane; k < copy; k += 64) lens[have + k] = (uint16_t)len;
          prevlen = len;
          have += copy;
        }
        if (iuni(lens[256]) == 0) FAIL(9, pos);
        Huff lh, dh;
        if (build(lh, lens, (int)nlen, 1)) FAIL(9, pos);
        if (build(dh, lens + nlen, (int)ndist, 2)) FAIL(9, pos);
        const int rr = codes(lh, dh);
        if (rr != R_OK) return rr;
      } else {
        FAIL(15, pos);                                      // invalid block type
      }
    } while (!last);
    // CHECK (Z/inflate.c:1174-1195)
    const uint32_t al = (uint32_t)((8 - (pos & 7)) & 7);
    drop(al);
    NEEDB(32);
    const uint32_t t = peek(32);
    const uint32_t want = ((t & 0xff) << 24) | ((t & 0xff00) << 8) | ((t >> 8) & 0xff00) | (t >> 24);
    drop(32);
    flush(true);
    const uint32_t adler = (ad_b << 16) | ad_a;
    if (want != adler) FAIL(16, pos);
    return R_OK;
  };
#undef NEEDB
#undef FAIL

  seek(8 * skip);
  const int rr = body();
  InfRes o;
  o.arena_off = (rr == R_OK && to_arena) ? arena_off : ARENA_NONE;
  o.produced = prod;
  o.err = errcode;
  if (rr == R_OK && !overflow) {
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
  if (lane == 0) res[j] = o;
}

}  // namespace atz
