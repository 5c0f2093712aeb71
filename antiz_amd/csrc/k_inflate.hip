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

static constexpr int INF_WAVES = 4;           // waves (= jobs) per workgroup
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
struct BitReader {
  const uint32_t* abase;  // 4-byte aligned base of the input
  uint64_t limit;         // bit limit in aligned coordinates
  uint64_t skip_bits;     // 8 * (misalignment of the job's first byte)
  uint64_t pos;           // aligned bit position of bb's bit 0
  uint64_t bb;
  uint32_t bc;
  uint64_t next_dw;
  uint64_t chunk;
  uint32_t cw;            // this lane's dword of the staged 256-byte chunk
};

__device__ inline void br_load_chunk(BitReader& r, uint64_t ch, int lane) {
  uint64_t dw = ch * 64 + lane;
  uint64_t byte0 = dw * 4;
  uint64_t lim_b = r.limit >> 3;
  uint32_t v = 0;
  if (byte0 < lim_b) {
    v = r.abase[dw];
    uint64_t valid = lim_b - byte0;
    if (valid < 4) v &= (1u << (8 * valid)) - 1;
  }
  r.cw = v;
  r.chunk = ch;
}

__device__ inline void br_refill(BitReader& r, int lane) {
  while (r.bc <= 32) {
    uint64_t k = r.next_dw;
    uint64_t ch = k >> 6;
    if (ch != r.chunk) br_load_chunk(r, ch, lane);
    uint32_t w = __builtin_amdgcn_readlane(r.cw, (int)(k & 63));
    r.bb |= (uint64_t)w << r.bc;
    r.bc += 32;
    r.next_dw = k + 1;
  }
}

__device__ inline void br_seek(BitReader& r, uint64_t apos, int lane) {
  r.bb = 0; r.bc = 0;
  r.next_dw = apos >> 5;
  r.pos = apos & ~31ull;
  br_refill(r, lane);
  uint32_t d = (uint32_t)(apos & 31);
  r.bb >>= d; r.bc -= d; r.pos += d;
  br_refill(r, lane);
}

__device__ inline uint32_t br_peek(const BitReader& r, uint32_t k) {
  return (uint32_t)(r.bb & ((k >= 32) ? 0xffffffffull : ((1ull << k) - 1)));
}
__device__ inline void br_drop(BitReader& r, uint32_t k, int lane) {
  r.bb >>= k; r.bc -= k; r.pos += k;
  if (r.bc <= 32) br_refill(r, lane);
}
__device__ inline bool br_has(const BitReader& r, uint64_t k) { return r.pos + k <= r.limit; }

// Per-wave canonical Huffman code: lane l (1..15) holds the values for code length l.
struct Huff {
  uint32_t first, count, offs;  // per-lane registers
  int max;                      // longest length (0: empty)
  int incomplete;               // incomplete (only legal with max==1) or empty
};

// inflate_table acceptance (Z/inftrees.c:32-141); type 0 CODES, 1 LENS, 2 DISTS. Returns 0 / -1.
__device__ int huff_build(Huff& h, const uint16_t* lens, int n, int type, uint16_t* syms, int lane) {
  uint32_t cnt = 0;
  for (int g = 0; g < n; g += 64) {
    int i = g + lane;
    uint32_t len = i < n ? lens[i] : 0;
    for (int l = 1; l <= 15; l++) {
      uint32_t c = __popcll(__ballot(len == (uint32_t)l));
      if (lane == l) cnt += c;
    }
  }
  int max = 0;
  int left = 1;
  int bad = 0;
  uint32_t code = 0, offs = 0;
  uint32_t my_first = 0, my_offs = 0;
  for (int l = 1; l <= 15; l++) {
    uint32_t c = __builtin_amdgcn_readlane(cnt, l);
    if (c) max = l;
    left <<= 1;
    left -= (int)c;
    if (left < 0) bad = 1;
    if (lane == l) { my_first = code; my_offs = offs; }
    code = (code + c) << 1;
    offs += c;
  }
  h.max = max;
  h.incomplete = 0;
  if (max == 0) { h.incomplete = 1; h.count = 0; h.first = 0; h.offs = 0; return 0; }
  if (bad) return -1;
  if (left > 0 && (type == 0 || max != 1)) return -1;
  if (left > 0) h.incomplete = 1;
  h.first = my_first; h.count = (lane >= 1 && lane <= 15) ? cnt : 0; h.offs = my_offs;
  // ballot-ranked symbol sort: syms[offs_l + rank] = i
  uint32_t run = my_offs;
  for (int g = 0; g < n; g += 64) {
    int i = g + lane;
    uint32_t len = i < n ? lens[i] : 0;
    uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int l = 1; l <= 15; l++) {
      uint64_t m = __ballot(len == (uint32_t)l);
      if (!m) continue;
      uint32_t base = __builtin_amdgcn_readlane(run, l);
      if (len == (uint32_t)l) syms[base + __popcll(m & lt)] = (uint16_t)i;
      if (lane == l) run += __popcll(m);
    }
  }
  return 0;
}

// Decode one symbol. Returns symbol >= 0, -1 invalid code (bits already dropped/accounted in *need),
// -2 need more input.  *need receives the relative bit position zlib would have required.
__device__ inline int huff_decode(BitReader& r, const Huff& h, const uint16_t* syms, int lane,
                                  bool cl_quirk, uint64_t& need) {
  if (h.max == 0) {
    need = r.pos + 1;
    if (!br_has(r, 1)) return -2;
    br_drop(r, 1, lane);
    return cl_quirk ? 0 : -1;
  }
  uint32_t v = __builtin_bitreverse32((uint32_t)r.bb) >> 17;   // first stream bit at bit 14
  uint32_t c = v >> (15 - (lane & 15));
  bool hit = lane >= 1 && lane <= 15 && (c - h.first) < h.count;
  uint64_t m = __ballot(hit);
  if (!m) {  // only incomplete codes have unused patterns: zlib's invalid entry has 1 bit
    need = r.pos + 1;
    if (!br_has(r, 1)) return -2;
    br_drop(r, 1, lane);
    return -1;
  }
  int L = __ffsll((unsigned long long)m) - 1;
  need = r.pos + (uint64_t)L;
  if (!br_has(r, (uint64_t)L)) return -2;
  uint32_t idx = __builtin_amdgcn_readlane(h.offs + (c - h.first), L);
  br_drop(r, (uint32_t)L, lane);
  return syms[idx];
}

__device__ __constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                                35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__device__ __constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                              2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__device__ __constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
                                                4097, 6145, 8193, 12289, 16385, 24577};
__device__ __constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                              6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__device__ __constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ inline uint64_t wave_sum_u64(uint64_t v) {
  for (int d = 32; d >= 1; d >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, d, 64);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

struct OutState {
  uint8_t* out;       // HBM output (nullptr: discard)
  uint64_t out_cap;
  uint64_t prod;      // bytes produced
  uint64_t flushed;   // bytes folded into Adler / written to HBM
  uint32_t a, b;      // Adler-32 halves
  int overflow;
};

__device__ void ring_flush(OutState& o, const uint8_t* ring, int lane) {
  uint64_t n = o.prod - o.flushed;
  if (!n) return;
  uint64_t S = 0, W = 0;
  for (uint64_t k = lane; k < n; k += 64) {
    uint32_t x = ring[(o.flushed + k) & RMASK];
    S += x;
    W += (n - k) * x;
    if (o.out && o.flushed + k < o.out_cap) o.out[o.flushed + k] = (uint8_t)x;
  }
  S = wave_sum_u64(S);
  W = wave_sum_u64(W);
  uint64_t a = o.a, b = o.b;
  b = (b + (n % 65521) * a + W) % 65521;
  a = (a + S) % 65521;
  o.a = (uint32_t)a; o.b = (uint32_t)b;
  if (o.out && o.prod > o.out_cap) o.overflow = 1;
  o.flushed = o.prod;
}

__device__ inline void put_lit(OutState& o, uint8_t* ring, uint32_t sym, int lane) {
  if (lane == 0) ring[o.prod & RMASK] = (uint8_t)sym;
  o.prod++;
  if (o.prod - o.flushed >= FLUSH_AT) ring_flush(o, ring, lane);
}

__device__ inline void put_copy(OutState& o, uint8_t* ring, uint32_t len, uint32_t dist, int lane) {
  uint8_t v[5];
#pragma unroll
  for (int r = 0; r < 5; r++) {
    uint32_t i = lane + 64 * r;
    uint32_t src = dist >= len ? i : i % dist;
    v[r] = i < len ? ring[(o.prod - dist + src) & RMASK] : 0;
  }
#pragma unroll
  for (int r = 0; r < 5; r++) {
    uint32_t i = lane + 64 * r;
    if (i < len) ring[(o.prod + i) & RMASK] = v[r];
  }
  o.prod += len;
  if (o.prod - o.flushed >= FLUSH_AT) ring_flush(o, ring, lane);
}

enum { R_OK = 0, R_ERR = -1, R_NEED = -2 };

struct Ctx {
  BitReader r;
  OutState o;
  uint64_t errneed;  // aligned bit position required by the failing item
  uint32_t errcode;
};

#define NEEDB(k) do { if (!br_has(c.r, (k))) return R_NEED; } while (0)
#define FAIL(code, needpos) do { c.errneed = (needpos); c.errcode = (code); return R_ERR; } while (0)

__device__ int decode_codes(Ctx& c, const Huff& lh, const uint16_t* lsym, const Huff& dh,
                            const uint16_t* dsym, uint8_t* ring, int lane) {
  uint64_t need;
  for (;;) {
    int sym = huff_decode(c.r, lh, lsym, lane, false, need);
    if (sym == -2) return R_NEED;
    if (sym == -1) FAIL(10, need);
    if (sym < 256) { put_lit(c.o, ring, (uint32_t)sym, lane); continue; }
    if (sym == 256) return R_OK;
    sym -= 257;
    if (sym >= 29) FAIL(11, need);                       // fixed codes 286/287
    uint32_t le = c_lext[sym];
    NEEDB(le);
    uint32_t len = c_lbase[sym] + br_peek(c.r, le);
    br_drop(c.r, le, lane);
    int ds = huff_decode(c.r, dh, dsym, lane, false, need);
    if (ds == -2) return R_NEED;
    if (ds == -1) FAIL(12, need);
    if (ds >= 30) FAIL(13, need);                        // fixed distance 30/31
    uint32_t de = c_dext[ds];
    NEEDB(de);
    uint32_t dist = c_dbase[ds] + br_peek(c.r, de);
    br_drop(c.r, de, lane);
    if ((uint64_t)dist > c.o.prod) FAIL(14, c.r.pos);     // invalid distance too far back
    put_copy(c.o, ring, len, dist, lane);
  }
}

__device__ int inflate_body(Ctx& c, uint8_t* ring, uint16_t* lsym, uint16_t* dsym, uint16_t* csym,
                            uint16_t* lens, int lane) {
  // HEAD (Z/inflate.c:640-685): wrap=1, wbits=15
  NEEDB(16);
  uint32_t cmf = br_peek(c.r, 8);
  uint32_t flg = (br_peek(c.r, 16) >> 8) & 0xff;
  if (((cmf << 8) + flg) % 31) FAIL(1, c.r.pos + 16);
  if ((cmf & 15) != 8) FAIL(2, c.r.pos + 16);
  if ((cmf >> 4) + 8 > 15) FAIL(3, c.r.pos + 16);
  br_drop(c.r, 16, lane);
  if (flg & 0x20) { NEEDB(32); FAIL(4, c.r.pos + 32); }   // preset dictionary: not a stream end
  int last;
  do {
    NEEDB(3);
    last = (int)br_peek(c.r, 1);
    uint32_t type = (br_peek(c.r, 3) >> 1) & 3;
    br_drop(c.r, 3, lane);
    if (type == 0) {                                      // STORED
      uint32_t al = (uint32_t)((8 - (c.r.pos & 7)) & 7);
      br_drop(c.r, al, lane);
      NEEDB(32);
      uint32_t len = br_peek(c.r, 16);
      uint32_t nlen = (br_peek(c.r, 32) >> 16) & 0xffff;
      if (len != (~nlen & 0xffff)) FAIL(5, c.r.pos + 32);
      br_drop(c.r, 32, lane);
      // copy `len` bytes straight from the input (byte aligned now)
      uint64_t avail = (c.r.limit - c.r.pos) >> 3;
      uint64_t take = len < avail ? len : avail;
      const uint8_t* src = reinterpret_cast<const uint8_t*>(c.r.abase) + (c.r.pos >> 3);
      uint64_t done = 0;
      while (done < take) {
        uint64_t step = take - done;
        if (step > 4096) step = 4096;
        uint64_t room = RING - (c.o.prod - c.o.flushed);
        if (step > room) { ring_flush(c.o, ring, lane); continue; }
        for (uint64_t k = lane; k < step; k += 64) ring[(c.o.prod + k) & RMASK] = src[done + k];
        c.o.prod += step;
        done += step;
        if (c.o.prod - c.o.flushed >= FLUSH_AT) ring_flush(c.o, ring, lane);
      }
      br_seek(c.r, c.r.pos + 8 * take, lane);
      if (take < len) return R_NEED;
    } else if (type == 1) {                               // FIXED
      for (int i = lane; i < 288; i += 64) lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
      Huff lh, dh;
      huff_build(lh, lens, 288, 1, lsym, lane);
      for (int i = lane; i < 32; i += 64) lens[i] = 5;
      huff_build(dh, lens, 32, 2, dsym, lane);
      int rr = decode_codes(c, lh, lsym, dh, dsym, ring, lane);
      if (rr != R_OK) return rr;
    } else if (type == 2) {                               // DYNAMIC (Z/inflate.c:908-1013)
      NEEDB(14);
      uint32_t nlen = br_peek(c.r, 5) + 257;
      uint32_t ndist = ((br_peek(c.r, 10) >> 5) & 31) + 1;
      uint32_t ncode = ((br_peek(c.r, 14) >> 10) & 15) + 4;
      if (nlen > 286 || ndist > 30) FAIL(6, c.r.pos + 14);
      br_drop(c.r, 14, lane);
      for (int i = lane; i < 320; i += 64) lens[i] = 0;
      for (uint32_t i = 0; i < ncode; i++) {
        NEEDB(3);
        uint32_t v = br_peek(c.r, 3);
        br_drop(c.r, 3, lane);
        if (lane == 0) lens[c_clorder[i]] = (uint16_t)v;
      }
      Huff ch;
      if (huff_build(ch, lens, 19, 0, csym, lane)) FAIL(7, c.r.pos);
      uint32_t have = 0;
      uint32_t total = nlen + ndist;
      uint64_t need;
      for (int i = lane; i < 320; i += 64) lens[i] = 0;
      while (have < total) {
        int sym = huff_decode(c.r, ch, csym, lane, true, need);
        if (sym == -2) return R_NEED;
        if (sym < 16) { if (lane == 0) lens[have] = (uint16_t)sym; have++; continue; }
        uint32_t copy, len = 0, eb;
        if (sym == 16) eb = 2; else if (sym == 17) eb = 3; else eb = 7;
        NEEDB(eb);
        if (sym == 16) {
          if (have == 0) FAIL(8, c.r.pos + eb);
          len = lens[have - 1];
          copy = 3 + br_peek(c.r, 2);
        } else if (sym == 17) {
          copy = 3 + br_peek(c.r, 3);
        } else {
          copy = 11 + br_peek(c.r, 7);
        }
        br_drop(c.r, eb, lane);
        if (have + copy > total) FAIL(8, c.r.pos);
        for (uint32_t k = lane; k < copy; k += 64) lens[have + k] = (uint16_t)len;
        have += copy;
      }
      if (lens[256] == 0) FAIL(9, c.r.pos);
      Huff lh, dh;
      if (huff_build(lh, lens, (int)nlen, 1, lsym, lane)) FAIL(9, c.r.pos);
      if (huff_build(dh, lens + nlen, (int)ndist, 2, dsym, lane)) FAIL(9, c.r.pos);
      int rr = decode_codes(c, lh, lsym, dh, dsym, ring, lane);
      if (rr != R_OK) return rr;
    } else {
      FAIL(15, c.r.pos);                                  // invalid block type
    }
  } while (!last);
  // CHECK (Z/inflate.c:1174-1195)
  uint32_t al = (uint32_t)((8 - (c.r.pos & 7)) & 7);
  br_drop(c.r, al, lane);
  NEEDB(32);
  uint32_t t = br_peek(c.r, 32);
  uint32_t want = ((t & 0xff) << 24) | ((t & 0xff00) << 8) | ((t >> 8) & 0xff00) | (t >> 24);
  br_drop(c.r, 32, lane);
  ring_flush(c.o, ring, lane);
  uint32_t adler = (c.o.b << 16) | c.o.a;
  if (want != adler) FAIL(16, c.r.pos);
  return R_OK;
}

struct InfShared {
  uint8_t ring[INF_WAVES][RING];
  uint16_t lsym[INF_WAVES][320];
  uint16_t dsym[INF_WAVES][32];
  uint16_t csym[INF_WAVES][32];
  uint16_t lens[INF_WAVES][320];
};

__global__ __launch_bounds__(64 * INF_WAVES) void k_inflate(const uint8_t* __restrict__ in_base,
                                                           uint8_t* __restrict__ out_base,
                                                           const InfJob* __restrict__ jobs,
                                                           InfRes* __restrict__ res, uint32_t njobs) {
  __shared__ InfShared sh;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const uint32_t j = blockIdx.x * INF_WAVES + wave;
  if (j >= njobs) return;
  const InfJob job = jobs[j];
  Ctx c;
  const uint8_t* p = in_base + job.in_off;
  uintptr_t ap = reinterpret_cast<uintptr_t>(p);
  uint64_t skip = ap & 3;
  c.r.abase = reinterpret_cast<const uint32_t*>(ap - skip);
  c.r.skip_bits = 8 * skip;
  c.r.limit = 8 * (skip + job.in_len);
  c.r.chunk = ~0ull;
  c.r.cw = 0;
  br_seek(c.r, 8 * skip, lane);
  c.o.out = job.out_off == NO_OUT ? nullptr : out_base + job.out_off;
  c.o.out_cap = job.out_cap;
  c.o.prod = 0; c.o.flushed = 0; c.o.a = 1; c.o.b = 0; c.o.overflow = 0;
  c.errneed = 0; c.errcode = 0;
  int rr = inflate_body(c, sh.ring[wave], sh.lsym[wave], sh.dsym[wave], sh.csym[wave], sh.lens[wave], lane);
  InfRes out;
  out.produced = c.o.prod;
  out.err = c.errcode;
  if (rr == R_OK && !c.o.overflow) {
    out.status = INF_END;
    out.consumed = (c.r.pos - c.r.skip_bits) >> 3;
  } else if (rr == R_NEED) {
    out.status = INF_NEED;
    out.consumed = job.in_len;
  } else {
    out.status = INF_ERROR;
    if (c.o.overflow) out.err = 17;
    uint64_t need = c.errneed > c.r.skip_bits ? c.errneed - c.r.skip_bits : 0;
    uint64_t cons = (need + 7) >> 3;
    out.consumed = cons > job.in_len ? job.in_len : cons;
  }
  if (lane == 0) res[j] = out;
}

}  // namespace atz
