// k_deflate.hip -- zlib 1.2.8-exact deflate trials on CDNA4 (gfx950).
//
// The reference's hot loop (testDeflateParams, main.cpp:603-731, ~83 % of its time inside zlib
// deflate) is re-designed for the GPU in two kernels:
//
// k_chains  (one wavefront per (stream, memLevel)): the hash chains of zlib's INSERT_STRING
//   (Z/deflate.c:181-190) for EVERY position, as a table of u16 distances to the previous
//   position with the same hash_bits=memLevel+7 rolling hash (0 = none within 32 KiB).  zlib's
//   rolling hash is a pure function of 3 bytes (3*hash_shift >= hash_bits), and deflate_slow
//   inserts every position, so these chains are parse-independent and shared by every trial
//   of the stream at that memLevel; deflate_fast's partial insertion is replayed by skipping
//   positions a per-trial LDS bitmap marks as not inserted.  Batches of 64 positions are
//   bitonic-sorted by hash across lanes; only the batch's first/last occurrence per hash touches
//   the head table.
//
// k_trial<KIND>  (one wavefront per (stream, clevel, window, memLevel) trial): replays
//   deflate_stored/deflate_fast/deflate_slow (Z/deflate.c:1564-1853) on absolute positions --
//   fill_window and the window slide are reduced to bookkeeping (the slide only matters through
//   zlib's NIL quirks, which are reproduced) -- walks the chains with longest_match's exact
//   stop rules (Z/deflate.c:1148-1289), tallies symbols into an HBM symbol buffer and LDS
//   frequency counters, and at every block flush builds the Huffman trees with zlib's heap,
//   depth tie-break and overflow fix-up (Z/trees.c:453-699), chooses stored/static/dynamic
//   (Z/trees.c:907-1004) and bit-packs the block lane-parallel: each lane encodes one symbol,
//   a wave prefix sum places its bits, LDS atomics assemble the words.  The emitted bytes are
//   compared positionally against the original stream as they are written, so the reference's
//   shortcut / size-difference gates (main.cpp:632-681) and "cannot beat the best so far" stop a
//   trial as early as its outcome is decided.
#include <hip/hip_runtime.h>
#include "atz_device.h"

// LDS-typed references make the non-inlined block-flush helpers use ds_* instructions (a generic
// reference would compile to flat accesses with longer latency and vmcnt coupling).
#define LDS __attribute__((address_space(3)))
#define CONSTANT __attribute__((address_space(4)))
#define GLOBAL __attribute__((address_space(1)))

#ifndef ATZ_VISITED_CHECK
#define ATZ_VISITED_CHECK 1   // fast levels: resolve slot-check failures by the visited nodes' insertion bits
#endif
#ifndef ATZ_VISITED_MAX
#define ATZ_VISITED_MAX 8     // ... for levels whose chain budget is at most this (level 3's 32: measured slower)
#endif
// Per-step shader-clock counters in the parse loop (diagnostics; s_memtime also forces lgkmcnt waits).
#ifndef ATZ_NOSLIDE_PATH
#define ATZ_NOSLIDE_PATH 1    // parse: skip the window-slide checks for streams that never slide
#endif
#ifndef ATZ_STEP_SPLIT
#define ATZ_STEP_SPLIT 0
#endif
#ifndef ATZ_STEP_CLOCKS
#define ATZ_STEP_CLOCKS 0
#endif
#if ATZ_STEP_CLOCKS
#define STEP_CLOCK() clock64()
#else
#define STEP_CLOCK() 0ull
#endif

namespace atz {

// ---------------------------------------------------------------------------------------------
// static tables (trees.c tr_static_init, generated on the host at context creation)
struct DeflTables {
  uint16_t st_lcode[288]; uint8_t st_llen[288];
  uint16_t st_dcode[30];  uint8_t st_dlen[30];
  uint8_t lcode[256];     // normalized match length -> length code 0..28
  uint8_t dcode[512];     // d_code()
  uint16_t lbase[29];
  uint16_t dbase[30];
};
__device__ __constant__ DeflTables c_t;
__device__ __constant__ uint8_t c_xlb[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
__device__ __constant__ uint8_t c_xdb[30] = {0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};
__device__ __constant__ uint8_t c_xblb[19] = {0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,2,3,7};
__device__ __forceinline__ uint32_t bl_order(uint32_t i) {   // {16,17,18,0,8,7,...,1,15}, 5 bits each
  return (uint32_t)((i < 12 ? (0x22caa324e804a30ull >> (5 * i)) : (0x3c2e1346cull >> (5 * (i - 12)))) & 31);
}
// configuration_table, Z/deflate.c:131-143: good, lazy, nice, chain
__device__ __constant__ uint16_t c_cfg[10][4] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32},{4,4,16,16},
    {8,16,32,32},{8,16,128,128},{8,32,128,256},{32,128,258,1024},{32,258,258,4096}};

// Values that are wave-uniform but come from memory, a call or a lane-masked region: re-declare
// them uniform so the parse state stays in SGPRs with scalar branches.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

extern "C" hipError_t atz_upload_defl_tables(const void* host_tables) {
  return hipMemcpyToSymbol(HIP_SYMBOL(c_t), host_tables, sizeof(DeflTables));
}

// ---------------------------------------------------------------------------------------------
// k_buckets: zlib's hash chains (INSERT_STRING, Z/deflate.c:181-190) for every position of a stream,
// as hash buckets: bpos[] = the positions sorted by (hash, position), sidx[p] = p's index in bpos.
// The chain of p is then the descending run bpos[sidx[p]-1], bpos[sidx[p]-2], ... down to the
// bucket's first entry (bit 31 set) -- contiguous memory instead of a linked list, so walks issue
// independent loads.  zlib's rolling hash is a pure function of 3 bytes (3*hash_shift >= hash_bits)
// and deflate_slow inserts every position, so the buckets depend only on (stream, memLevel) and
// are shared by every trial; deflate_fast's partial insertion is handled in the trial.
// Layout at chain_off (u32 units): sidx[npad] then bpos[npad], npad = n rounded up to 64.
struct ChainJob {
  uint64_t infl_off;   // stream bytes in the inflated buffer
  uint64_t n;          // I_s
  uint64_t chain_off;  // u32 units in the chain buffer
  uint32_t memlevel;
  uint32_t slot;       // scratch slot (2 x 65536 words)
  uint32_t dslot;      // k_buckets_sort: index of the job's deepest-bucket entry in its depth output
  uint32_t pad_;
};
static constexpr uint32_t BUCKET_FIRST = 0x80000000u;

__global__ __launch_bounds__(64) void k_buckets(const uint8_t* __restrict__ infl, const ChainJob* __restrict__ jobs,
                                               uint32_t* __restrict__ chains, uint64_t* __restrict__ scratch,
                                               uint32_t njobs) {
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const int lane = threadIdx.x;
  const ChainJob jb = jobs[j];
  const uint8_t* in = infl + jb.infl_off;
  const uint32_t n = (uint32_t)jb.n;
  const uint32_t npad = (n + 63) & ~63u;
  uint32_t* sidx = chains + jb.chain_off;
  uint32_t* bpos = sidx + npad;
  const uint32_t hbits = jb.memlevel + 7, hsize = 1u << hbits, hmask = hsize - 1, hshift = (hbits + 2) / 3;
  // per hash one 64-bit word: count during the histogram, then (first index << 32) | assigned
  uint64_t* word = scratch + (uint64_t)jb.slot * 65536;
  for (uint32_t i = lane; i < hsize; i += 64) word[i] = 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  const uint32_t nh = n >= 3 ? n - 2 : 0;                 // positions with a hash (p + 3 <= n)
  auto hash = [&](uint32_t p) -> uint32_t {
    return (((uint32_t)in[p] << (2 * hshift)) ^ ((uint32_t)in[p + 1] << hshift) ^ in[p + 2]) & hmask;
  };
  for (uint32_t p = lane; p < nh; p += 64) atomicAdd((unsigned long long*)&word[hash(p)], 1ull);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  // exclusive scan of the counts -> first index of each bucket (8 chunks of loads in flight)
  uint32_t run = 0;
  for (uint32_t g0 = 0; g0 < hsize; g0 += 512) {
    uint32_t c[8];
#pragma unroll
    for (int u = 0; u < 8; u++) c[u] = g0 + 64 * u < hsize ? (uint32_t)word[g0 + 64 * u + lane] : 0u;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (g0 + 64 * u >= hsize) break;
      uint32_t incl = c[u];
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
      }
      word[g0 + 64 * u + lane] = (uint64_t)(run + incl - c[u]) << 32;
      run += __shfl(incl, 63, 64);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  // assignment in position order: 64 positions at a time, bitonic-sorted by (hash, lane); one
  // returning atomic per group gives (first index, assigned so far) -- same-address atomics of
  // one wave complete in issue order, so no fence is needed between batches
  uint32_t hn = lane < (int)nh ? hash((uint32_t)lane) : 0x3ffffffu;   // next batch's hashes, loaded ahead
  for (uint32_t b0 = 0; b0 < nh; b0 += 64) {
    const uint32_t h = hn;
    const uint32_t pn = b0 + 64 + lane;
    hn = pn < nh ? hash(pn) : 0x3ffffffu;
    uint32_t key = (h << 6) | (uint32_t)lane;
    for (int k = 2; k <= 64; k <<= 1)
      for (int st = k >> 1; st > 0; st >>= 1) {
        const uint32_t o = __shfl_xor(key, st, 64);
        const bool up = (lane & k) == 0, lower = (lane & st) == 0;
        const uint32_t mn = key < o ? key : o, mx = key < o ? o : key;
        key = (lower == up) ? mn : mx;
      }
    const uint32_t kh = key >> 6;
    const uint32_t mypos = b0 + (key & 63);
    const uint32_t pk = __shfl_up(key, 1, 64), nk = __shfl_down(key, 1, 64);
    const bool first = lane == 0 || (pk >> 6) != kh;
    const bool last = lane == 63 || (nk >> 6) != kh;
    const bool real = kh != 0x3ffffffu;
    const uint64_t fm = __ballot(first);
    const uint64_t below = fm & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
    const uint32_t gstart = 63 - (uint32_t)__clzll((long long)below);
    const uint64_t lm = __ballot(last);
    const uint64_t above = lm & (~0ull << lane);
    const uint32_t gend = (uint32_t)__ffsll((unsigned long long)above) - 1;
    uint64_t old = 0;
    if (real && first) old = atomicAdd((unsigned long long*)&word[kh], (unsigned long long)(gend - gstart + 1));
    const uint32_t olo = __shfl((uint32_t)old, (int)gstart, 64), ohi = __shfl((uint32_t)(old >> 32), (int)gstart, 64);
    if (real) {
      const uint32_t r = olo + (uint32_t)lane - gstart;
      sidx[mypos] = ohi + r;
      bpos[ohi + r] = mypos | (r == 0 ? BUCKET_FIRST : 0u);
    }
  }
}

// LDS variant for hash tables of <= TABLE (4096, 16384 or 32768) entries and streams < 65536 positions: one workgroup
// (4 waves) per job, one 32-bit LDS word per hash = (first index << 16) | assigned.  Zeroing, the
// histogram and the scan use all 256 threads; the in-order assignment runs on wave 0 with LDS
// atomics (~100-cycle round trips instead of HBM ones).
template <uint32_t TABLE>
__global__ __launch_bounds__(256) void k_buckets_lds(const uint8_t* __restrict__ infl,
                                                    const ChainJob* __restrict__ jobs,
                                                    uint32_t* __restrict__ chains, uint32_t njobs) {
  __shared__ uint32_t word[TABLE];
  __shared__ uint32_t wsum[4];
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const ChainJob jb = jobs[j];
  const uint8_t* in = infl + jb.infl_off;
  const uint32_t n = (uint32_t)jb.n;
  const uint32_t npad = (n + 63) & ~63u;
  uint32_t* sidx = chains + jb.chain_off;
  uint32_t* bpos = sidx + npad;
  const uint32_t hbits = jb.memlevel + 7, hsize = 1u << hbits, hmask = hsize - 1, hshift = (hbits + 2) / 3;
  for (uint32_t i = tid; i < hsize; i += 256) word[i] = 0;
  __syncthreads();
  const uint32_t nh = n >= 3 ? n - 2 : 0;
  auto hash = [&](uint32_t p) -> uint32_t {
    return (((uint32_t)in[p] << (2 * hshift)) ^ ((uint32_t)in[p + 1] << hshift) ^ in[p + 2]) & hmask;
  };
  for (uint32_t p0 = 0; p0 < nh; p0 += 1024) {   // 4 positions per thread in flight
    uint32_t hs[4];
#pragma unroll
    for (int u = 0; u < 4; u++) { const uint32_t p = p0 + 256 * u + tid; hs[u] = p < nh ? hash(p) : 0xffffffffu; }
#pragma unroll
    for (int u = 0; u < 4; u++) if (hs[u] != 0xffffffffu) atomicAdd(&word[hs[u]], 1u);
  }
  __syncthreads();
  // exclusive scan: each wave scans a quarter of the table, then the quarters are offset
  const uint32_t q = hsize / 4;   // >= 64
  uint32_t run = 0;
  for (uint32_t g = wave * q; g < (wave + 1) * q; g += 64) {
    const uint32_t c = word[g + lane];
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(incl, d, 64);
      if (lane >= d) incl += t;
    }
    word[g + lane] = run + incl - c;
    run += __shfl(incl, 63, 64);
  }
  if (lane == 0) wsum[wave] = run;
  __syncthreads();
  uint32_t off = 0;
  for (int w = 0; w < wave; w++) off += wsum[w];
  for (uint32_t g = wave * q; g < (wave + 1) * q; g += 64) word[g + lane] = (word[g + lane] + off) << 16;
  __syncthreads();
  if (wave != 0) return;
  // In-order assignment, 64 positions at a time: one LDS atomic per lane gives (bucket base,
  // assigned so far).  Lanes of one batch that share a hash receive their ranks in an undefined
  // order; a read-back after the batch's atomics shows them (the count moved by more than one),
  // and only those groups (rare: ~6 % of batches at hash_bits 15) are re-ranked by lane.
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t hn = lane < (int)nh ? hash((uint32_t)lane) : 0u;
  for (uint32_t b0 = 0; b0 < nh; b0 += 64) {
    const uint32_t h = hn;
    const uint32_t p = b0 + (uint32_t)lane;
    const uint32_t pn = p + 64;
    hn = pn < nh ? hash(pn) : 0u;
    const bool real = p < nh;
    uint32_t old = 0;
    if (real) old = atomicAdd(&word[h], 1u);
    const uint32_t cur = real ? __hip_atomic_load(&word[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0u;
    uint32_t r = old & 0xffffu;
    uint64_t todo = __ballot(real && (cur & 0xffffu) != r + 1u);
    while (todo) {
      const int l0 = __ffsll((unsigned long long)todo) - 1;
      const uint32_t hh = (uint32_t)__builtin_amdgcn_readlane((int)h, l0);
      const uint64_t g = __ballot(real && h == hh);
      const uint32_t end = (uint32_t)__builtin_amdgcn_readlane((int)cur, l0) & 0xffffu;
      if (real && h == hh) r = end - (uint32_t)__popcll(g) + (uint32_t)__popcll(g & lt);
      todo &= ~g;
    }
    if (real) {
      const uint32_t at = (old >> 16) + r;
      sidx[p] = at;
      bpos[at] = p | (r == 0 ? BUCKET_FIRST : 0u);
    }
  }
}

// memLevel 8 / 9 (2^15 / 2^16 hashes), streams < 65536 positions: two 16-bit counters per LDS word
// (64 / 128 KiB: half the LDS of 32-bit counters) for the histogram and then "assigned so far"; the
// bucket bases go to HBM scratch (read-only after the scan, loaded one batch ahead with the hashes).
// No HBM atomics.
template <uint32_t HBITS>
__global__ __launch_bounds__(256) void k_buckets_pk(const uint8_t* __restrict__ infl,
                                                   const ChainJob* __restrict__ jobs,
                                                   uint32_t* __restrict__ chains, uint32_t* __restrict__ scratch,
                                                   uint32_t njobs) {
  constexpr uint32_t PW = (1u << HBITS) / 2, QW = PW / 4;   // pair words, pair words per wave
  __shared__ uint32_t pair[PW];   // counters of hashes 2i (low half) and 2i+1 (high half)
  __shared__ uint32_t wsum[4];
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const ChainJob jb = jobs[j];
  const uint8_t* in = infl + jb.infl_off;
  const uint32_t n = (uint32_t)jb.n;
  const uint32_t npad = (n + 63) & ~63u;
  uint32_t* sidx = chains + jb.chain_off;
  uint32_t* bpos = sidx + npad;
  uint32_t* base = scratch + (uint64_t)jb.slot * 65536;
  const uint32_t hmask = (1u << HBITS) - 1, hshift = (HBITS + 2) / 3;
  for (uint32_t i = tid; i < PW; i += 256) pair[i] = 0;
  __syncthreads();
  const uint32_t nh = n >= 3 ? n - 2 : 0;
  auto hash = [&](uint32_t p) -> uint32_t {
    return (((uint32_t)in[p] << (2 * hshift)) ^ ((uint32_t)in[p + 1] << hshift) ^ in[p + 2]) & hmask;
  };
  for (uint32_t p = tid; p < nh; p += 256) {
    const uint32_t h = hash(p);
    atomicAdd(&pair[h >> 1], 1u << (16 * (h & 1)));
  }
  __syncthreads();
  // exclusive scan over the 2^HBITS counts (each wave a quarter; lane handles 2 counts per word)
  uint32_t run = 0;
  for (uint32_t g = wave * QW; g < (wave + 1) * QW; g += 64) {
    const uint32_t w = pair[g + lane];
    const uint32_t c = (w & 0xffffu) + (w >> 16);
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(incl, d, 64);
      if (lane >= d) incl += t;
    }
    const uint32_t e0 = run + incl - c;
    base[2 * (g + lane)] = e0;
    base[2 * (g + lane) + 1] = e0 + (w & 0xffffu);
    pair[g + lane] = 0;
    run += __shfl(incl, 63, 64);
  }
  if (lane == 0) wsum[wave] = run;
  __syncthreads();
  uint32_t off = 0;
  for (int w = 0; w < wave; w++) off += wsum[w];
  if (off)
    for (uint32_t g = wave * QW; g < (wave + 1) * QW; g += 64) {
      base[2 * (g + lane)] += off;
      base[2 * (g + lane) + 1] += off;
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (wave != 0) return;
  // in-order assignment as in k_buckets_lds (one atomic per lane on the hash's 16-bit field, a
  // read-back to find the lanes that shared a field, re-ranked by lane)
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t hn = lane < (int)nh ? hash((uint32_t)lane) : 0u;
  uint32_t bn = lane < (int)nh ? base[hn] : 0u;
  for (uint32_t b0 = 0; b0 < nh; b0 += 64) {
    const uint32_t h = hn, bh = bn;
    const uint32_t p = b0 + (uint32_t)lane;
    const uint32_t pn = p + 64;
    hn = pn < nh ? hash(pn) : 0u;
    bn = pn < nh ? base[hn] : 0u;
    const bool real = p < nh;
    const uint32_t sh = 16u * (h & 1u);
    uint32_t old = 0;
    if (real) old = atomicAdd(&pair[h >> 1], 1u << sh);
    const uint32_t cur = real ? __hip_atomic_load(&pair[h >> 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0u;
    uint32_t r = (old >> sh) & 0xffffu;
    uint64_t todo = __ballot(real && ((cur >> sh) & 0xffffu) != r + 1u);
    while (todo) {
      const int l0 = __ffsll((unsigned long long)todo) - 1;
      const uint32_t hh = (uint32_t)__builtin_amdgcn_readlane((int)h, l0);
      const uint64_t g = __ballot(real && h == hh);
      const uint32_t end = ((uint32_t)__builtin_amdgcn_readlane((int)cur, l0) >> (16u * (hh & 1u))) & 0xffffu;
      if (real && h == hh) r = end - (uint32_t)__popcll(g) + (uint32_t)__popcll(g & lt);
      todo &= ~g;
    }
    if (real) {
      const uint32_t at = bh + r;
      sidx[p] = at;
      bpos[at] = p | (r == 0 ? BUCKET_FIRST : 0u);
    }
  }
}

// k_buckets_sort: the same bucket arrays by a stable LSD radix sort of the positions by hash, on every
// wave of the block (the kernels above assign positions in order on one wave, which left a 128 KiB-LDS
// block's CU mostly idle).  One pass per <= 8-bit digit (hash_bits = memLevel + 7: one pass for
// memLevel 1, two above), each pass a stable counting sort: every wave owns a contiguous tile of the
// current order and holds it in registers as (hash << 16 | position), 64 positions per VGPR; it counts
// its digits per batch of 64 (lanes sharing a digit found with one ballot per digit bit), an exclusive
// scan over (digit, wave) gives each wave's output ranges in digit-major, wave-minor order, and the
// waves scatter their tiles' positions into one u16 array in LDS.  Before the next pass every wave
// reloads its tile of that array (re-reading each position's 3 input bytes for its hash), so the
// scatter can overwrite it.  The sorted tile then writes bpos (first entry of a hash flagged
// BUCKET_FIRST) and scatters the inverse permutation into the same LDS array, which is copied out as
// sidx.  So HBM sees exactly one coalesced write of bpos and one of sidx (8 bytes per position); an
// earlier version scattered both arrays through HBM/L2 and wrote 2.8 GB per launch.  The result is the
// unique (hash, position) order, identical to the other kernels' output.
// LDS: 2 bytes per position + 2 bytes per (digit, wave); streams of < 64 Ki positions.  MAXC: batches
// of 64 positions per wave (the tile a wave keeps in registers), from the host's size class.
static constexpr uint32_t BSORT_THREADS = 1024, BSORT_W = BSORT_THREADS / 64;
static constexpr uint32_t BSORT_CNT_BYTES = 256 * BSORT_W * 2;
__host__ __device__ constexpr uint32_t bsort_lds_bytes(uint32_t npad) { return 2 * npad + BSORT_CNT_BYTES; }
__host__ __device__ constexpr uint32_t bsort_chunks(uint32_t npad) { return (npad + BSORT_THREADS - 1) / BSORT_THREADS; }
// lanes of the wave (among `valid` ones) whose `bits`-bit digit equals this lane's
__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid, uint32_t bits) {
  uint64_t m = __ballot(valid);
  for (uint32_t k = 0; k < bits; k++) {
    const bool b = (d >> k) & 1u;
    const uint64_t bal = __ballot(b);
    m &= b ? bal : ~bal;
  }
  return m;
}
__device__ __forceinline__ uint32_t bhash(const uint8_t* in, uint32_t p, uint32_t hs, uint32_t hm) {
  return ((((uint32_t)in[p] << (2 * hs)) ^ ((uint32_t)in[p + 1] << hs) ^ in[p + 2]) & hm);
}
template <uint32_t MAXC>
__global__ __launch_bounds__(BSORT_THREADS, MAXC <= 20 ? 8 : 4) void k_buckets_sort(
    const uint8_t* __restrict__ infl, const ChainJob* __restrict__ jobs, uint32_t* __restrict__ chains,
    uint32_t njobs, uint32_t* __restrict__ depth_out) {
  extern __shared__ uint32_t dyn_lds[];
  __shared__ uint32_t wtot[BSORT_W];
  __shared__ uint32_t dmax;
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: the tile loops branch on scalars
  const ChainJob jb = jobs[j];
  const uint8_t* in = infl + jb.infl_off;
  const uint32_t n = (uint32_t)jb.n;
  const uint32_t npad = (n + 63) & ~63u;
  uint32_t* sidx = chains + jb.chain_off;
  uint32_t* bpos = sidx + npad;
  const uint32_t hbits = jb.memlevel + 7, hmask = (1u << hbits) - 1, hshift = (hbits + 2) / 3;
  const uint32_t nh = n >= 3 ? n - 2 : 0;
  LDS uint16_t* Y = (LDS uint16_t*)dyn_lds;   // positions in the current order; at the end sidx
  LDS uint16_t* cnt = Y + npad;               // [digit * BSORT_W + wave]: count, then output offset
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint32_t T = ((nh + BSORT_W - 1) / BSORT_W + 63) & ~63u;   // tile of a wave (<= 64 * MAXC)
  const uint32_t t0 = (uint32_t)wave * T < nh ? (uint32_t)wave * T : nh;
  const uint32_t t1 = t0 + T < nh ? t0 + T : nh;
  // The tile: hash << 16 | position per batch, or (MAXC > 16, the larger classes) two positions per
  // register with the hashes re-read from the input when needed.  The batch loops stay rolled: the
  // tile is indexed in registers (s_set_gpr_idx); unrolled, the compiler interleaved the batches and
  // spilled.
  constexpr bool PK = MAXC > 16;
  uint32_t v[PK ? (MAXC + 1) / 2 : MAXC];
  auto setv = [&](uint32_t c, uint32_t h, uint32_t p) {
    if constexpr (PK) { if (c & 1) v[c >> 1] |= p << 16; else v[c >> 1] = p; } else v[c] = (h << 16) | p;
  };
  auto posv = [&](uint32_t c) -> uint32_t { return PK ? (v[c >> 1] >> (16 * (c & 1))) & 0xffffu : v[c] & 0xffffu; };
  auto hashv = [&](uint32_t c) -> uint32_t { return PK ? bhash(in, posv(c), hshift, hmask) : v[c] >> 16; };
  // the tile in input order, or (reload) the wave's tile of the order in Y; every batch is assigned
#pragma unroll 1
  for (uint32_t c = 0; c < MAXC; c++) {
    const uint32_t i = t0 + 64 * c + (uint32_t)lane;
    setv(c, PK || i >= t1 ? 0u : bhash(in, i, hshift, hmask), i < t1 ? i : 0u);
  }
  auto reload = [&]() {
    __syncthreads();   // Y complete
#pragma unroll 1
    for (uint32_t c = 0; c < MAXC; c++) {
      const uint32_t i = t0 + 64 * c + (uint32_t)lane;
      const uint32_t p = i < t1 ? (uint32_t)Y[i] : 0u;
      setv(c, PK || i >= t1 ? 0u : bhash(in, p, hshift, hmask), p);
    }
  };
  // one stable counting-sort pass on digit (hash >> shift) & (2^bits - 1): tile -> Y
  auto pass = [&](uint32_t shift, uint32_t bits) {
    const uint32_t dmask = (1u << bits) - 1;
    __syncthreads();   // every wave holds its tile (Y may be overwritten), cnt free
    for (uint32_t i = tid; i < 256 * BSORT_W; i += BSORT_THREADS) cnt[i] = 0;
    __syncthreads();
#pragma unroll 1
    for (uint32_t c = 0; c < MAXC; c++) {
      if (t0 + 64 * c >= t1) break;
      const uint32_t i = t0 + 64 * c + (uint32_t)lane;
      const bool valid = i < t1;
      const uint32_t d = (hashv(c) >> shift) & dmask;
      const uint64_t pm = digit_peers(d, valid, bits);
      if (valid && (pm & lt) == 0) cnt[d * BSORT_W + wave] += (uint16_t)__popcll(pm);
    }
    __syncthreads();
    // exclusive scan of the 256 x BSORT_W counts (4 per thread, then across the block)
    const uint32_t b4 = 4u * (uint32_t)tid;
    uint32_t c4[4], s = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) { c4[u] = cnt[b4 + u]; s += c4[u]; }
    const uint32_t incl = wave_incl_scan(s);
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    // the totals of the waves before this one, lane-parallel
    const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(lane < wave ? wtot[lane] : 0u), 63);
    uint32_t e = off + incl - s;
#pragma unroll
    for (int u = 0; u < 4; u++) { cnt[b4 + u] = (uint16_t)e; e += c4[u]; }
    __syncthreads();
#pragma unroll 1
    for (uint32_t c = 0; c < MAXC; c++) {
      if (t0 + 64 * c >= t1) break;
      const uint32_t i = t0 + 64 * c + (uint32_t)lane;
      const bool valid = i < t1;
      const uint32_t d = (hashv(c) >> shift) & dmask;
      const uint64_t pm = digit_peers(d, valid, bits);
      const uint32_t base = valid ? (uint32_t)cnt[d * BSORT_W + wave] : 0u;
      if (valid) {
        Y[base + (uint32_t)__popcll(pm & lt)] = (uint16_t)posv(c);
        if ((pm & lt) == 0) cnt[d * BSORT_W + wave] = (uint16_t)(base + (uint32_t)__popcll(pm));
      }
    }
  };
  static_assert(256 * BSORT_W == 4 * BSORT_THREADS, "the scan takes 4 counters per thread");
  if (hbits <= 8) {
    pass(0, hbits);
  } else {
    pass(0, hbits - 8);
    reload();
    pass(hbits - 8, 8);
  }
  reload();
  // per wave, its contiguous tile [t0, t1) of the sorted order: bucket starts from the neighbour's hash,
  // and (when asked) the deepest bucket, as the largest distance from an element back to its bucket's
  // start (carried across batches and, after one barrier, across the waves' tiles)
  uint32_t* const last_start = wtot;   // free after the last pass's scan
  if (tid == 0) dmax = 0;
  uint32_t carry = 0, mine = 0;   // start of the bucket open at the tile's current batch (0: before the tile)
  bool before = true;              // no start seen yet in this tile
  uint32_t lead = 0;               // elements of the tile before its first start (belong to an earlier bucket)
  uint32_t hprev = t0 > 0 && t0 < t1 ? bhash(in, (uint32_t)Y[t0 - 1], hshift, hmask) : ~0u;   // element t0 - 1
#pragma unroll 1
  for (uint32_t c = 0; c < MAXC; c++) {
    if (t0 + 64 * c >= t1) break;
    const uint32_t i0 = t0 + 64 * c;
    const uint32_t i = i0 + (uint32_t)lane;
    const bool valid = i < t1;
    const uint32_t h = hashv(c);
    const uint32_t up = (uint32_t)__shfl_up((int)h, 1, 64);
    const uint32_t hp = lane ? up : hprev;
    hprev = (uint32_t)__builtin_amdgcn_readlane((int)h, 63);
    const bool first = valid && (i == 0 || hp != h);
    if (valid) bpos[i] = posv(c) | (first ? BUCKET_FIRST : 0u);
    if (depth_out) {
      const uint64_t fm = __ballot(first);
      const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
      const uint64_t at = fm & le;
      const uint32_t st = at ? i0 + (63u - (uint32_t)__builtin_clzll(at)) : carry;
      if (valid && (at || !before)) mine = mine > i - st ? mine : i - st;
      if (valid && !at && before) lead = i - t0 + 1;   // counted after the barrier
      if (fm) { carry = i0 + 63u - (uint32_t)__builtin_clzll(fm); before = false; }
    }
  }
  if (depth_out && lane == 0) last_start[wave] = before ? ~0u : carry;
  __syncthreads();   // every tile read from Y; last_start complete
  // inverse permutation through Y: Y[p] = p's index in bpos
#pragma unroll 1
  for (uint32_t c = 0; c < MAXC; c++) {
    if (t0 + 64 * c >= t1) break;
    const uint32_t i = t0 + 64 * c + (uint32_t)lane;
    if (i < t1) Y[posv(c)] = (uint16_t)i;
  }
  if (depth_out) {
    // the tile's leading elements continue the last bucket started in an earlier tile
    uint32_t prev = ~0u;
    for (int w = wave - 1; w >= 0 && prev == ~0u; w--) prev = last_start[w];
    uint32_t lm = 0;
    if (lead && prev != ~0u) lm = t0 + lead - 1u - prev;   // the last leading element is the farthest
    lm = lm > mine ? lm : mine;
    for (int d = 32; d >= 1; d >>= 1) { const uint32_t o = __shfl_xor(lm, d, 64); lm = lm > o ? lm : o; }
    if (lane == 0 && lm) atomicMax(&dmax, lm);
  }
  __syncthreads();
  for (uint32_t q = tid; q < nh; q += BSORT_THREADS) sidx[q] = Y[q];
  if (depth_out && tid == 0) depth_out[jb.dslot] = dmax;
}

// k_bucket_depth: only the deepest bucket of a (stream, memLevel) (size - 1, as k_buckets_sort
// reports it), for pairs whose trials may all be symbol replays: one returning LDS atomic per
// position on packed 16-bit hash counters (streams < 64 Ki positions), no sort, no tables written.
static constexpr uint32_t BDEPTH_THREADS = 1024;
__global__ __launch_bounds__(BDEPTH_THREADS) void k_bucket_depth(const uint8_t* __restrict__ infl,
                                                                const ChainJob* __restrict__ jobs, uint32_t njobs,
                                                                uint32_t* __restrict__ depth_out) {
  extern __shared__ uint32_t dyn_lds[];
  __shared__ uint32_t dmax;
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const int tid = threadIdx.x;
  const ChainJob jb = jobs[j];
  const uint8_t* in = infl + jb.infl_off;
  const uint32_t n = (uint32_t)jb.n;
  const uint32_t hbits = jb.memlevel + 7, hmask = (1u << hbits) - 1, hshift = (hbits + 2) / 3;
  const uint32_t nw = 1u << (hbits - 1);   // two counters per word
  LDS uint32_t* cnt = (LDS uint32_t*)dyn_lds;
  for (uint32_t w = tid; w < nw; w += BDEPTH_THREADS) cnt[w] = 0;
  if (tid == 0) dmax = 0;
  __syncthreads();
  const uint32_t nh = n >= 3 ? n - 2 : 0;
  uint32_t mine = 0;
  for (uint32_t p = tid; p < nh; p += BDEPTH_THREADS) {
    const uint32_t h = (((uint32_t)in[p] << (2 * hshift)) ^ ((uint32_t)in[p + 1] << hshift) ^ in[p + 2]) & hmask;
    const uint32_t sh = 16u * (h & 1u);
    const uint32_t old = __hip_atomic_fetch_add(&cnt[h >> 1], 1u << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t c = ((old >> sh) & 0xffffu) + 1u;
    mine = mine > c ? mine : c;
  }
  for (int d = 32; d >= 1; d >>= 1) { const uint32_t o = __shfl_xor(mine, d, 64); mine = mine > o ? mine : o; }
  if ((tid & 63) == 0 && mine) atomicMax(&dmax, mine);
  __syncthreads();
  if (tid == 0) depth_out[jb.dslot] = dmax ? dmax - 1u : 0u;
}

// ---------------------------------------------------------------------------------------------
// k_match: longest_match (Z/deflate.c:1148-1289) for every position of a trial, lanes = positions.
//
// zlib's result at position p depends on the parse only through prev_length (deflate_slow):
// the chain budget is quartered when prev_length >= good_match, and a candidate must beat
// prev_length.  The winner is the FIRST candidate reaching the maximum length, so computing the
// first-maximum from MIN_MATCH-1 and comparing it with prev_length at parse time is exact; both
// budgets are evaluated in one walk (the quarter budget sees a prefix of the same candidates).
// The window slide does not change the walk: with S the slide offset, zlib stops at nodes
// <= max(p - MAX_DIST, S), and S > 0 implies S <= p - MAX_DIST; its only trace is hash_head == S
// (NIL after the slide), which the parse checks.  nice_match is clamped to the lookahead, i.e.
// to n - p near the end; bytes beyond the input can only extend candidates that already reach
// n - p, which break at nice_match first.
#ifndef ATZ_HOLE_SLOTS
#define ATZ_HOLE_SLOTS 256   // C4 A/B (3 runs each): 1024 ~877, 512 ~878, 256 ~895, 128 ~869 MB/s (fast LDS 18.2 -> 15.1 KB)
#endif
static constexpr uint32_t HOLE_SLOTS_M = ATZ_HOLE_SLOTS;   // == HOLE_SLOTS (fast-level hash slots; a collision only makes the hole check conservative)
static_assert(HOLE_SLOTS_M <= 2048 && (HOLE_SLOTS_M & (HOLE_SLOTS_M - 1)) == 0, "slot field is 11 bits of the match entry");

// 16 bytes at byte offset x of a 4-byte aligned buffer: 5 aligned dword loads (independent, one
// round trip) joined with v_alignbyte.  Reads up to 4 bytes past x + 16 (buffers carry slack).
template <typename P>
__device__ __forceinline__ void load16(P in32, uint32_t x, uint32_t v[4]) {
  const uint32_t w = x >> 2, sh = x & 3;
  const uint32_t a0 = in32[w], a1 = in32[w + 1], a2 = in32[w + 2], a3 = in32[w + 3], a4 = in32[w + 4];
  v[0] = __builtin_amdgcn_alignbyte(a1, a0, sh);
  v[1] = __builtin_amdgcn_alignbyte(a2, a1, sh);
  v[2] = __builtin_amdgcn_alignbyte(a3, a2, sh);
  v[3] = __builtin_amdgcn_alignbyte(a4, a3, sh);
}
// number of equal leading bytes (0..16) of the 16 bytes at a and at b (pb: b's bytes if preloaded)
template <typename P>
__device__ __forceinline__ uint32_t match16(P in32, uint32_t a, uint32_t b, const uint32_t* pb, int) {
  uint32_t va[4], vb[4];
  load16(in32, a, va);
  if (pb) { vb[0] = pb[0]; vb[1] = pb[1]; vb[2] = pb[2]; vb[3] = pb[3]; }
  else load16(in32, b, vb);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = va[k] ^ vb[k];
    if (x) return 4 * k + ((uint32_t)__builtin_ctz(x) >> 3);
  }
  return 16;
}

// One trial's positions [p0, p1) on 256 lanes.  Candidate bytes are read through in32: the stream in
// HBM, or its first bytes staged in LDS (k_match_lds).
template <typename P>
__device__ __forceinline__ void match_positions(const MatchJob& jb, const uint8_t* __restrict__ in, P in32,
                                                const uint32_t* __restrict__ chains, uint2* __restrict__ R) {
  const uint32_t n = (uint32_t)jb.n, npad = (n + 63) & ~63u;
  const uint32_t* sidx = chains + jb.chain_off;
  const uint32_t* bpos = sidx + npad;
  uint2* r = R + jb.r_off;
  const uint32_t B = c_cfg[jb.level][3], nice = c_cfg[jb.level][2], Bq = B >> 2;
  const uint32_t maxdist = (1u << jb.window) - 262;
  const uint32_t hbits = jb.memlevel + 7u, hmask = (1u << hbits) - 1u, hshift = (hbits + 2u) / 3u;
  for (uint32_t p = (uint32_t)jb.p0 + threadIdx.x; p < (uint32_t)jb.p1; p += 256) {
    uint32_t bf = 2, df = 0, bq = 2, dq = 0, valid = 0, slot = 0, budget_out = 0;
    uint32_t reach = p;
    const uint32_t s0 = in[p];
    if (p + 3 <= n) {
      const uint32_t s1 = in[p + 1];
      slot = (((s0 << (2 * hshift)) ^ (s1 << hshift) ^ (uint32_t)in[p + 2]) & hmask) & (HOLE_SLOTS_M - 1);
      const uint32_t lim = p > maxdist ? p - maxdist : 0u;   // walk continues to q only if q > lim
      uint32_t idx = sidx[p];
      uint32_t e = bpos[idx];
      if (!(e & BUCKET_FIRST)) {
        e = bpos[--idx];
        uint32_t cur = e & ~BUCKET_FIRST;
        if (cur >= 1 && cur + maxdist >= p) {                 // hash_head valid
          valid = 1;
          const uint32_t left = n - p;
          const uint32_t cap = left < 258 ? left : 258u;
          const uint32_t nn = nice < cap ? nice : cap;
          uint32_t pv[4];
          load16(in32, p, pv);
          for (uint32_t i = 0;;) {
            reach = cur;
            const bool more = !(e & BUCKET_FIRST);
            const uint32_t en = more ? bpos[idx - 1] : 0u;    // next node, loaded ahead of the compare
            // exact common length, 16 bytes per round trip (any candidate that could beat bf gets
            // its exact length; zlib's quick reject only skips candidates that cannot)
            uint32_t len = match16(in32, cur, p, pv, 0);
            if (len == 16)
              while (len < cap) {
                const uint32_t l2 = match16(in32, cur + len, p + len, nullptr, 0);
                len += l2;
                if (l2 < 16) break;
              }
            if (len > cap) len = cap;
            if (len > bf) {
              bf = len; df = p - cur;
              if (i < Bq) { bq = len; dq = df; }
              if (len >= nn) break;
            }
            if (++i == B) {   // budget spent: only here can skipped positions let deflate_fast see more nodes
              budget_out = (more && (en & ~BUCKET_FIRST) > lim) ? 1u : 0u;
              break;
            }
            if (!more) break;
            e = en;
            idx--;
            cur = e & ~BUCKET_FIRST;
            if (cur <= lim) break;
          }
        }
      }
    }
    // .x = len_full:9 | dist_full:15 | input byte:8
    // .y = slow: len_quarter:9 | dist_quarter:15 | 0:7 | head valid:1
    //      fast: (p - lowest visited node):16 | 0:3 | budget spent with nodes left:1 | hash slot:11 | head valid:1
    uint2 o;
    o.x = (bf > 2 ? (bf << 23) | (df << 8) : 0u) | s0;
    if (jb.fast) o.y = ((p - reach) << 16) | (budget_out << 12) | (slot << 1) | valid;
    else o.y = (bq > 2 ? (bq << 23) | (dq << 8) : 0u) | valid;
    r[p] = o;
  }
}

__global__ __launch_bounds__(256) void k_match(const uint8_t* __restrict__ infl, const uint32_t* __restrict__ chains,
                                              uint2* __restrict__ R, const MatchJob* __restrict__ jobs) {
  const MatchJob jb = jobs[blockIdx.x];
  const uint8_t* in = infl + jb.infl_off;
  match_positions(jb, in, reinterpret_cast<const uint32_t*>(in), chains, R);   // stream bases are 256-byte aligned
}

// k_match_lds: the same walks with everything they touch in LDS.  The block stages the stream bytes
// the walks can read and, for every position q the walks can visit, its predecessor in its hash bucket
// (prev[q] = bpos[sidx[q] - 1], NIL if q opens its bucket: zlib's prev[] chain), gathered from the
// bucket arrays with all loads in flight at once.  A walk is then a chain of LDS reads instead of
// dependent HBM round trips.
// Walks from the job's positions [p0, p1) visit only nodes > p - MAX_DIST >= p0 - MAX_DIST, so the
// block stages the window [lo, p1 + 258 + 24) with lo = p0 - MAX_DIST (rounded down to a word, 0 for
// p0 <= MAX_DIST); offsets within it are 16-bit.  A node below lo ends a walk exactly as zlib's
// `cur_match > limit` test does, so it is staged as NIL.  The host cuts longer streams (C3's 64 KiB
// PNG-like streams) into position ranges whose window fits one block's LDS (launch_match).
static constexpr uint32_t PREV_NIL = 0xffffu;
#ifndef ATZ_MATCH_THREADS
#define ATZ_MATCH_THREADS 1024  // threads per k_match_lds block, all sharing the staged stream (C4: 256 ~913, 512 ~974, 1024 ~986 MB/s)
#endif
static constexpr uint32_t MATCH_THREADS = ATZ_MATCH_THREADS;
struct LdsWin {   // the staged words of [lo, ...) addressed by absolute word index
  const LDS uint32_t* p;
  uint32_t off;   // lo / 4
  __device__ __forceinline__ uint32_t operator[](uint32_t w) const { return p[w - off]; }
};
__global__ __launch_bounds__(MATCH_THREADS) void k_match_lds(const uint8_t* __restrict__ infl, const uint32_t* __restrict__ chains,
                                                  uint2* __restrict__ R, const MatchJob* __restrict__ jobs) {
  extern __shared__ uint32_t dyn_lds[];
  const MatchJob jb = jobs[blockIdx.x];
  const uint8_t* in = infl + jb.infl_off;
  const uint32_t* g32 = reinterpret_cast<const uint32_t*>(in);
  const uint32_t n = (uint32_t)jb.n, npad = (n + 63) & ~63u;
  const uint32_t* sidx = chains + jb.chain_off;
  const uint32_t* bpos = sidx + npad;
  const uint32_t maxdist = (1u << jb.window) - 262;
  const uint32_t lo = (uint32_t)jb.p0 > maxdist ? ((uint32_t)jb.p0 - maxdist) & ~3u : 0u;
  const uint32_t w0 = lo >> 2;
  const uint64_t want = jb.p1 + 258 + 24;
  const uint32_t nw = (uint32_t)(((want < n ? want : n) + 3) >> 2) - w0;   // staged words
  LDS uint32_t* l32 = (LDS uint32_t*)dyn_lds;
  LDS uint16_t* prv = (LDS uint16_t*)(l32 + nw + 8);   // prv[q - lo]
  for (uint32_t w = threadIdx.x; w < nw + 8; w += MATCH_THREADS) l32[w] = w < nw ? g32[w0 + w] : 0u;
  const uint32_t nh = n >= 3 ? n - 2 : 0;
  const uint32_t P = (uint32_t)jb.p1 < nh ? (uint32_t)jb.p1 : nh;   // candidates and walk starts are < P
  // a bucket entry's predecessor as staged: NIL when q opens its bucket or it lies below the window
  auto pred = [&](uint32_t a, uint32_t b) -> uint16_t {
    const uint32_t pq = b & ~BUCKET_FIRST;
    return ((a & BUCKET_FIRST) || pq < lo) ? (uint16_t)PREV_NIL : (uint16_t)(pq - lo);
  };
  if (P > lo && 4 * (P - lo) >= nh) {
    // most positions wanted: one coalesced pass over the bucket array (entry i's predecessor is
    // entry i - 1 unless i opens its bucket), scattered into LDS -- no dependent gathers
    for (uint32_t i0 = 0; i0 < nh; i0 += 8 * MATCH_THREADS) {
      uint32_t a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t i = i0 + MATCH_THREADS * u + threadIdx.x;
        a[u] = i < nh ? bpos[i] : BUCKET_FIRST | 0x7fffffffu;
        b[u] = (i < nh && i) ? bpos[i - 1] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t q = a[u] & ~BUCKET_FIRST;
        if (q >= lo && q < P) prv[q - lo] = pred(a[u], b[u]);
      }
    }
  } else {
    for (uint32_t q0 = lo; q0 < P; q0 += 8 * MATCH_THREADS) {
      uint32_t ix[8], a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; u++) { const uint32_t q = q0 + MATCH_THREADS * u + threadIdx.x; ix[u] = q < P ? sidx[q] : 1u; }
#pragma unroll
      for (int u = 0; u < 8; u++) { a[u] = bpos[ix[u]]; b[u] = ix[u] ? bpos[ix[u] - 1] : 0u; }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t q = q0 + MATCH_THREADS * u + threadIdx.x;
        if (q < P) prv[q - lo] = pred(a[u], b[u]);
      }
    }
  }
  __syncthreads();
  const LdsWin in32{l32, w0};
  auto byte = [&](uint32_t x) -> uint32_t { return (in32[x >> 2] >> (8 * (x & 3))) & 0xffu; };
  uint2* r = R + jb.r_off;
  const uint32_t B = c_cfg[jb.level][3], nice = c_cfg[jb.level][2], Bq = B >> 2;
  const uint32_t hbits = jb.memlevel + 7u, hmask = (1u << hbits) - 1u, hshift = (hbits + 2u) / 3u;
  for (uint32_t p = (uint32_t)jb.p0 + threadIdx.x; p < (uint32_t)jb.p1; p += MATCH_THREADS) {
    uint32_t bf = 2, df = 0, bq = 2, dq = 0, valid = 0, slot = 0, budget_out = 0;
    uint32_t reach = p;
    const uint32_t s0 = byte(p);
    if (p + 3 <= n) {
      slot = (((s0 << (2 * hshift)) ^ (byte(p + 1) << hshift) ^ byte(p + 2)) & hmask) & (HOLE_SLOTS_M - 1);
      const uint32_t lim = p > maxdist ? p - maxdist : 0u;   // walk continues to q only if q > lim
      const uint32_t h0 = prv[p - lo];
      uint32_t cur = h0 + lo;
      if (h0 != PREV_NIL && cur >= 1 && cur + maxdist >= p) {   // hash_head valid
        valid = 1;
        const uint32_t left = n - p;
        const uint32_t cap = left < 258 ? left : 258u;
        const uint32_t nn = nice < cap ? nice : cap;
        uint32_t pv[4];
        load16(in32, p, pv);
        for (uint32_t i = 0;;) {
          reach = cur;
          const uint32_t nr = prv[cur - lo];                   // next node, read ahead of the compare
          const bool more = nr != PREV_NIL;
          const uint32_t nx = nr + lo;
          uint32_t len = match16(in32, cur, p, pv, 0);
          if (len == 16)
            while (len < cap) {
              const uint32_t l2 = match16(in32, cur + len, p + len, nullptr, 0);
              len += l2;
              if (l2 < 16) break;
            }
          if (len > cap) len = cap;
          if (len > bf) {
            bf = len; df = p - cur;
            if (i < Bq) { bq = len; dq = df; }
            if (len >= nn) break;
          }
          if (++i == B) {
            budget_out = (more && nx > lim) ? 1u : 0u;
            break;
          }
          if (!more) break;
          cur = nx;
          if (cur <= lim) break;
        }
      }
    }
    uint2 o;
    o.x = (bf > 2 ? (bf << 23) | (df << 8) : 0u) | s0;
    if (jb.fast) o.y = ((p - reach) << 16) | (budget_out << 12) | (slot << 1) | valid;
    else o.y = (bq > 2 ? (bq << 23) | (dq << 8) : 0u) | valid;
    r[p] = o;
  }
}

// ---------------------------------------------------------------------------------------------
// k_trial
static constexpr int NLC = 286, NDC = 30, NBLC = 19, HEAPN = 2 * NLC + 1;
static constexpr uint32_t LOOKMIN = 262;
// fast-mode insertion ring, position mod 32768: queries are for chain nodes newer than p - MAX_DIST
// (> p - 32768, so unambiguous); an older node only ever decides "no match within reach", which
// holds whatever its (aliased) bit says, since every newer node is examined first
static constexpr uint32_t BITMAP_BITS = 32768;
static constexpr uint32_t HOLE_SLOTS = HOLE_SLOTS_M;   // fast mode: latest skipped position per hash slot

struct TreeWork {      // one tree under construction (zlib's heap / bl_count in LDS; dad and freq in TreeScratch)
  uint32_t heap[HEAPN + 1];  // packed keys (freq:16 | depth:5 | node:10) in [1, heap_len]; node ids from heap_max
  uint16_t bl_count[16];
  uint32_t blc32[16];        // gen_bitlen's per-length leaf counters (LDS atomics)
};

// Pointer-jumping scratch of gen_bitlen.  It lives in the match-table ring's LDS (the parse is
// paused while a block is flushed; the ring is reloaded from HBM afterwards), which keeps the
// trial kernels' LDS small enough for more waves per CU.
struct TreeScratch {
  uint16_t anc[2][HEAPN];    // anc[1] holds zlib's dad[] while the heap runs (read once into anc[0])
  uint8_t dep[2][HEAPN];
  uint16_t freq[NLC];        // leaf frequencies of the tree being built (forced leaves set to 1)
};

struct BitOut {
  GLOBAL uint8_t* out;
  uint64_t cap;
  uint64_t pos;      // bytes written
  uint64_t bb;       // pending bits (< 8 after every flush)
  uint32_t bc;
  // comparison against the original
  const GLOBAL uint8_t* orig;
  uint64_t clen;     // C_s
  uint64_t shortcut; // shortcut length, 0 if the shortcut does not apply
  uint64_t eq_all;   // equal bytes at positions < min(pos, C_s)
  uint64_t eq_sc;    // equal bytes at positions < min(pos, shortcut)
  int overflow;
  uint64_t cyc_tree, cyc_emit, blocks;   // diagnostics (shader clock)
  uint64_t cyc_heap, cyc_scan, cyc_send;   // diagnostics (ATZ_STEP_CLOCKS)
};

static constexpr uint32_t STAGE_WORDS = 196;   // 64 * SYM_PER_LANE * 48 / 32 + 2 (+ pad)
struct BlockFreq {       // a block's symbol frequencies, two 16-bit counts per word (symbol 2i low)
  uint32_t lfreq2[(NLC + 1) / 2];
  uint32_t dfreq2[NDC / 2];
};
struct TreeCodes {       // the three trees of the block being flushed
  uint16_t lcode[NLC]; uint8_t llen[NLC + 2];
  uint16_t dcode[NDC]; uint8_t dlen[NDC + 2];
  uint16_t bcode[NBLC]; uint8_t blen[NBLC + 2];
  uint32_t bfreq[NBLC];
  TreeWork w;
};
struct TrialShared {
  BitOut b;              // output / compare state of the trial (in LDS: the flush helpers take it by LDS reference)
  BlockFreq f;           // the block being parsed
  TreeCodes k;
  uint64_t stop_at;      // speculative rounds: the stream's stop word (SweepArgs::stopj), 0: none
  uint32_t stop_j, pad_; // the trial's place in the round
  // the bit-packing staging words (STAGE_WORDS) live in the match-table ring's LDS: they are only
  // used while a block is emitted, when the parse is paused (like TreeScratch during build_tree)
};

// INS: bits of the insertion ring, position mod INS (BITMAP_BITS serves every stream; a 16 Kibit ring
// for streams of at most 16384 positions, 2 KiB less LDS, measured slower: DESIGN.md s3.5)
template <uint32_t INS>
struct TrialSharedFast {
  static constexpr uint32_t INS_BITS = INS;
  TrialShared t;
  uint64_t ring[512];   // match-table entries around the parse window (RING_SLOW)
  uint32_t ins[INS / 32];   // insertion ring (InsRing)
  uint32_t holes[HOLE_SLOTS];   // position + 1 of the latest non-inserted position with hash & (SLOTS-1)
};

static constexpr uint32_t RING_SLOW = 512;   // >= 127 + 2 * 258 + 64: a walk never leaves the ring
struct TrialSharedSlow {
  TrialShared t;
  uint64_t ring[RING_SLOW];   // match-table entries (.x low, .y high) of the positions around the window
};
static_assert(sizeof(TreeScratch) <= RING_SLOW * sizeof(uint64_t), "tree scratch overlays the ring");
static_assert(offsetof(BitOut, cyc_scan) == offsetof(BitOut, cyc_heap) + 8, "block_trees' cyc[0], cyc[1]");
static_assert(STAGE_WORDS * 4 <= RING_SLOW * sizeof(uint64_t), "emission staging overlays the ring");

// Multi-wave trials (small blocks: memLevel <= Pipe::mw_cap, host side).  A block of lit_bufsize
// = 2^(memLevel + 6) symbols is flushed every ~128-256 positions, and the flush -- three Huffman trees
// with zlib's serial heap, then the block's bits -- costs more than parsing it, so such a trial is
// bound by its flushes (a stream's 90 block trees at memLevel 1 took most of a tail round).  Wave 0
// parses as a single-wave trial does and hands each finished block (its frequencies and bounds; the
// symbols stay in HBM) to flusher wave 1 + (block mod MW_F); the flushers build their blocks' trees
// side by side and emit them strictly in block order, each block appending to the one bit output
// and comparing it with the original.  A flusher that decides the trial (the early-exit gates, or
// the final gates after the last block) raises `stop`; the parser checks it at every hand-over.
#ifndef ATZ_MW_F
#define ATZ_MW_F 3
#endif
static constexpr int MW_F = ATZ_MW_F;   // flusher waves per multi-wave trial
struct MWSlot {                  // a finished block waiting for its flusher
  BlockFreq f;
  int64_t block_start;
  uint64_t p, S;
  uint32_t last_lit, sbase, last, seq;   // seq: block index + 1 while the slot holds a block, 0 when free
};
struct MWFlusher {
  TreeCodes k;
  TreeScratch sc;                // gen_bitlen scratch, then the emission staging
  uint64_t cyc_tree, cyc_emit;   // diagnostics
  uint64_t cyc_heap, cyc_scan;   // diagnostics (ATZ_STEP_CLOCKS; consecutive: block_trees' cyc[0], cyc[1])
};
static_assert(offsetof(MWFlusher, cyc_scan) == offsetof(MWFlusher, cyc_heap) + 8, "block_trees' cyc[0], cyc[1]");
struct MWCtl {
  uint32_t next_emit;   // index of the next block to emit
  uint32_t stop;        // the trial is decided (state), or the parser gave up (TR_NEED_R)
  uint32_t parse_done, nblocks;
  uint32_t state, hazard;
};
struct MWPart {
  MWSlot slot[MW_F];
  MWFlusher fl[MW_F];
  MWCtl ctl;
};
template <uint32_t INS>
struct TrialSharedFastMW {
  static constexpr uint32_t INS_BITS = INS;
  TrialShared t;
  uint64_t ring[512];
  uint32_t ins[INS / 32];
  uint32_t holes[HOLE_SLOTS];
  MWPart mw;
};
struct TrialSharedSlowMW {
  TrialShared t;
  uint64_t ring[RING_SLOW];
  MWPart mw;
};
static_assert(sizeof(TrialSharedFastMW<BITMAP_BITS>) <= 64 * 1024 && sizeof(TrialSharedSlowMW) <= 64 * 1024, "static LDS of a block");
template <typename T> struct HasMW { static constexpr bool value = false; };
template <uint32_t INS> struct HasMW<TrialSharedFastMW<INS>> { static constexpr bool value = true; };
template <> struct HasMW<TrialSharedSlowMW> { static constexpr bool value = true; };
__device__ __forceinline__ uint32_t ld_acq(const LDS uint32_t& x) {
  return uni(__hip_atomic_load(&x, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void st_rel(LDS uint32_t& x, uint32_t v, int lane) {
  if (lane == 0) __hip_atomic_store(&x, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct SweepArgs {
  const uint8_t* file;          // original compressed bytes
  const uint8_t* infl;          // inflated bytes
  const uint32_t* chains;       // hash buckets (k_buckets)
  const uint2* R;               // match tables (k_match)
  const StreamDev* streams;
  const Trial* trials;
  TrialRes* res;
  // speculative rounds: per stream, the lowest Trial::spec_j of the round whose result stops the stream
  // (reference's rule, main.cpp:685-700; ~0: none yet), or null
  uint32_t* stopj;
  uint8_t* out;                 // per-trial output scratch (Trial::out_off)
  uint32_t* syms;               // symbol buffers (Trial::sym_off)
  const uint32_t* adler;        // per-stream Adler-32 of the inflated data
  SweepOpts o;
  uint32_t ntrials;
};

__device__ inline uint64_t wsum64(uint64_t v) {
  for (int d = 32; d >= 1; d >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, d, 64), hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// write the `nb` bytes of the staging words (byte k = byte k & 3 of stage[k >> 2]) and compare them
// with the original on the fly.  Lane w takes word w: its 4 output bytes and 4 original bytes are
// independent accesses, all in flight together.
__device__ inline void emit_bytes_from_stage(LDS BitOut& b, const LDS uint32_t* stage, uint32_t nb, int lane) {
  uint32_t eqa = 0, eqs = 0;
  // BitOut lives in LDS: its fields read back as VGPRs, so they are made uniform explicitly (the
  // loops and branches on them are then scalar, the pointers usable as SGPR bases)
  nb = uni(nb);
  const uint64_t pos = uni(b.pos), cap = uni(b.cap), clen = uni(b.clen), sc = uni(b.shortcut);
  GLOBAL uint8_t* const out = (GLOBAL uint8_t*)(uintptr_t)uni((uint64_t)(uintptr_t)b.out);
  const GLOBAL uint8_t* const orig = (const GLOBAL uint8_t*)(uintptr_t)uni((uint64_t)(uintptr_t)b.orig);
  for (uint32_t w = (uint32_t)lane; 4 * w < nb; w += 64) {
    const uint32_t word = stage[w];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t k = 4 * w + j;
      const uint8_t x = (uint8_t)(word >> (8 * j));
      const uint64_t at = pos + k;
      if (k < nb && at < cap) out[at] = x;
      if (k < nb && at < clen) {
        const uint32_t e = orig[at] == x ? 1u : 0u;
        eqa += e;
        if (at < sc) eqs += e;
      }
    }
  }
  b.eq_all += wsum64(eqa);
  b.eq_sc += wsum64(eqs);
  if (pos + nb > cap) b.overflow = 1;
  b.pos = pos + nb;
}

// scalar emission (block headers, tree descriptions): bits accumulate in bb; whole bytes go out in
// groups through the staging words.
__device__ inline void put_bits(LDS BitOut& b, LDS uint32_t* stage, uint32_t v, uint32_t n, int lane) {
  const uint32_t bc = uni(b.bc) + n;
  const uint64_t bb = uni(b.bb) | ((uint64_t)uni(v) << uni(b.bc));
  if (bc >= 32) {
    if (lane == 0) stage[0] = (uint32_t)bb;
    emit_bytes_from_stage(b, stage, 4, lane);
    b.bb = bb >> 32;
    b.bc = bc - 32;
  } else {
    b.bb = bb;
    b.bc = bc;
  }
}
__device__ inline void flush_bits_bytes(LDS BitOut& b, LDS uint32_t* stage, int lane) {  // whole bytes only
  const uint32_t bc = uni(b.bc), nb = bc >> 3;
  if (!nb) return;
  const uint64_t bb = uni(b.bb);
  if (lane == 0) { stage[0] = (uint32_t)bb; stage[1] = (uint32_t)(bb >> 32); }
  emit_bytes_from_stage(b, stage, nb, lane);
  b.bb = nb >= 8 ? 0 : (bb >> (8 * nb));
  b.bc = bc - 8 * nb;
}
__device__ inline void windup(LDS BitOut& b, LDS uint32_t* stage, int lane) {  // bi_windup
  flush_bits_bytes(b, stage, lane);
  if (uni(b.bc)) {
    if (lane == 0) stage[0] = (uint32_t)b.bb;
    emit_bytes_from_stage(b, stage, 1, lane);
    b.bb = 0; b.bc = 0;
  }
}

// ---- Huffman tree construction, Z/trees.c:453-699 ----
// zlib's heap algorithm is kept step for step (its tie-breaks decide the code lengths).  Heap
// entries are packed keys freq:16 | depth:5 | node:10, so zlib's smaller() (freq, then depth <=)
// is one compare of key >> 10 and a sift-down level is one ds_read2 of the sibling pair.
__device__ __forceinline__ uint32_t tkey(uint32_t f, uint32_t d, uint32_t n) { return (f << 15) | (d << 10) | n; }

// pqdownheap (Z/trees.c:453-476).  One lane-parallel LDS read gathers the 62 descendants of k
// within 5 levels (lanes [2^t - 2, 2^(t+1) - 2) hold level t); the sift path through them is
// chosen with v_readlane, so a sift-down costs one LDS round trip per 5 levels, not one per level.
__device__ __forceinline__ void pq_down(LDS uint32_t* heap, int heap_len, int k, int lane) {
  const uint32_t v = uni(heap[k]);
  const uint32_t vk = v >> 10;
  const int t_l = 31 - __builtin_clz((uint32_t)lane + 2u);   // level of this lane (6 for lanes 62, 63)
  const int off_l = lane + 2 - (1 << t_l);
  for (;;) {
    if (2 * k > heap_len) break;
    const int idx = (k << t_l) + off_l;
    const uint32_t g = (t_l <= 5 && idx <= heap_len) ? heap[idx] : 0xffffffffu;
    int p = k;
    bool stop = false;
    // A child past heap_len reads ~0u from the gather, a key above every real one, so v stops there:
    // the stop test also ends the path at the heap's bottom.  lj, the gathered lane of the left
    // child, follows the path: a lane's left child is lane 2 * lane + 2 (k itself counts as -1).
    int lj = 0;
#pragma unroll
    for (int t = 1; t <= 5; t++) {
      // the right child (ties go right)
      const uint32_t hl = (uint32_t)__builtin_amdgcn_readlane((int)g, lj);
      const uint32_t hr = (uint32_t)__builtin_amdgcn_readlane((int)g, lj + 1);
      const uint32_t c = (hr >> 10) <= (hl >> 10) ? 1u : 0u;
      const uint32_t hj = c ? hr : hl;
      if (vk <= (hj >> 10)) { stop = true; break; }
      heap[p] = hj;
      p = 2 * p + (int)c;
      lj = 2 * (lj + (int)c) + 2;
    }
    k = p;
    if (stop) break;
  }
  heap[k] = v;
}

// Arguments of a non-inlined function are divergent to the compiler (any caller could pass
// per-lane values), so a uniform argument used in control flow is re-asserted with readfirstlane:
// the loops over it then run on SGPRs and scalar branches instead of exec-mask bookkeeping.
template <typename T> __device__ __forceinline__ const CONSTANT T* uni_ptr(const CONSTANT T* p) {
  return (const CONSTANT T*)(uintptr_t)uni((uint64_t)(uintptr_t)p);
}
template <typename T> __device__ __forceinline__ const GLOBAL T* uni_ptr(const GLOBAL T* p) {
  return (const GLOBAL T*)(uintptr_t)uni((uint64_t)(uintptr_t)p);
}

struct TreeRes {
  int max_code;
  uint64_t d_opt, d_static;   // increments of opt_len / static_len (modulo 2^64, as zlib's ulg sums)
};

// build_tree + gen_bitlen (Z/trees.c:488-565, 617-699) from sc.freq[0..elems).  Leaves' lengths land
// in lenv, bl_count in w.bl_count; returns max_code and the opt_len / static_len increments (in
// registers: references to the caller's locals would put them in scratch memory).
__device__ __noinline__ TreeRes build_tree(LDS TreeWork& w, LDS TreeScratch& sc, LDS uint8_t* lenv, int elems, int max_length, const CONSTANT uint8_t* xbits,
                                           int xbase, const CONSTANT uint8_t* stlen, LDS uint64_t& cyc_heap, int lane) {
  elems = (int)uni((uint32_t)elems);
  max_length = (int)uni((uint32_t)max_length);
  xbase = (int)uni((uint32_t)xbase);
  xbits = uni_ptr(xbits);
  stlen = uni_ptr(stlen);
  uint64_t opt_len = 0, static_len = 0;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  LDS uint32_t* const heap = w.heap;
  // leaves enter heap[1..] in increasing symbol order (Z/trees.c:631-638)
  int heap_len = 0, max_code = -1;
  for (int g = 0; g < elems; g += 64) {
    const int n = g + lane;
    const uint32_t f = n < elems ? sc.freq[n] : 0u;
    const uint64_t m = __ballot(f != 0);
    if (f) heap[heap_len + 1 + __popcll(m & lt)] = tkey(f, 0, (uint32_t)n);
    else if (n < elems) lenv[n] = 0;
    if (m) max_code = g + 63 - __clzll((long long)m);
    heap_len += __popcll(m);
  }
  // force at least two codes (Z/trees.c:645-653)
  while (heap_len < 2) {
    const int node = max_code < 2 ? ++max_code : 0;
    ++heap_len;
    if (lane == 0) { heap[heap_len] = tkey(1, 0, (uint32_t)node); sc.freq[node] = 1; }
    opt_len--;
    if (stlen) static_len -= stlen[node];
  }
  const uint64_t ch0 = STEP_CLOCK();
  int heap_max = HEAPN;
  uint32_t node = (uint32_t)elems;
  uint32_t root;
  if (heap_len <= 63) {
    // The whole heap in one VGPR (heap[i] in lane i): every sift level is two v_readlane and a
    // lane select, no LDS round trip.  Same steps, same tie-breaks as the LDS heap below.
    // Lanes 0 and past heap_len hold ~0u (a key above every real one), so a sift level reads both
    // children without testing j < len (lane 64 wraps to lane 0); the loop has one exit.
    uint32_t H = lane >= 1 && lane <= heap_len ? heap[lane] : 0xffffffffu;
    auto rd = [&](int i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)H, i); };
    auto wr = [&](int i, uint32_t v) { H = lane == i ? v : H; };
    auto down = [&](int len, int k) {
      const uint32_t v = rd(k), vk = v >> 10;
      int j = k << 1;
      bool go = j <= len;
      while (go) {
        const uint32_t a = rd(j), b = rd(j + 1);
        const uint32_t c = (b >> 10) <= (a >> 10) ? 1u : 0u;   // ties go right
        const uint32_t hj = c ? b : a;
        j += (int)c;
        go = vk > (hj >> 10);
        if (go) { wr(k, hj); k = j; j = k << 1; go = j <= len; }
      }
      wr(k, v);
    };
    for (int n = heap_len / 2; n >= 1; n--) down(heap_len, n);
    do {
      const uint32_t kn = rd(1);
      wr(1, rd(heap_len));
      wr(heap_len, 0xffffffffu);
      heap_len--;
      down(heap_len, 1);
      const uint32_t km = rd(1);
      const uint32_t dn = (kn >> 10) & 31u, dm = (km >> 10) & 31u;
      if (lane == 0) {
        heap[--heap_max] = kn & 1023u;
        heap[--heap_max] = km & 1023u;
        sc.anc[1][kn & 1023u] = (uint16_t)node;
        sc.anc[1][km & 1023u] = (uint16_t)node;
      } else {
        heap_max -= 2;
      }
      wr(1, tkey((kn >> 15) + (km >> 15), (dn >= dm ? dn : dm) + 1u, node));
      node++;
      down(heap_len, 1);
    } while (heap_len >= 2);
    root = rd(1) & 1023u;
  } else {
  for (int n = heap_len / 2; n >= 1; n--) pq_down(heap, heap_len, n, lane);
  // combine the two least frequent nodes until one is left (Z/trees.c:663-690)
  do {
    const uint32_t kn = uni(heap[1]);
    heap[1] = uni(heap[heap_len]);
    heap_len--;
    pq_down(heap, heap_len, 1, lane);
    const uint32_t km = uni(heap[1]);
    const uint32_t dn = (kn >> 10) & 31u, dm = (km >> 10) & 31u;
    if (lane == 0) {
      heap[--heap_max] = kn & 1023u;
      heap[--heap_max] = km & 1023u;
      sc.anc[1][kn & 1023u] = (uint16_t)node;
      sc.anc[1][km & 1023u] = (uint16_t)node;
    } else {
      heap_max -= 2;
    }
    heap[1] = tkey((kn >> 15) + (km >> 15), (dn >= dm ? dn : dm) + 1u, node);
    node++;
    pq_down(heap, heap_len, 1, lane);
  } while (heap_len >= 2);
  root = uni(heap[1]) & 1023u;
  }
  if (lane == 0) cyc_heap += STEP_CLOCK() - ch0;
  --heap_max;
  if (lane == 0) heap[heap_max] = root;
  // gen_bitlen: every node's depth by pointer jumping over dad[] (lane-parallel, depth <= 31 so
  // five rounds), bits = min(depth, max_length); zlib counts the nodes it had to cap (overflow).
  const int nn = (int)node;   // node ids 0..nn-1 (leaves not in the tree are never read)
  for (int i = lane; i < nn; i += 64) {
    const bool in_tree = i >= elems || (i <= max_code && sc.freq[i] != 0);
    const bool r = (uint32_t)i == root || !in_tree;   // leaves outside the tree: never followed
    sc.anc[0][i] = r ? (uint16_t)root : sc.anc[1][i];
    sc.dep[0][i] = r ? 0 : 1;
  }
  int cur = 0;
  for (int round = 0; round < 5; round++) {
    for (int i = lane; i < nn; i += 64) {
      const uint32_t a = sc.anc[cur][i];
      sc.dep[cur ^ 1][i] = (uint8_t)(sc.dep[cur][i] + sc.dep[cur][a]);
      sc.anc[cur ^ 1][i] = sc.anc[cur][a];
    }
    cur ^= 1;
  }
  // bl_count by LDS atomics: one ds_add per 64 nodes instead of 15 ballots (the adds to one
  // counter serialise in the LDS pipe, not in the issue slots)
  if (lane < 16) w.blc32[lane] = 0;
  int overflow = 0;
  for (int g = 0; g < nn; g += 64) {
    const int i = g + lane;
    bool in_tree = false;
    uint32_t bits = 0;
    if (i < nn) {
      in_tree = i >= elems || (i <= max_code && sc.freq[i] != 0);   // internal node or leaf in the heap
      bits = sc.dep[cur][i];
    }
    const bool capped = in_tree && (uint32_t)i != root && bits > (uint32_t)max_length;
    overflow += __popcll(__ballot(capped));
    if (bits > (uint32_t)max_length) bits = (uint32_t)max_length;
    const bool leaf = in_tree && i <= max_code;
    if (leaf) {
      lenv[i] = (uint8_t)bits;
      __hip_atomic_fetch_add(&w.blc32[bits], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  uint32_t blc = lane >= 1 && lane < 16 ? w.blc32[lane] : 0u;   // lane b: bl_count[b]
  if (overflow) {   // Z/trees.c:531-564 (rare): sequential, as zlib
    auto bl = [&](int b) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)blc, b); };
    auto blset = [&](int b, uint32_t v) { blc = lane == b ? v : blc; };
    do {
      int bits = max_length - 1;
      while (bl(bits) == 0) bits--;
      blset(bits, bl(bits) - 1);
      blset(bits + 1, bl(bits + 1) + 2);
      blset(max_length, bl(max_length) - 1);
      overflow -= 2;
    } while (overflow > 0);
    int h = HEAPN;
    for (int bits = max_length; bits != 0; bits--) {
      uint32_t cnt = bl(bits);
      while (cnt != 0) {
        const uint32_t m = uni(heap[--h]);
        if ((int)m > max_code) continue;
        if (lane == 0) lenv[m] = (uint8_t)bits;
        cnt--;
      }
    }
  }
  if (lane < 16) w.bl_count[lane] = (uint16_t)blc;
  // opt_len / static_len over the final lengths (= zlib's running sums + fix-up terms)
  uint64_t o = 0, st = 0;
  for (int n = lane; n < elems && n <= max_code; n += 64) {
    const uint32_t f = sc.freq[n];
    if (f) {
      const uint32_t l = lenv[n];
      const uint32_t xb = (xbits && n >= xbase) ? xbits[n - xbase] : 0u;
      o += (uint64_t)f * (l + xb);
      if (stlen) st += (uint64_t)f * (stlen[n] + xb);
    }
  }
  opt_len += wsum64(o);
  if (stlen) static_len += wsum64(st);
  return TreeRes{max_code, opt_len, static_len};
}

// gen_codes (Z/trees.c:575-607), lane-parallel: the codes of one length are consecutive in
// symbol order, so a ballot per length ranks the symbols.
__device__ __noinline__ void gen_codes(const LDS TreeWork& w, int max_code, LDS uint16_t* codes, LDS uint8_t* lens,
                                       int lane) {
  max_code = (int)uni((uint32_t)max_code);
  // lane b: next_code[b] = sum over i < b of bl_count[i] << (b - i), i.e. the exclusive prefix sum of
  // bl_count[i] << (15 - i), shifted down by 15 - b (one DPP scan instead of zlib's 15-step loop)
  const bool lb = lane >= 1 && lane <= 15;
  const uint32_t bc = lb ? (uint32_t)w.bl_count[lane] : 0u;
  const uint32_t wv = bc << ((15 - lane) & 15);
  uint32_t nc = lb ? (wave_incl_scan(wv) - wv) >> (15 - lane) : 0u;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t present = __ballot(bc != 0);   // lengths in use
  for (int g = 0; g <= max_code; g += 64) {
    const int n = g + lane;
    const uint32_t l = n <= max_code ? lens[n] : 0u;   // build_tree left the lengths here
    uint32_t mine = 0;
    for (uint64_t pm = present; pm; pm &= pm - 1) {
      const int b = __ffsll((unsigned long long)pm) - 1;
      const uint64_t m = __ballot(l == (uint32_t)b);
      if (!m) continue;
      const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)nc, b);
      if (l == (uint32_t)b) mine = base + (uint32_t)__popcll(m & lt);
      if (lane == b) nc += (uint32_t)__popcll(m);
    }
    if (n <= max_code && l) codes[n] = (uint16_t)(__builtin_bitreverse32(mine) >> (32 - l));
  }
}

__device__ __forceinline__ uint32_t len_code(uint32_t len) {   // _length_code[len], len = length - 3
  if (len < 8) return len;
  if (len == 255) return 28;
  const uint32_t lg = 31u - (uint32_t)__clz(len);
  return 4u * (lg - 1u) + ((len >> (lg - 2u)) & 3u);
}
__device__ __forceinline__ uint32_t dist_code(uint32_t d) {    // d_code(d), d = distance - 1
  if (d < 4) return d;
  const uint32_t lg = 31u - (uint32_t)__clz(d);
  return 2u * lg + ((d >> (lg - 1u)) & 1u);
}
// RFC 1951 extra bits / bases in closed form (no table loads per symbol)
__device__ __forceinline__ uint32_t lcode_extra(uint32_t c) { return (c < 8 || c == 28) ? 0u : (c - 4) >> 2; }
__device__ __forceinline__ uint32_t lcode_base(uint32_t c) {   // base_length[c] (length - 3)
  return c < 8 ? c : c == 28 ? 255u : ((4 + (c & 3)) << lcode_extra(c));
}
__device__ __forceinline__ uint32_t dcode_extra(uint32_t d) { return d < 2 ? 0u : (d >> 1) - 1; }
__device__ __forceinline__ uint32_t dcode_base(uint32_t d) { return d < 2 ? d : ((2 + (d & 1)) << dcode_extra(d)); }  // base_dist[d]


// Early-exit test after output progress: returns TR_* state to stop with, or ~0u to continue.
__device__ inline uint32_t early_exit(const LDS BitOut& b, const SweepOpts& o, uint64_t best_ident, bool full_needed) {
  if (uni((uint32_t)b.overflow)) return TR_OVERFLOW;
  if (full_needed) return ~0u;
  const uint64_t pos = uni(b.pos), clen = uni(b.clen), sc = uni(b.shortcut);
  if (sc) {
    uint64_t seen = pos < sc ? pos : sc;
    uint64_t mism = seen - uni(b.eq_sc);
    uint64_t thr = o.shortcut_len - o.recomp_tresh;   // uint64 wrap as in main.cpp:649
    if (thr > sc || mism > sc - thr) return TR_SHORTCUT;
  }
  if (pos > clen + o.sizediff_tresh) return TR_SIZEDIFF;
  uint64_t seen = pos < clen ? pos : clen;
  if (clen - (seen - uni(b.eq_all)) <= best_ident) return TR_CANT_BEAT;
  return ~0u;
}

// Lane-parallel compress_block (Z/trees.c:1060-1105): 128 symbols per step, two per lane (one
// 8-byte load), bit offsets by a wave prefix sum, words assembled with LDS atomics.
static constexpr uint32_t SYM_PER_LANE = 2;
template <typename C16, typename C8>
__device__ __forceinline__ void sym_bits(uint32_t sy, bool valid, bool end, C16 lc, C8 ll, C16 dc, C8 dl,
                                         uint64_t& v, uint32_t& nb) {
  v = 0; nb = 0;
  if (valid) {
    uint32_t dist = sy >> 8;
    const uint32_t c = sy & 0xff;
    if (dist == 0) {
      v = lc[c]; nb = ll[c];
    } else {
      const uint32_t code = len_code(c);
      v = lc[code + 257]; nb = ll[code + 257];
      const uint32_t xe = lcode_extra(code);
      if (xe) { v |= (uint64_t)(c - lcode_base(code)) << nb; nb += xe; }
      dist--;
      const uint32_t dcd = dist_code(dist);
      v |= (uint64_t)dc[dcd] << nb; nb += dl[dcd];
      const uint32_t xd = dcode_extra(dcd);
      if (xd) { v |= (uint64_t)(dist - dcode_base(dcd)) << nb; nb += xd; }
    }
  } else if (end) {
    v = lc[256]; nb = ll[256];   // END_BLOCK
  }
}
__device__ __forceinline__ void stage_or(LDS uint32_t* stage, uint32_t off, uint64_t v, uint32_t nb) {
  if (!nb) return;
  const uint32_t wi = off >> 5, sh = off & 31;
  const uint64_t lo = v << sh;                       // bits 0..63 of the shifted value
  const uint32_t hi = sh ? (uint32_t)(v >> (64 - sh)) : 0;
  __atomic_fetch_or(&stage[wi], (uint32_t)lo, __ATOMIC_RELAXED);
  if ((uint32_t)(lo >> 32)) __atomic_fetch_or(&stage[wi + 1], (uint32_t)(lo >> 32), __ATOMIC_RELAXED);
  if (hi) __atomic_fetch_or(&stage[wi + 2], hi, __ATOMIC_RELAXED);
}
// scan_tree / send_tree (Z/trees.c:705-799), lane-parallel.  zlib walks the code lengths
// ln[0..max_code] once, cutting each run of equal lengths into chunks; the cut points depend only
// on the run: a run of v != 0 is cut after 7, then every 6 elements (max_count 7, then 6 while the
// run goes on); a run of zeros every 138.  A chunk of `cnt` elements is coded as cnt literal v codes
// if cnt < min_count (4 for the first chunk of a nonzero run, else 3), else as [v] REP_3_6+2 bits
// (v only in the run's first chunk, where prevlen != v), REPZ_3_10+3 or REPZ_11_138+7.  So every
// element finds its run (ballot masks of run starts; max_code + 1 is zlib's guard) and a chunk's
// first element contributes the chunk: send = its bits in element order, else its bl_tree counts.
// send: the chunks' bits go into the staging words at bit offset `off` on (in element order); returns
// the offset after them.
__device__ uint32_t rle_tree(LDS TreeCodes& s, LDS uint32_t* stage, const LDS uint8_t* ln, int max_code, bool send,
                             uint32_t off, int lane) {
  const int N = max_code + 1;   // elements; position N acts as a run start (the guard)
  const int G = N / 64 + 1;     // groups covering 0..N (N <= 286: at most 5)
  uint64_t M[5];
#pragma unroll
  for (int g = 0; g < 5; g++) {
    M[g] = 0;
    if (g < G) {
      const int n = 64 * g + lane;
      bool st = false;
      if (n == 0 || n == N) st = true;
      else if (n < N) st = ln[n] != ln[n - 1];
      M[g] = __ballot(st);
    }
  }
  for (int g = 0; g < G; g++) {
    const int n = 64 * g + lane;
    uint64_t v64 = 0;
    uint32_t nb = 0;
    if (n < N) {
      // run start: highest start <= n; run end: lowest start > n
      int st = -1, en = -1;
      const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
#pragma unroll
      for (int h = 4; h >= 0; h--)
        if (st < 0 && h <= g) {
          const uint64_t m = h == g ? (M[h] & le) : M[h];
          if (m) st = 64 * h + 63 - __clzll((long long)m);
        }
#pragma unroll
      for (int h = 0; h < 5; h++)
        if (en < 0 && h >= g) {
          const uint64_t m = h == g ? (M[h] & ~le) : M[h];
          if (m) en = 64 * h + __ffsll((unsigned long long)m) - 1;
        }
      const uint32_t v = ln[n];
      const int k = n - st, R = en - st;
      int cnt = 0, minc = 3;
      bool first = false;
      if (v != 0) {
        if (k == 0) { cnt = R < 7 ? R : 7; minc = 4; first = true; }
        else if (k >= 7 && (k - 7) % 6 == 0) cnt = R - k < 6 ? R - k : 6;
      } else if (k % 138 == 0) {
        cnt = R - k < 138 ? R - k : 138;
      }
      if (cnt) {
        if (!send) {
          if (cnt < minc) __atomic_fetch_add(&s.bfreq[v], (uint32_t)cnt, __ATOMIC_RELAXED);
          else if (v != 0) {
            if (first) __atomic_fetch_add(&s.bfreq[v], 1u, __ATOMIC_RELAXED);
            __atomic_fetch_add(&s.bfreq[16], 1u, __ATOMIC_RELAXED);
          } else __atomic_fetch_add(&s.bfreq[cnt <= 10 ? 17 : 18], 1u, __ATOMIC_RELAXED);
        } else {
          const uint32_t cv = s.bcode[v], cl = s.blen[v];
          if (cnt < minc) {
            for (int q = 0; q < cnt; q++) { v64 |= (uint64_t)cv << nb; nb += cl; }
          } else if (v != 0) {
            if (first) { v64 = cv; nb = cl; }
            v64 |= (uint64_t)s.bcode[16] << nb; nb += s.blen[16];
            v64 |= (uint64_t)(cnt - (first ? 1 : 0) - 3) << nb; nb += 2;
          } else if (cnt <= 10) {
            v64 = s.bcode[17]; nb = s.blen[17];
            v64 |= (uint64_t)(cnt - 3) << nb; nb += 3;
          } else {
            v64 = s.bcode[18]; nb = s.blen[18];
            v64 |= (uint64_t)(cnt - 11) << nb; nb += 7;
          }
        }
      }
    }
    if (send) {
      const uint32_t incl = wave_incl_scan(nb);
      stage_or(stage, off + incl - nb, v64, nb);
      off += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
  }
  return off;
}

// The trial's outcome gates (early_exit) are monotone in the output emitted so far, so they are
// tested after every step: a bailed trial stops inside its first block instead of emitting all of
// it.  Returns true when the trial is decided (the caller re-evaluates early_exit).
template <typename C16, typename C8>
__device__ bool compress_block(LDS BitOut& b, LDS uint32_t* stage, const GLOBAL uint32_t* syms, uint32_t nsym,
                               C16 lc, C8 ll, C16 dc, C8 dl, const SweepOpts& o, uint64_t best_ident,
                               bool full_needed, int lane) {
  // the symbols were stored by other lanes during the parse: order those HBM stores before the reads
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  for (uint32_t base = 0; base <= nsym; base += 64 * SYM_PER_LANE) {
    const uint32_t k0 = base + SYM_PER_LANE * (uint32_t)lane;
    // symbol buffers are 256-byte aligned with >= 4 KiB slack after the last one: the pair load
    // may read past nsym (those values are not used)
    const uint64_t sp = *(const GLOBAL uint64_t*)(syms + k0);
    uint64_t v0, v1;
    uint32_t n0, n1;
    sym_bits((uint32_t)sp, k0 < nsym, k0 == nsym, lc, ll, dc, dl, v0, n0);
    sym_bits((uint32_t)(sp >> 32), k0 + 1 < nsym, k0 + 1 == nsym, lc, ll, dc, dl, v1, n1);
    const uint32_t nb = n0 + n1;
    // exclusive prefix sum of bit lengths
    const uint32_t incl = wave_incl_scan(nb);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (total == 0) break;
    // stage words: word 0..1 seeded with the pending bits
    for (int i = lane; i < (int)STAGE_WORDS; i += 64) stage[i] = 0;
    const uint32_t bc = uni(b.bc);
    if (lane == 0) { stage[0] = (uint32_t)b.bb; stage[1] = (uint32_t)(b.bb >> 32); }
    const uint32_t off = bc + incl - nb;
    stage_or(stage, off, v0, n0);
    stage_or(stage, off + n0, v1, n1);
    const uint32_t all = bc + total;
    const uint32_t full = all >> 3;
    emit_bytes_from_stage(b, stage, full, lane);
    const uint32_t rem = all & 7;
    const uint32_t lastw = stage[full >> 2];
    b.bb = rem ? ((lastw >> (8 * (full & 3))) & 0xff) & ((1u << rem) - 1) : 0;
    b.bc = rem;
    if (!full_needed && early_exit(b, o, best_ident, false) != ~0u) return true;
  }
  return false;
}

struct Lz {
  // parameters
  uint32_t level, kind, wsize, maxdist, lbs, good, lazy, nice, chain;
  // absolute-position state
  // 32-bit positions (streams < 2 GiB, checked on the host): the scalar unit has no 64-bit
  // ordered compares, so 64-bit positions would turn every comparison into VALU + VCC round trips
  uint32_t n;           // I_s
  uint32_t p;           // strstart
  uint32_t lookahead;
  uint32_t S;           // total window slide
  uint32_t block_start; // absolute
  uint32_t match_start, prev_match;
  uint32_t match_length, prev_length;
  int match_available;
  uint32_t last_lit;
  uint32_t nsym;
};

// Double-buffered lane-resident window over the trial's match table: lane l holds the entry of
// position rb + l and the entry of rb + 64 + l is in flight, so the wave-uniform parse reads its
// per-position data with v_readlane and the next HBM round trip overlaps ~64 positions of work.
// fill_window bookkeeping (Z/deflate.c:1390-1532) on absolute positions
__device__ __forceinline__ void fill(Lz& z) {
  do {
    uint32_t sw = z.p - z.S;
    uint32_t more = 2u * z.wsize - z.lookahead - sw;
    if (sw >= z.wsize + z.maxdist) { z.S += z.wsize; more += z.wsize; }
    uint32_t rd = z.p + z.lookahead;
    if (rd >= z.n) break;
    uint32_t k = z.n - rd;
    if (k > more) k = more;
    z.lookahead += k;
  } while (z.lookahead < LOOKMIN && z.p + z.lookahead < z.n);
}

// common prefix length of in[a..] and in[b..] starting at offset `from`, capped at `cap` (lanes)
__device__ inline uint32_t common_len(const uint8_t* in, uint64_t a, uint64_t b, uint32_t from, uint32_t cap,
                                      int lane) {
  for (uint32_t k0 = from; k0 < cap; k0 += 64) {
    uint32_t k = k0 + lane;
    bool ne = k < cap && in[a + k] != in[b + k];
    if (k >= cap) ne = true;
    uint64_t m = __ballot(ne);
    if (m) {
      uint32_t f = k0 + (uint32_t)(__ffsll((unsigned long long)m) - 1);
      return f < cap ? f : cap;
    }
  }
  return cap;
}

// _tr_flush_block (Z/trees.c:907-1004), in two parts: the trees of a block (from its frequencies
// alone) and its emission (in block order: it appends to the trial's bit output).  A single-wave
// trial runs both back to back (flush_block); a multi-wave trial builds the trees of several blocks
// at once on its flusher waves and emits them in order (trial_flusher).
struct BlockPlan {
  uint64_t opt_lenb, static_lenb;
  int lmax, dmax, max_blindex;
};
// cyc[0] / cyc[1]: the caller's heap / scan_tree clock counters (ATZ_STEP_CLOCKS), its own: a
// multi-wave trial's flushers build trees at the same time
__device__ __noinline__ BlockPlan block_trees(const LDS BlockFreq& f, LDS TreeCodes& s, LDS TreeScratch& sc, LDS uint64_t* cyc,
                                              uint32_t level, uint64_t stored_len, int lane) {
  level = uni(level);
  stored_len = uni(stored_len);
  BlockPlan pl{};
  uint64_t opt_len = 0, static_len = 0;
  if (level > 0) {
    // literal/length tree
    for (int i = lane; i < NLC; i += 64) sc.freq[i] = (uint16_t)(f.lfreq2[i >> 1] >> (16 * (i & 1)));
    TreeRes r = build_tree(s.w, sc, s.llen, NLC, 15, (const CONSTANT uint8_t*)c_xlb, 257, (const CONSTANT uint8_t*)c_t.st_llen,
                           cyc[0], lane);
    pl.lmax = (int)uni((uint32_t)r.max_code);
    opt_len += uni(r.d_opt);
    static_len += uni(r.d_static);
    gen_codes(s.w, pl.lmax, s.lcode, s.llen, lane);
    for (int i = pl.lmax + 1 + lane; i < NLC + 2; i += 64) s.llen[i] = 0;
    // distance tree
    for (int i = lane; i < NDC; i += 64) sc.freq[i] = (uint16_t)(f.dfreq2[i >> 1] >> (16 * (i & 1)));
    r = build_tree(s.w, sc, s.dlen, NDC, 15, (const CONSTANT uint8_t*)c_xdb, 0, (const CONSTANT uint8_t*)c_t.st_dlen,
                   cyc[0], lane);
    pl.dmax = (int)uni((uint32_t)r.max_code);
    opt_len += uni(r.d_opt);
    static_len += uni(r.d_static);
    gen_codes(s.w, pl.dmax, s.dcode, s.dlen, lane);
    for (int i = pl.dmax + 1 + lane; i < NDC + 2; i += 64) s.dlen[i] = 0;
    // bit length tree
    for (int i = lane; i < NBLC; i += 64) s.bfreq[i] = 0;
    const uint64_t cs0 = STEP_CLOCK();
    rle_tree(s, nullptr, s.llen, pl.lmax, false, 0, lane);
    rle_tree(s, nullptr, s.dlen, pl.dmax, false, 0, lane);
    if (lane == 0) cyc[1] += STEP_CLOCK() - cs0;
    for (int i = lane; i < NBLC; i += 64) sc.freq[i] = (uint16_t)s.bfreq[i];
    r = build_tree(s.w, sc, s.blen, NBLC, 7, (const CONSTANT uint8_t*)c_xblb, 0, nullptr, cyc[0], lane);
    const int bmax = (int)uni((uint32_t)r.max_code);
    opt_len += uni(r.d_opt);
    gen_codes(s.w, bmax, s.bcode, s.blen, lane);
    for (int i = bmax + 1 + lane; i < NBLC + 2; i += 64) s.blen[i] = 0;
    int mb;
    for (mb = NBLC - 1; mb >= 3; mb--)
      if (s.blen[bl_order((uint32_t)mb)] != 0) break;
    pl.max_blindex = mb;
    opt_len += 3 * ((uint64_t)mb + 1) + 5 + 5 + 4;
    pl.opt_lenb = (opt_len + 3 + 7) >> 3;
    pl.static_lenb = (static_len + 3 + 7) >> 3;
    if (pl.static_lenb <= pl.opt_lenb) pl.opt_lenb = pl.static_lenb;
  } else {
    pl.opt_lenb = pl.static_lenb = stored_len + 5;
  }
  return pl;
}

// The block's bits, compared with the original as they are written.  Returns the overlay-hazard bit.
__device__ __noinline__ uint32_t block_emit(LDS TreeCodes& s, LDS uint32_t* stage, LDS BitOut& b, const GLOBAL uint32_t* syms,
                                            const GLOBAL uint8_t* in, int64_t block_start, uint64_t p, uint64_t S,
                                            uint32_t last_lit, uint32_t lbs, int last, SweepOpts opt, uint64_t best_ident,
                                            bool full_needed, uint64_t opt_lenb, uint64_t static_lenb, int lmax, int dmax,
                                            int max_blindex, int lane) {
  syms = uni_ptr(syms);
  in = uni_ptr(in);
  block_start = (int64_t)uni((uint64_t)block_start);
  p = uni(p);
  S = uni(S);
  last_lit = uni(last_lit);
  lbs = uni(lbs);
  last = (int)uni((uint32_t)last);
  opt.recomp_tresh = uni(opt.recomp_tresh);
  opt.sizediff_tresh = uni(opt.sizediff_tresh);
  opt.shortcut_len = uni(opt.shortcut_len);
  opt.mismatch_tol = uni(opt.mismatch_tol);
  best_ident = uni(best_ident);
  full_needed = uni((uint32_t)full_needed) != 0;
  opt_lenb = uni(opt_lenb);
  static_lenb = uni(static_lenb);
  lmax = (int)uni((uint32_t)lmax);
  dmax = (int)uni((uint32_t)dmax);
  max_blindex = (int)uni((uint32_t)max_blindex);
  uint32_t hazard = 0;
  const bool bufok = block_start >= (int64_t)S;
  const uint64_t stored_len = (uint64_t)((int64_t)p - block_start);
  const uint64_t blk_start_bytes = b.pos;
  b.blocks++;
  if (stored_len + 4 <= opt_lenb && bufok) {
    put_bits(b, stage, (uint32_t)last, 3, lane);
    windup(b, stage, lane);
    uint32_t len = (uint32_t)stored_len;
    put_bits(b, stage, (len & 0xffff) | ((~len & 0xffff) << 16), 32, lane);
    // copy the block's input bytes (now byte aligned, bc == 0)
    const GLOBAL uint8_t* src = in + block_start;
    for (uint64_t o = 0; o < stored_len; o += 256) {
      uint32_t nb = stored_len - o < 256 ? (uint32_t)(stored_len - o) : 256u;
      for (uint32_t k = lane; k < 64; k += 64) {
        uint32_t wv = 0;
        for (int q = 0; q < 4; q++) {
          uint32_t at = 4 * k + q;
          if (at < nb) wv |= (uint32_t)src[o + at] << (8 * q);
        }
        stage[k] = wv;
      }
      emit_bytes_from_stage(b, stage, nb, lane);
      if (!full_needed && early_exit(b, opt, best_ident, false) != ~0u) break;
    }
  } else if (static_lenb == opt_lenb) {
    // the 3 header bits join the pending bits (fewer than 32 at a block start): compress_block writes them
    const uint32_t bc0 = uni(b.bc);
    b.bb = uni(b.bb) | ((uint64_t)((1u << 1) + (uint32_t)last) << bc0);
    b.bc = bc0 + 3;
    compress_block(b, stage, syms, last_lit, (const CONSTANT uint16_t*)c_t.st_lcode, (const CONSTANT uint8_t*)c_t.st_llen,
                   (const CONSTANT uint16_t*)c_t.st_dcode, (const CONSTANT uint8_t*)c_t.st_dlen, opt, best_ident,
                   full_needed, lane);
  } else {
    int lcodes = lmax + 1, dcodes = dmax + 1, blcodes = max_blindex + 1;
    // The whole block header -- BTYPE, HLIT / HDIST / HCLEN, the bit-length codes' lengths and the
    // run-length coded literal and distance code lengths (send_all_trees, Z/trees.c:836-860) -- is
    // assembled in the staging words behind the pending bits (fewer than 32 at a block start; at most
    // ~4.6 kbit in all) and written and compared in one pass.
    const uint64_t cs0 = STEP_CLOCK();
    for (int i = lane; i < (int)STAGE_WORDS; i += 64) stage[i] = 0;
    const uint32_t bc0 = uni(b.bc);
    const uint64_t bb0 = uni(b.bb);
    if (lane == 0) { stage[0] = (uint32_t)bb0; stage[1] = (uint32_t)(bb0 >> 32); }
    uint32_t off = bc0;
    if (lane == 0)
      stage_or(stage, off, (uint64_t)((2u << 1) + (uint32_t)last) | ((uint64_t)(lcodes - 257) << 3) |
                               ((uint64_t)(dcodes - 1) << 8) | ((uint64_t)(blcodes - 4) << 13), 17);
    off += 17;
    if (lane < blcodes) stage_or(stage, off + 3u * (uint32_t)lane, s.blen[bl_order((uint32_t)lane)], 3);
    off += 3u * (uint32_t)blcodes;
    off = rle_tree(s, stage, s.llen, lcodes - 1, true, off, lane);
    off = rle_tree(s, stage, s.dlen, dcodes - 1, true, off, lane);
    {
      const uint32_t full = off >> 3;
      emit_bytes_from_stage(b, stage, full, lane);
      const uint32_t rem = off & 7;
      const uint32_t lastw = stage[full >> 2];
      b.bb = rem ? ((lastw >> (8 * (full & 3))) & 0xff) & ((1u << rem) - 1) : 0;
      b.bc = rem;
    }
    b.cyc_send += STEP_CLOCK() - cs0;
    compress_block(b, stage, syms, last_lit, (const LDS uint16_t*)s.lcode, (const LDS uint8_t*)s.llen,
                   (const LDS uint16_t*)s.dcode, (const LDS uint8_t*)s.dlen, opt, best_ident, full_needed, lane);
  }
  // 1.2.8 pending_buf/d_buf overlay condition (conservative, cf. oracle/ora_deflate.c)
  if (b.pos - blk_start_bytes > (uint64_t)lbs + 2ull * last_lit && last_lit) hazard = 1;
  if (last) windup(b, stage, lane);
  return hazard;
}

__device__ __forceinline__ void init_block(LDS BlockFreq& f, int lane) {   // Z/trees.c:409-425
  for (int i = lane; i < (NLC + 1) / 2; i += 64) f.lfreq2[i] = 0;
  for (int i = lane; i < NDC / 2; i += 64) f.dfreq2[i] = 0;
  if (lane == 0) f.lfreq2[128] = 1;   // END_BLOCK (symbol 256: low half)
}

// _tr_flush_block + FLUSH_BLOCK_ONLY bookkeeping on one wave: trees, emission, init_block.  The emission
// staging overlays the tree scratch.  Returns the overlay-hazard bit.
__device__ __forceinline__ uint32_t flush_block(LDS TrialShared& s, LDS TreeScratch& sc, LDS BitOut& b, const GLOBAL uint32_t* syms,
                                                const GLOBAL uint8_t* in, int64_t block_start, uint64_t p, uint64_t S,
                                                uint32_t last_lit, uint32_t level, uint32_t lbs, int last, const SweepOpts& opt,
                                                uint64_t best_ident, bool full_needed, int lane) {
  const uint64_t c0 = clock64();
  const BlockPlan pl = block_trees(s.f, s.k, sc, &b.cyc_heap, level, (uint64_t)((int64_t)p - block_start), lane);
  const uint64_t c1 = clock64();
  b.cyc_tree += c1 - c0;
  const uint32_t hz = block_emit(s.k, (LDS uint32_t*)&sc, b, syms, in, block_start, p, S, last_lit, lbs, last, opt, best_ident,
                                 full_needed, pl.opt_lenb, pl.static_lenb, pl.lmax, pl.dmax, pl.max_blindex, lane);
  init_block(s.f, lane);
  b.cyc_emit += clock64() - c1;
  return hz;
}

// The parse path through a window of 64 lanes (lane i = position wb + i).  Lane i's node kind:
// Am bit = a step without a match (the path goes on at i + 1: runs of such lanes are one hop to the
// run's end), Nm bit = the node needs match-table entries not built yet; otherwise `rel` holds the
// next node's offset from wb (>= 64: beyond the window).  The scalar unit only chains readlanes
// through the hop starts H; which lanes lie on the path is then derived in lanes.
struct WinPath {
  uint64_t H;       // hop starts (path nodes where a hop begins)
  uint32_t end;     // offset of the position after the path (the next canonical position)
  bool need;        // the path stops at a node that needs more match-table entries (at `end`)
};
__device__ __forceinline__ uint32_t run_end_rel(uint64_t Am, int lane) {   // first lane > lane not in Am
  const uint64_t above = lane == 63 ? 0ull : (Am >> (lane + 1));
  return (uint32_t)lane + 1u + (uint32_t)__builtin_ctzll(~above);
}
__device__ __forceinline__ WinPath follow_path(uint32_t rel, uint64_t Nm, uint32_t lim) {
  WinPath w;
  uint64_t H = 0;
  uint32_t i = 0;
  while (i < lim) {   // lim = min(64, n - wb); rel of a need lane is 0xffff
    H |= 1ull << i;
    i = (uint32_t)__builtin_amdgcn_readlane((int)rel, (int)i);
  }
  w.need = (H & Nm) != 0;
  if (w.need) {   // the loop stopped right after entering the need node
    i = 63u - (uint32_t)__builtin_clzll(H & Nm);
    H &= ~Nm;
  }
  w.H = H;
  w.end = i;
  return w;
}
// lane's place on the path: on it, and whether a literal is pending when the path reaches it
// (only meaningful for hop starts and run members; ma_in: pending literal at the window start)
__device__ __forceinline__ void path_lane(const WinPath& w, uint64_t Am, uint32_t ma_in, int lane, bool& onp,
                                          uint32_t& mab) {
  const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);   // lanes <= lane
  const uint64_t hb = w.H & le;
  onp = false;
  mab = 0;
  if (hb) {
    const int h = 63 - __builtin_clzll(hb);
    if (h == lane) {
      onp = true;
      const uint64_t hs = w.H & (le >> 1);   // hop starts below
      mab = hs ? (uint32_t)((Am >> (63 - __builtin_clzll(hs))) & 1ull) : ma_in;
    } else if ((Am >> h) & 1ull) {   // member of the run starting at h: all lanes h..lane in Am
      const uint64_t seg = le & ~((1ull << h) - 1ull);
      onp = (~Am & seg) == 0;
      mab = 1;
    }
  }
}
// exclusive prefix sum of small per-lane counts over the wave by ballot bit planes (no LDS)
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t cnt, uint64_t lt, uint32_t& total) {
  uint32_t o = 0, T = 0;
  for (uint32_t bit = 0; bit < 32; bit++) {
    const uint64_t m = __ballot((cnt >> bit) & 1u);
    o += (uint32_t)__popcll(m & lt) << bit;
    T += (uint32_t)__popcll(m) << bit;
    if (!__ballot(cnt >> (bit + 1))) break;
  }
  total = T;
  return o;
}

// One flusher wave of a multi-wave trial: blocks f, f + MW_F, f + 2 MW_F, ... (see MWSlot).
// Speculative rounds (SweepArgs::stopj).  A trial whose result stops its stream -- full output, its ident
// within mismatch_tol of C and above the best it started from -- records its place in the round; the
// stream's rule walk stops there or earlier (any earlier trial reaching C - tol also stops it), so its
// later trials of the round are never walked and may end at once.  (Relaxed device-scope atomics: a
// trial that misses a fresh value only runs to its end, as without the flag.)
// The stream's word and the trial's place sit in LDS (TrialShared::stop_at / stop_j, set at the trial's
// start), so the parse loop keeps no registers for them.
__device__ __forceinline__ void spec_init(LDS TrialShared& s, const SweepArgs& A, const Trial& tr, int lane) {
  if (lane == 0) {
    s.stop_at = A.stopj ? (uint64_t)(uintptr_t)(A.stopj + tr.stream) : 0ull;
    s.stop_j = tr.spec_j;
  }
}
__device__ __forceinline__ bool spec_stopped(const LDS TrialShared& s) {
  const uint64_t a = uni(s.stop_at);
  const uint32_t j = uni(s.stop_j);
  if (!a || !j) return false;
  return uni(__hip_atomic_load((const GLOBAL uint32_t*)(uintptr_t)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < j;
}
__device__ __forceinline__ void spec_stop(const LDS TrialShared& s, const SweepArgs& A, uint64_t best_ident, uint32_t state,
                                          uint64_t ident, uint64_t clen, int lane) {
  const uint64_t a = uni(s.stop_at);
  if (!a || state != TR_FULL || ident <= best_ident) return;
  if (ident != clen && ident + A.o.mismatch_tol < clen) return;
  if (lane == 0) __hip_atomic_fetch_min((GLOBAL uint32_t*)(uintptr_t)a, uni(s.stop_j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void trial_flusher(const SweepArgs& A, LDS TrialShared& s, LDS MWPart& mw, const Trial& tr,
                              const GLOBAL uint32_t* syms, const GLOBAL uint8_t* in, uint32_t level, uint32_t lbs,
                              bool full_needed, int f, int lane) {
  LDS BitOut& b = s.b;
  LDS MWFlusher& me = mw.fl[f];
  LDS MWSlot& sl = mw.slot[f];
  LDS MWCtl& ctl = mw.ctl;
  LDS uint32_t* const stage = (LDS uint32_t*)&me.sc;
  for (uint32_t k = (uint32_t)f;; k += MW_F) {
    bool have = false;
    for (;;) {   // block k arrives in slot f
      if (ld_acq(ctl.stop)) break;
      if (ld_acq(sl.seq) == k + 1) { have = true; break; }
      if (ld_acq(ctl.parse_done) && k >= ld_acq(ctl.nblocks)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (!have) break;
    const int64_t bs = (int64_t)uni((uint64_t)sl.block_start);
    const uint64_t p = uni(sl.p), S = uni(sl.S);
    const uint32_t last_lit = uni(sl.last_lit), sbase = uni(sl.sbase);
    const int last = (int)uni(sl.last);
    const uint64_t c0 = clock64();
    const BlockPlan pl = block_trees(sl.f, me.k, me.sc, &me.cyc_heap, level, (uint64_t)((int64_t)p - bs), lane);
    st_rel(sl.seq, 0u, lane);   // the parser may refill the slot
    const uint64_t c1 = clock64();
    bool turn = false;
    for (;;) {   // emission in block order
      if (ld_acq(ctl.stop)) break;
      if (ld_acq(ctl.next_emit) == k) { turn = true; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!turn) break;
    const uint64_t c2 = clock64();
    const uint32_t hz = uni(block_emit(me.k, stage, b, syms + sbase, in, bs, p, S, last_lit, lbs, last, A.o, tr.best_ident,
                                       full_needed, pl.opt_lenb, pl.static_lenb, pl.lmax, pl.dmax, pl.max_blindex, lane));
    if (hz && lane == 0) __hip_atomic_fetch_or(&ctl.hazard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint32_t st = ~0u;
    if (last) {
      // adler32 trailer and the final gates (main.cpp:632-681), as a single-wave trial ends
      const uint32_t ad = A.adler[tr.stream];
      const uint32_t be = ((ad >> 24) & 0xff) | ((ad >> 8) & 0xff00) | ((ad << 8) & 0xff0000) | (ad << 24);
      put_bits(b, stage, be, 32, lane);
      flush_bits_bytes(b, stage, lane);
      if (uni((uint32_t)b.overflow)) st = TR_OVERFLOW;
      else if (full_needed) st = TR_FULL;
      else {
        const uint64_t thr = A.o.shortcut_len - A.o.recomp_tresh;
        const uint64_t L = uni(b.pos), clen = uni(b.clen);
        const int64_t dd = (int64_t)(L - clen);
        const uint64_t ad2 = (uint64_t)(dd < 0 ? -dd : dd);
        if (uni(b.shortcut) && uni(b.eq_sc) < thr) st = TR_SHORTCUT;
        else if (ad2 > A.o.sizediff_tresh) st = TR_SIZEDIFF;
        else st = TR_FULL;
      }
    } else {
      st = uni(early_exit(b, A.o, tr.best_ident, full_needed));
    }
    if (lane == 0) { me.cyc_tree += c1 - c0; me.cyc_emit += clock64() - c2; }
    if (last) spec_stop(s, A, tr.best_ident, st, uni(b.eq_all), uni(b.clen), lane);
    if (st != ~0u) {
      if (lane == 0) ctl.state = st;
      st_rel(ctl.stop, 1u, lane);
    }
    st_rel(ctl.next_emit, k + 1, lane);
    if (st != ~0u) break;
  }
}

static constexpr uint32_t TR_DECIDED = 0xfffffffeu;   // parser-side: a flusher decided the trial (MWCtl::state)

// One trial (a wave, or a parse wave and MW_F flushers): the stream's zlib header, the level's parse
// over the match tables -- deflate_stored, a replay of a saved symbol sequence, deflate_fast or
// deflate_slow -- with its blocks flushed as they fill, then the trailer and the final gates.  The
// parse state lives in the members (registers, once everything is inlined).
template <int KIND, typename SH>
struct TrialRun {
  static constexpr bool MW = HasMW<SH>::value;
  const SweepArgs& A;
  SH& shm;
  const int lane, wave;
  LDS TrialShared& s;
  LDS uint32_t* const stg;   // emission staging (overlays the ring)
  LDS BitOut& b;
  const uint32_t t;
  const Trial tr;
  const StreamDev sd;
  const uint8_t* const in;
  // hash buckets of (stream, memLevel): sidx[npad] then bpos[npad]
  const uint32_t npad;
  const uint32_t* const sidx;
  const uint32_t* const bpos;
  const bool full_needed;
  const uint64_t lt;   // lanes below this one
  Lz z;
  bool saving = false, replay = false, rec = false;
  // global (not generic) pointers: a flat store counts in lgkmcnt too, so every later LDS wait of the
  // parse would also wait for the store to reach L2
  GLOBAL uint32_t* syms = nullptr;
  GLOBAL uint64_t* rtab = nullptr;
  uint32_t sbase = 0;            // symbols in the flushed blocks
  uint32_t saved_flags = 0;
  uint32_t run_len = 0, run_imp = 0;   // slow parses: longest match length any of its reads saw, longest
                                       // prev_length a lazy read improved (per lane, reduced at the end)
  uint64_t cstart = 0;
  uint32_t rtstart = 0;
  uint32_t hazard = 0;
  // Symbols and block statistics are tallied straight into HBM (syms) and LDS (lfreq / dfreq).
  uint32_t state = ~0u;
  uint64_t fallbacks = 0, cyc_fb = 0;
  uint64_t csec[4] = {0, 0, 0, 0};   // diagnostics (ATZ_STEP_CLOCKS)
  uint32_t nblk = 0;   // multi-wave: blocks handed to the flushers
  // the parse (wave 0): match-table ring, the stream's geometry; deflate_fast's holes and insertion bits
  LDS uint64_t* ring = nullptr;
  const GLOBAL uint64_t* Rt = nullptr;
  uint32_t n = 0, wsz = 0, maxd = 0, xlim = 0;
  bool noslide = false;
  uint32_t hi = 0;
  uint64_t pf = 0;
  LDS uint32_t* holes = nullptr;
  LDS uint32_t* ins = nullptr;

  __device__ __forceinline__ TrialRun(const SweepArgs& A_, SH& shm_, int lane_)
      : A(A_), shm(shm_), lane(lane_), wave(MW ? (int)(threadIdx.x >> 6) : 0), s(*(LDS TrialShared*)&shm_.t),
        stg((LDS uint32_t*)shm_.ring), b(s.b), t(blockIdx.x), tr(A_.trials[t]), sd(A_.streams[tr.stream]),
        in(A_.infl + sd.infl_off), npad((uint32_t)((sd.infl_len + 63) & ~63ull)),
        sidx(KIND == 0 ? nullptr : A_.chains + tr.chain_off), bpos(KIND == 0 ? nullptr : sidx + npad),
        full_needed(tr.mode & 1), lt(lane_ ? (~0ull >> (64 - lane_)) : 0ull) {
    z.level = tr.clevel; z.kind = KIND;
    z.wsize = 1u << tr.window; z.maxdist = z.wsize - LOOKMIN; z.lbs = 1u << (tr.memlevel + 6);
    z.good = c_cfg[z.level][0]; z.lazy = c_cfg[z.level][1]; z.nice = c_cfg[z.level][2]; z.chain = c_cfg[z.level][3];
    z.n = sd.infl_len; z.p = 0; z.lookahead = 0; z.S = 0; z.block_start = 0;
    z.match_start = 0; z.prev_match = 0; z.match_length = 2; z.prev_length = 2; z.match_available = 0;
    z.last_lit = 0; z.nsym = 0;
    if (wave == 0) {
      b.out = (GLOBAL uint8_t*)(A.out + tr.out_off); b.cap = tr.out_cap; b.pos = 0; b.bb = 0; b.bc = 0;
      b.orig = (const GLOBAL uint8_t*)(A.file + sd.orig_off); b.clen = sd.comp_len;
      b.shortcut = sd.comp_len > A.o.shortcut_len ? A.o.shortcut_len : 0;
      b.eq_all = 0; b.eq_sc = 0; b.overflow = 0;
    }
    // fast and slow levels: a saving trial writes its whole symbol sequence at rp_syms (block k's
    // symbols at sbase, the count of symbols in the blocks before it); a replaying trial reads one
    saving = KIND != 0 && (tr.mode & 4);
    replay = KIND != 0 && (tr.mode & 8);
    if (KIND == 2 && replay && (tr.mode & 16)) {
      const uint32_t tlim = tr.x_lim < sd.infl_len ? (uint32_t)tr.x_lim : (uint32_t)sd.infl_len;   // entries present
      // replay only if this trial's table agrees with the saver's on every entry the saver's parse
      // read (bit 0 of a saved half: that half was read): then this trial's parse reads the same
      // entries, step by step, and takes the same path.  A read compares the length and distance
      // (the head-valid bit only matters with a length > 2, which it implies; the literal byte is
      // the input's)
      const GLOBAL uint64_t* mt = (const GLOBAL uint64_t*)(A.R + tr.r_off);   // .x low, .y high
      const GLOBAL uint64_t* st = (const GLOBAL uint64_t*)(uintptr_t)tr.rp_tab;
      bool same = true;
      for (uint32_t p0 = 0; p0 < tlim && same; p0 += 256) {
        bool d = false;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint32_t p = p0 + 64u * (uint32_t)u + (uint32_t)lane;
          if (p < tlim) {
            const uint64_t sv = st[p], df = mt[p] ^ sv;
            d |= ((sv & 1ull) && (df & 0xffffff00ull)) || ((sv >> 32) & 1ull && (df & 0xffffff0000000000ull));
          }
        }
        same = __ballot(d) == 0;
      }
      replay = same;
    }
    syms = saving || replay ? (GLOBAL uint32_t*)(uintptr_t)tr.rp_syms : (GLOBAL uint32_t*)(A.syms + tr.sym_off);
    // a saving slow trial records the match-table entries its parse reads (rp_tab, cleared first)
    rec = KIND == 2 && saving && (tr.mode & 32);
    rtab = (GLOBAL uint64_t*)(uintptr_t)tr.rp_tab;
    if (rec && wave == 0) {
      for (uint32_t p = (uint32_t)lane; p < sd.infl_len; p += 64) rtab[p] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the clears land before the records
    }
    if (wave == 0) {
      b.cyc_tree = b.cyc_emit = b.blocks = 0;
      b.cyc_heap = b.cyc_scan = b.cyc_send = 0;
    }
    cstart = clock64();
    rtstart = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (wave == 0) init_block(s.f, lane);
    // zlib header (Z/deflate.c:738-759)
    if (wave == 0) {
      uint32_t header = (8u + ((uint32_t)(tr.window - 8) << 4)) << 8;
      uint32_t lf = z.level < 2 ? 0 : z.level < 6 ? 1 : z.level == 6 ? 2 : 3;
      header |= lf << 6;
      header += 31 - (header % 31);
      put_bits(b, stg, ((header >> 8) & 0xff) | ((header & 0xff) << 8), 16, lane);   // < 32 bits: no staging
    }
  }

  static constexpr uint32_t ins_mask() { return SH::INS_BITS / 32 - 1; }
  __device__ __forceinline__ bool ins_get(uint32_t q) const { return (ins[(q >> 5) & ins_mask()] >> (q & 31)) & 1u; }
  // S at an iteration at q >= one with S0
  __device__ __forceinline__ uint32_t S_iter(uint32_t S0, uint32_t q) const {
      uint32_t Sx = S0;
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const bool exh = n <= Sx + 2u * wsz;
        const bool slide = exh ? (q + LOOKMIN > n && q >= Sx + wsz + maxd) : (q > Sx + wsz + maxd);
        if (slide) Sx += wsz;
      }
      return Sx;
  }
  // multi-wave: hand the finished block to its flusher; false when the trial is already decided
  __device__ __forceinline__ bool publish(int last) {
      if constexpr (MW) {
        LDS MWPart& mw = *(LDS MWPart*)&shm.mw;
        const uint32_t f = nblk % (uint32_t)MW_F;
        LDS MWSlot& sl = mw.slot[f];
        for (;;) {
          if (ld_acq(mw.ctl.stop)) return false;
          if (ld_acq(sl.seq) == 0) break;
          __builtin_amdgcn_s_sleep(1);
        }
        for (int i = lane; i < (NLC + 1) / 2; i += 64) sl.f.lfreq2[i] = s.f.lfreq2[i];
        for (int i = lane; i < NDC / 2; i += 64) sl.f.dfreq2[i] = s.f.dfreq2[i];
        if (lane == 0) {
          sl.block_start = (int64_t)z.block_start; sl.p = z.p; sl.S = z.S;
          sl.last_lit = z.last_lit; sl.sbase = sbase; sl.last = (uint32_t)last;
        }
        st_rel(sl.seq, nblk + 1, lane);   // after the wave's symbol stores and the slot writes
        nblk++;
        init_block(s.f, lane);
        sbase += z.last_lit;
        z.last_lit = 0;
        z.block_start = z.p;
      }
      return true;
  }
  __device__ __forceinline__ void FLUSH(int last) {
      hazard |= uni(flush_block(s, *(LDS TreeScratch*)shm.ring, b, (const GLOBAL uint32_t*)syms + ((saving || replay) ? sbase : 0u),
                                (const GLOBAL uint8_t*)in, (int64_t)z.block_start, z.p, z.S, z.last_lit, z.level, z.lbs, last,
                                A.o, tr.best_ident, full_needed, lane));
      sbase += z.last_lit;
      z.last_lit = 0;
      z.block_start = z.p;
      if (KIND != 0 && !replay) {   // the tree scratch overlaid the ring: reload its resident chunks
        for (uint32_t c0 = hi >= RING_SLOW ? hi - RING_SLOW : 0u; c0 < hi; c0 += 64) {
          const uint32_t pos = c0 + (uint32_t)lane;
          if (pos < n) ring[pos & (RING_SLOW - 1)] = Rt[pos];
        }
      }
  }
  // a block is full: flush it (single wave) or hand it over (multi-wave); returns the early-exit state
  __device__ __forceinline__ uint32_t FLUSH0() {
      if constexpr (MW) {
        return publish(0) ? ~0u : TR_DECIDED;
      } else {
        FLUSH(0);
        const uint32_t e = uni(early_exit(b, A.o, tr.best_ident, full_needed));
        return e == ~0u && spec_stopped(s) ? TR_SKIPPED : e;
      }
  }

  __device__ __forceinline__ void parse_setup() {
    // fast and slow kinds: match-table entries of the positions around the parse window in an LDS
    // ring; window slides (fill_window at the top of an iteration when lookahead < MIN_LOOKAHEAD)
    // are a function of the iteration position, so any lane can evaluate them.
    if constexpr (KIND != 0) ring = (LDS uint64_t*)shm.ring;   // position & (RING_SLOW - 1); .x low, .y high
    Rt = (const GLOBAL uint64_t*)(A.R + tr.r_off);
    n = z.n; wsz = z.wsize; maxd = z.maxdist; xlim = (uint32_t)tr.x_lim;
    // fill_window never slides a stream of at most wsize + MAX_DIST bytes (Z/deflate.c:1419-1451:
    // strstart stays below it), so S is 0 throughout and the NIL-after-slide checks drop out (wave-
    // uniform: the walks skip them with a scalar branch)
    noslide = ATZ_NOSLIDE_PATH && n <= wsz + maxd;
    // ring: chunks of 64 entries below `hi` are resident; the chunk at `hi` is in flight in pf
    if (KIND != 0 && n && !replay) pf = Rt[lane];
  }

  // deflate_stored (Z/deflate.c:1564-1619)
  __device__ __forceinline__ void parse_stored() {
  uint64_t max_block = 0xffff;
  if (max_block > 4ull * z.lbs - 5) max_block = 4ull * z.lbs - 5;
  for (;;) {
    if (z.lookahead <= 1) { fill(z); if (z.lookahead == 0) break; }
    z.p += z.lookahead;
    z.lookahead = 0;
    const uint32_t max_start = z.block_start + (uint32_t)max_block;
    if (z.p == 0 || z.p >= max_start) {
      z.lookahead = z.p - max_start;
      z.p = max_start;
      state = FLUSH0();
      if (state != ~0u) break;
    }
    if (z.p - z.block_start >= z.maxdist) {
      state = FLUSH0();
      if (state != ~0u) break;
    }
  }
  }

  __device__ __forceinline__ void parse_replay() {
  // Symbol replay.  The sequence saved by a trial of this stream at the same (level, window) and
  // another memLevel is this trial's own: the host proved that no chain walk of either memLevel
  // reaches its budget (every bucket holds at most B + 1 positions, B = max_chain for deflate_fast,
  // whose prev_length never reaches good_match, and max_chain / 4 for deflate_slow), so each walk
  // examines the same-trigram positions in the same order (other hashes in a chain never match:
  // their first two bytes differ) and returns the same match; deflate_fast's insertions follow the
  // match lengths, and neither parse depends on lit_bufsize.  Only the blocks differ: the symbols
  // are tallied into this memLevel's blocks of lit_bufsize - 1, each flushed at the position after
  // its last symbol (deflate_slow tallies a literal at iteration pos + 1, a match when strstart
  // reaches its end; deflate_fast flushes after strstart moved past the symbol); deflate_slow's
  // end-of-input pending literal is tallied without a flush check (Z/deflate.c:1842-1846).
  // A replay checked against a table prefix (x_lim < n) stops where the parse would read past it.
  const GLOBAL uint32_t* sv = (const GLOBAL uint32_t*)syms;
  const uint32_t nsv = tr.rp_nsym;
  const bool endlit = (tr.rp_flags & 2u) != 0;
  saved_flags |= 4;
  uint32_t k = 0, pos = 0;
  while (k < nsv) {
    const uint32_t cnt = nsv - k < 64u ? nsv - k : 64u;
    const bool valid = (uint32_t)lane < cnt;
    const uint32_t v = valid ? sv[k + (uint32_t)lane] : 0u;
    const uint32_t len = valid ? ((v >> 8) ? (v & 0xffu) + 3u : 1u) : 0u;
    const uint32_t incl = wave_incl_scan(len);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (xlim < n && pos + tot + 2u > xlim) { state = TR_NEED_R; z.p = pos; break; }
    uint32_t base = 0;
    while (base < cnt) {
      const uint32_t room = z.lbs - 1u - z.last_lit;
      const uint32_t seg_end = cnt - base < room ? cnt : base + room;
      if ((uint32_t)lane >= base && (uint32_t)lane < seg_end) {
        if (v >> 8) {
          const uint32_t lc = 257u + len_code(v & 0xffu), dc = dist_code((v >> 8) - 1u);
          __hip_atomic_fetch_add(&s.f.lfreq2[lc >> 1], 1u << (16 * (lc & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(&s.f.dfreq2[dc >> 1], 1u << (16 * (dc & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          __hip_atomic_fetch_add(&s.f.lfreq2[v >> 1], 1u << (16 * (v & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      z.last_lit += seg_end - base;
      z.nsym += seg_end - base;
      if (z.last_lit == z.lbs - 1u && !(endlit && k + seg_end == nsv)) {
        z.p = pos + (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)seg_end - 1);
        state = FLUSH0();
        if (state != ~0u) break;
      }
      base = seg_end;
    }
    if (state != ~0u) break;
    pos += tot;
    k += cnt;
  }
  if (state == ~0u) {
    z.p = n;
    z.S = 0;
  }
  }

  // deflate_fast: whether the table's step at path node x may differ from deflate_fast's own walk
  __device__ __forceinline__ bool fast_node_bad(bool onp, uint32_t x, uint32_t ex, uint32_t ey, uint32_t Sx, uint32_t sxl) {
  bool bad = false;
  if (onp && x + 3u <= n) {
    const uint32_t hl = holes[(ey >> 1) & (HOLE_SLOTS - 1)];
    bool exact = hl == 0 || hl - 1u < x - (ey >> 16);
    if (!exact && !((ey >> 12) & 1u)) {
      // Skipped nodes only shrink the visited set -- except at the MAX_DIST edge: deflate_fast
      // walks its hash head at distance MAX_DIST (Z/deflate.c:1660) but later chain nodes only
      // above it (Z/deflate.c:1227), so when holes above it made a hole the table's head, the
      // node at exactly x - MAX_DIST can be examined by deflate_fast and not by the table walk.
      // Such a node is resolved by the exact walk below.
      const uint32_t q0 = x - maxd;
      const uint32_t hb = tr.memlevel + 7u, hs = (hb + 2u) / 3u, hm = (1u << hb) - 1u;
      const bool edge = x > maxd && q0 > Sx &&
                        ((((uint32_t)in[q0] << (2u * hs)) ^ ((uint32_t)in[q0 + 1] << hs) ^ in[q0 + 2]) & hm) ==
                        ((((uint32_t)in[x] << (2u * hs)) ^ ((uint32_t)in[x + 1] << hs) ^ in[x + 2]) & hm);
      if (edge) exact = false;
      else if ((ex >> 23) <= 2) exact = true;
      else {
        const uint32_t wpos = x - ((ex >> 8) & 0x7fffu);
        exact = wpos > Sx && ins_get(wpos);
      }
    } else if (!exact && ATZ_VISITED_CHECK && z.chain <= ATZ_VISITED_MAX) {
      // the walk spent its budget and a hole shares the slot: the entry is still exact when
      // every node the walk visited (the bucket entries below x down to the lowest visited
      // one, at most `chain` of them) was inserted -- deflate_fast's chain then starts with
      // the same nodes and spends the same budget on them
      const uint32_t lo = x - (ey >> 16);
      const int32_t si = (int32_t)sxl;
      bool ok = true, stop = false;
      for (int32_t k = si - 1; ok && !stop && k > si - 1 - (int32_t)z.chain; k -= 4) {
        uint32_t e4[4];
#pragma unroll
        for (int u = 0; u < 4; u++) e4[u] = k - u >= 0 ? bpos[k - u] : BUCKET_FIRST;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          if (!ok || stop || k - u <= si - 1 - (int32_t)z.chain) break;
          const uint32_t pos = e4[u] & ~BUCKET_FIRST;
          if (k - u < 0 || pos < lo) { stop = true; break; }
          ok = pos > Sx && ins_get(pos);
          if (e4[u] & BUCKET_FIRST) stop = true;
        }
      }
      exact = ok;
    }
    bad = !exact;
  }
    return bad;
  }

  // deflate_fast's longest_match (Z/deflate.c:1148-1289) over the INSERTED same-hash positions, for up to
  // eight bad nodes of a window at once: node g of the batch (the g-th set bit of bm, nb nodes) walks on
  // lanes [g*S, g*S + S), S = 64 / G, S bucket entries per step in walk order (descending bucket index);
  // lanes test insertion and compare bytes in parallel.  Each node is walked as if the window's path
  // stands up to it, which is how the caller uses its result (it stops at the first node whose exact
  // step differs from the table's).  The walk order, the budget count, the first maximum and the nice
  // stop do not depend on the chunk size, so every node's result is the single 64-lane walk's.  Lane
  // g*S of rml / rms gets node g's match (length 0: none).  One batch replaces a chain of dependent walks
  // (bucket chunk, then candidate bytes, one HBM round trip each) per bad node: the slowest trials of a
  // round (fast levels at memLevel 1-3, 1 000-4 000 walks each) have several bad nodes per window.
  __device__ __forceinline__ void fast_exact_walks(uint64_t bm, uint32_t nb, uint32_t G, uint32_t wb, uint32_t Sb,
                                                   uint32_t sxl, uint32_t& rml, uint32_t& rms) {
    const uint32_t lg = G == 1 ? 6u : G == 2 ? 5u : G == 4 ? 4u : 3u;   // log2 S
    const uint32_t S = 1u << lg;
    const uint32_t ll = (uint32_t)lane & (S - 1u), g = (uint32_t)lane >> lg, base = g << lg;
    const uint64_t smask = S == 64 ? ~0ull : ((1ull << S) - 1ull);
    const uint64_t ltl = ll ? (~0ull >> (64 - ll)) : 0ull;   // lanes of the segment below this one
    auto seg = [&](bool pred) -> uint64_t { return (__ballot(pred) >> base) & smask; };
    uint32_t fl = 0;   // this segment's node: its lane in the window
    {
      uint64_t m = bm;
      for (uint32_t gi = 0; gi < nb; gi++) {
        const uint32_t bit = (uint32_t)__builtin_ctzll(m);
        m &= m - 1ull;
        fl = g == gi ? bit : fl;
      }
    }
    const uint32_t f = wb + fl;
    const uint32_t si = (uint32_t)__shfl((int)sxl, (int)fl, 64);
    const uint32_t Sf = S_iter(Sb, f);
    const uint32_t la = n - f < LOOKMIN ? n - f : LOOKMIN;   // lookahead (>= 258 stands for more)
    const uint32_t limit = f > maxd ? f - maxd : 0u;          // later nodes only while > limit
    const uint32_t cap = n - f < 258u ? n - f : 258u;
    const uint32_t nicec = z.nice < la ? z.nice : la;         // <= cap
    // the first chunk starts at f's own entry (local lane 0), whose first-of-bucket flag says whether f
    // has a chain at all
    int32_t top = (int32_t)si;
    uint32_t skip = 1;
    bool done = g >= nb, head_done = false, hv = false, won = false, nicew = false;
    uint32_t examined = 0, best = 2, win = 0;
    while (__ballot(!done)) {
      const int32_t k = top - (int32_t)ll;
      const uint32_t e = (!done && k >= 0) ? bpos[k] : BUCKET_FIRST;
      const uint32_t e0 = (uint32_t)__shfl((int)e, (int)base, 64);
      if (!done && skip && (e0 & BUCKET_FIRST)) done = true;   // first of its bucket: no chain
      const uint64_t fm = seg(!done && (e & BUCKET_FIRST) != 0 && ll >= skip);
      const uint32_t flane = fm ? (uint32_t)__builtin_ctzll(fm) : S;   // the bucket's first entry: last node
      const uint32_t qc = e & ~BUCKET_FIRST;
      const bool insd = !done && ll >= skip && ll <= flane && k >= 0 && ins_get(qc);
      const uint64_t im = seg(insd);
      bool go = !done;
      uint32_t from = 0, head_ll = S;   // head_ll < S: the head was found in this chunk
      if (go && !head_done) {
        if (!im) {   // no inserted node in this chunk yet
          if (flane < S) done = true;
          go = false;
        } else {
          head_ll = (uint32_t)__builtin_ctzll(im);
          head_done = true;
          from = head_ll;
        }
      }
      const uint32_t hh = (uint32_t)__shfl((int)qc, (int)(base + (head_ll < S ? head_ll : 0u)), 64);
      if (go && head_ll < S) {
        hv = hh > Sf && f - hh <= maxd;   // zlib calls longest_match only then
        if (!hv) { done = true; go = false; }
      }
      // the walk stops at the first inserted node <= limit (the head is always examined)
      const uint64_t sm = seg(go && insd && ll >= from && ll != head_ll && qc <= limit);
      const uint32_t slane = sm ? (uint32_t)__builtin_ctzll(sm) : S;
      bool cand = go && insd && ll >= from && ll < slane;
      cand = cand && (uint32_t)__popcll(seg(cand) & ltl) < z.chain - examined;
      if (go) examined += (uint32_t)__popcll(seg(cand));
      // match lengths capped at nice (16 bytes per round trip); the first candidate reaching nice ends
      // the walk, so capped lengths decide the winner
      uint32_t len = 0;
      bool more = cand;
      while (__ballot(more)) {
        if (more) {
          const uint32_t run = match16((const GLOBAL uint32_t*)in, qc + len, f + len, nullptr, 0);
          const uint32_t left = nicec - len;
          len += run < left ? run : left;
          more = run == 16 && len < nicec;
        }
      }
      const uint64_t nm = seg(cand && len >= nicec);
      uint32_t mx = cand ? len : 0u;
      for (uint32_t d = S >> 1; d >= 1; d >>= 1) {
        const uint32_t o2 = (uint32_t)__shfl_xor((int)mx, (int)d, 64);
        mx = mx > o2 ? mx : o2;
      }
      const uint64_t xm = seg(cand && len == mx);
      const uint32_t pick = nm ? (uint32_t)__builtin_ctzll(nm) : xm ? (uint32_t)__builtin_ctzll(xm) : 0u;
      const uint32_t wq = (uint32_t)__shfl((int)qc, (int)(base + pick), 64);
      if (go) {
        if (nm) { win = wq; won = true; nicew = true; done = true; }
        else {
          if (mx > best) { win = wq; best = mx; won = true; }
          if (examined >= z.chain || slane < S || flane < S) done = true;
        }
      }
      top -= (int32_t)S;
      skip = 0;
    }
    // the full length of a nice winner (its first nicec bytes match), 16 bytes per lane per step: the
    // first lane of the segment whose run ends gives it (its end lies before every later lane's offset)
    bool need = nicew;
    uint32_t o = nicec + 16u * ll;
    while (__ballot(need)) {
      uint32_t endp = ~0u;
      if (need) {
        if (o >= cap) endp = cap;
        else {
          const uint32_t r = match16((const GLOBAL uint32_t*)in, win + o, f + o, nullptr, 0);
          if (r < 16 || o + r >= cap) endp = o + r < cap ? o + r : cap;
        }
      }
      for (uint32_t d = S >> 1; d >= 1; d >>= 1) {
        const uint32_t o2 = (uint32_t)__shfl_xor((int)endp, (int)d, 64);
        endp = endp < o2 ? endp : o2;
      }
      if (need && endp != ~0u) { best = endp; need = false; }
      o += 16u * S;
    }
    rml = (hv && won) ? (best <= la ? best : la) : 0u;
    rms = win;
  }

  __device__ __forceinline__ void parse_fast() {
  // deflate_fast (Z/deflate.c:1628-1722), lane-parallel.  Every deflate_fast iteration starts in
  // the same state, so a window takes the match table's step at each of its 64 positions in
  // lanes, the scalar unit follows the parse path through them, and the path's insertion state
  // and symbols are written lane-parallel.  A table entry is the walk over ALL same-hash
  // positions; deflate_fast walks the INSERTED ones (interiors of matches longer than
  // max_insert_length are skipped: "holes"), so every path node is checked: the entry is exact
  // unless a hole with its hash slot lies in the walked range [lowest visited node, p) AND it
  // can matter -- skipped nodes only shrink the visited set, so a walk that ended by nice_match
  // or by the end of the chain keeps its winner W if W itself was inserted (and with no winner
  // the step emits a literal either way); only a walk that spent its budget with nodes left can
  // see new nodes (bit 12).  The first node that fails the check is walked exactly over the
  // inserted positions and the window ends there.  holes[] keeps per slot the latest hole; the
  // window's own holes are entered before the check, so a hole behind the node only makes the
  // check conservative (slot collisions likewise).
  holes = (LDS uint32_t*)shm.holes;
  ins = (LDS uint32_t*)shm.ins;   // insertion bits, position mod SH::INS_BITS
  for (int i = lane; i < (int)HOLE_SLOTS; i += 64) holes[i] = 0;
  // insertion bits and holes of the positions [lo, hi) covered by path nodes; cover(p) gives the
  // node y <= p covering p and its match length (0: literal).  cover runs with all lanes active
  // (it may shuffle: a lane outside EXEC would read as 0).
  auto span_set = [&](uint32_t lo, uint32_t hi2, auto cover) {
    for (uint32_t c0 = lo & ~63u; c0 < hi2; c0 += 64) {
      const uint32_t p = c0 + (uint32_t)lane;
      const bool insp = p >= lo && p < hi2;
      bool insd = false, hole = false;
      uint32_t y, Ly;
      cover(p, y, Ly);
      if (insp) {
        if (p == y) insd = p + 3u <= n;
        else if (Ly <= z.lazy && y + Ly + 3u <= n) insd = true;
        else hole = p + 3u <= n;
      }
      const uint64_t bits = __ballot(insd), sm = __ballot(insp);
      if (lane < 2) {
        const uint32_t sh = 32u * (uint32_t)lane;
        const uint32_t m = (uint32_t)(sm >> sh), bv = (uint32_t)(bits >> sh);
        if (m) {
          LDS uint32_t& w = ins[((c0 + sh) >> 5) & ins_mask()];
          w = (w & ~m) | (bv & m);
        }
      }
      if (hole) {
        const uint32_t slot = ((uint32_t)(ring[p & (RING_SLOW - 1)] >> 32) >> 1) & (HOLE_SLOTS - 1);
        __hip_atomic_fetch_max(&holes[slot], p + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  };
  // one symbol, tallied by the scalar unit; returns true when the block is full
  auto tally1 = [&](uint32_t v) -> bool {
    if (lane == 0) {
      syms[(saving || MW ? sbase : 0u) + z.last_lit] = v;
      if (v >> 8) {
        __hip_atomic_fetch_add(&s.f.lfreq2[(257u + len_code(v & 0xffu)) >> 1], 1u << (16 * ((257u + len_code(v & 0xffu)) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&s.f.dfreq2[(dist_code((v >> 8) - 1u)) >> 1], 1u << (16 * ((dist_code((v >> 8) - 1u)) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        __hip_atomic_fetch_add(&s.f.lfreq2[(v) >> 1], 1u << (16 * ((v) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    z.last_lit++;
    z.nsym++;
    return z.last_lit == z.lbs - 1u;
  };
  uint32_t q = 0, Sb = 0;
  bool need = false;
  while (q < n) {
    const uint32_t wb = q, bal = wb & ~63u;
    uint64_t t0 = STEP_CLOCK();
    while (hi < bal + RING_SLOW) {
      ring[(hi + lane) & (RING_SLOW - 1)] = pf;
      hi += 64;
      if (hi < n) pf = Rt[hi + lane];
    }
    Sb = S_iter(Sb, wb);
    if (ATZ_STEP_CLOCKS) { (void)ring[wb & (RING_SLOW - 1)]; __builtin_amdgcn_s_waitcnt(0); }
    uint64_t t1 = STEP_CLOCK(); csec[0] += t1 - t0; t0 = t1;
    // ---- the table's step at x = wb + lane: wt 0 none (x >= n), 1 literal, 2 match, 3 needs R >= x_lim
    const uint32_t x = wb + lane;
    // x's bucket index, loaded now and read only by the node checks and the exact walks below (its
    // latency hides behind the window's own work instead of opening a walk)
    const uint32_t sxl = x < n ? sidx[x] : 0u;
    uint32_t wt = 0, L = 0, D = 0, ex = 0, ey = 0, Sx = Sb;
    if (x < n) {
      if (x >= xlim) wt = 3;
      else {
        const uint64_t e64 = ring[x & (RING_SLOW - 1)];
        ex = (uint32_t)e64; ey = (uint32_t)(e64 >> 32);
        if (!noslide) Sx = S_iter(Sb, x);
        bool hv = x + 3u <= n && (ey & 1u);
        if (!noslide && hv && Sx != 0 && x - Sx <= maxd) {   // hash_head == S is NIL after a slide
          const uint32_t si = sidx[x];
          hv = (bpos[si] & BUCKET_FIRST) || (bpos[si - 1] & ~BUCKET_FIRST) != Sx;
        }
        const uint32_t len = ex >> 23;
        if (hv && len > 2) { wt = 2; L = len; D = (ex >> 8) & 0x7fffu; }
        else wt = 1;
      }
    }
    // ---- follow the parse path through the window
    const uint64_t Am = __ballot(wt == 1), Nm = __ballot(wt == 3);
    t1 = STEP_CLOCK(); csec[1] += t1 - t0; t0 = t1;
    const uint32_t rel = wt == 1 ? run_end_rel(Am, lane) : wt == 2 ? (uint32_t)lane + L : 0xffffu;
    const WinPath wp = follow_path(rel, Nm, n - wb < 64 ? n - wb : 64u);
    bool onp;
    uint32_t mab_unused;
    path_lane(wp, Am, 0, lane, onp, mab_unused);
    const uint64_t P = __ballot(onp);
    need = wp.need;
    const uint32_t qn = wb + wp.end;
    const uint32_t last = P ? wb + 63u - (uint32_t)__builtin_clzll(P) : wb;
    // ---- insertion state of the path, then the check of its nodes
    t1 = STEP_CLOCK(); csec[2] += t1 - t0; t0 = t1;
    if (qn > wb)
      span_set(wb, qn, [&](uint32_t p, uint32_t& y, uint32_t& Ly) {
        const uint32_t i = p - wb;   // huge for p < wb (such lanes are outside the span)
        uint32_t yl = last - wb;
        if (i < 64) yl = 63u - (uint32_t)__builtin_clzll(P & (~0ull >> (63 - i)));
        y = wb + yl;
        Ly = (uint32_t)__shfl((int)L, (int)yl, 64);
      });
#if ATZ_STEP_SPLIT
    t1 = STEP_CLOCK(); csec[0] += t1 - t0; t0 = t1;   // (diagnostics: span_set counted with refill)
#endif
    const bool bad = fast_node_bad(onp, x, ex, ey, Sx, sxl);
    // Bad nodes are resolved one at a time by an exact walk.  When the walk's length equals the
    // table's (or both give a literal), the parse path is unchanged: the node keeps its place on
    // the path (with the walk's distance) and the window goes on to its next bad node.  Only a
    // different length ends the window there.
    uint64_t badm = __ballot(bad);
    uint64_t donem = 0;   // path nodes tallied so far
    uint32_t Dx = D;      // this lane's match distance (an exact walk may replace the table's)
    bool restart = false;
    uint32_t qnext = qn;
    uint64_t batchm = 0;           // bad nodes of the current batch of exact walks
    uint32_t rml = 0, rms = 0, bS = 64;
    for (;;) {
      // ---- tally the committed nodes' symbols lane-parallel, in position order
      const uint64_t Pc = (badm ? P & ((1ull << __builtin_ctzll(badm)) - 1ull) : P) & ~donem;
      {
        const bool mine = (Pc >> lane) & 1ull;
        const uint32_t o = (uint32_t)__popcll(Pc & lt);
        const uint32_t T = (uint32_t)__popcll(Pc);
        z.nsym += T;
        uint32_t base = 0;
        while (base < T) {
          const uint32_t room = z.lbs - 1u - z.last_lit;
          const uint32_t seg_end = T - base < room ? T : base + room;
          if (mine && o >= base && o < seg_end) {
            uint32_t v;
            if (wt == 2) {
              v = (Dx << 8) | (L - 3u);
              __hip_atomic_fetch_add(&s.f.lfreq2[(257u + len_code(L - 3u)) >> 1], 1u << (16 * ((257u + len_code(L - 3u)) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_add(&s.f.dfreq2[(dist_code(Dx - 1u)) >> 1], 1u << (16 * ((dist_code(Dx - 1u)) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
              v = ex & 0xffu;
              __hip_atomic_fetch_add(&s.f.lfreq2[(v) >> 1], 1u << (16 * ((v) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            syms[(saving || MW ? sbase : 0u) + z.last_lit + (o - base)] = v;
          }
          z.last_lit += seg_end - base;
          if (z.last_lit == z.lbs - 1u) {   // flush after the node tallied last: strstart past its step
            const uint64_t om = __ballot(mine && o == seg_end - 1u);
            const int ol = (int)__builtin_ctzll(om);
            const uint32_t fx = (uint32_t)__builtin_amdgcn_readlane((int)x, ol);
            const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)L, ol);
            z.p = fx + (fl ? fl : 1u);
            z.S = S_iter(Sb, fx);
            state = FLUSH0();
            if (state != ~0u) break;
          }
          base = seg_end;
        }
      }
      donem |= Pc;
      if (state != ~0u || !badm) break;
      // ---- the first node that may differ: deflate_fast's longest_match over the INSERTED
      // same-hash positions (Z/deflate.c:1148-1289): 64 bucket entries per step, lanes test
      // insertion and compare bytes in parallel; the walk order is the lane order.
      fallbacks++;
      const int fln = __builtin_ctzll(badm);
      const uint32_t f = wb + (uint32_t)fln;
      const uint32_t Sf = S_iter(Sb, f);
      if (!((batchm >> fln) & 1ull)) {   // the next batch: up to eight of the bad nodes left, from fln on
        const uint64_t cf0 = STEP_CLOCK();
        const uint32_t nbad = (uint32_t)__popcll(badm);
        const uint32_t G = nbad >= 5 ? 8u : nbad >= 3 ? 4u : nbad;
        const uint32_t nb = nbad < G ? nbad : G;
        uint64_t m = badm;
        batchm = 0;
        for (uint32_t i = 0; i < nb; i++) { batchm |= m & (0ull - m); m &= m - 1ull; }
        fast_exact_walks(batchm, nb, G, wb, Sb, sxl, rml, rms);
        bS = 64u / G;
        cyc_fb += STEP_CLOCK() - cf0;
      }
      const uint32_t gidx = (uint32_t)__popcll(batchm & ((1ull << fln) - 1ull));
      const uint32_t ml = uni((uint32_t)__builtin_amdgcn_readlane((int)rml, (int)(gidx * bS)));
      const uint32_t ms = uni((uint32_t)__builtin_amdgcn_readlane((int)rms, (int)(gidx * bS)));
      const uint32_t twt = uni((uint32_t)__builtin_amdgcn_readlane((int)wt, fln));
      const uint32_t tL = uni((uint32_t)__builtin_amdgcn_readlane((int)L, fln));
      if (ml >= 3 ? (twt == 2 && tL == ml) : twt == 1) {   // same step: the path stands
        if (ml >= 3 && lane == fln) Dx = f - ms;
        badm &= badm - 1ull;
        continue;
      }
      // the path changes at f: its exact step, then a new window after it
      fallbacks += 1ull << 32;   // diagnostics: walks that changed the path (high half)
      const uint32_t step = ml >= 3 ? ml : 1u;
      span_set(f, f + step, [&](uint32_t p, uint32_t& y, uint32_t& Ly) { y = f; Ly = ml >= 3 ? ml : 0u; });
      const bool full = tally1(ml >= 3 ? (((f - ms) << 8) | (ml - 3u)) : (uint32_t)in[f]);
      if (full) {
        z.p = f + step;
        z.S = Sf;
        state = FLUSH0();
      }
      qnext = f + step;
      restart = true;
      break;
    }
    t1 = STEP_CLOCK(); csec[3] += t1 - t0;
    if (state != ~0u) break;
    if (!restart && need) { state = TR_NEED_R; z.p = qn; break; }
    q = qnext;
  }
  if (state == ~0u) {
    z.p = n;
    z.S = S_iter(Sb, n);
  }
  }

  __device__ __forceinline__ void parse_slow() {
  // deflate_slow (Z/deflate.c:1730-1853), lane-parallel.
  // After an emitted match (and at the start) deflate_slow's state is canonical: prev_length 2,
  // no pending literal; after a literal with no match pending it is prev_length 2 with a pending
  // literal.  So the iterations from a position x up to the next canonical state -- "the walk
  // from x": either no match at x (next state at x + 1), or a lazy chain of c improving matches
  // that emits literals x .. m-1 and then the match at m = x + c (next state at m + length) --
  // depend on x alone.  A window computes the walks from its 64 positions in lanes, the scalar
  // unit follows the parse path through them (one hop per match or literal run), and the path's
  // symbols are tallied lane-parallel in position order, which is deflate_slow's tally order.
  // Window slides are a function of the iteration position (fill_window runs at the top of the
  // iteration when lookahead < MIN_LOOKAHEAD), so each lane evaluates them itself.
  uint32_t q = 0, ma = 0, Sb = 0, prevb = 0;   // canonical position, pending literal, S there, byte q-1
  bool need = false;
  while (q < n) {
    const uint32_t wb = q, bal = wb & ~63u;
    uint64_t t0 = STEP_CLOCK();
    while (hi < bal + RING_SLOW) {
      ring[(hi + lane) & (RING_SLOW - 1)] = pf;
      hi += 64;
      if (hi < n) pf = Rt[hi + lane];
    }
    Sb = S_iter(Sb, wb);
    if (ATZ_STEP_CLOCKS) { (void)ring[wb & (RING_SLOW - 1)]; __builtin_amdgcn_s_waitcnt(0); }
    uint64_t t1 = STEP_CLOCK(); csec[0] += t1 - t0; t0 = t1;
    // ---- the walk from x = wb + lane: wt 0 none (x >= n), 1 no match, 2 match, 3 needs R >= x_lim
    const uint32_t x = wb + lane;
    uint32_t wt = 0, nxt = 0, c = 0, L = 0, D = 0;
    uint32_t rd_last = 0, rd_ey = ~0u;   // rec: last entry the walk read, first quarter-budget read
    uint32_t w_len = 0, w_imp = 0;       // longest length the walk read; longest PL a lazy read improved
    if (x < n) {
      uint32_t qq = x, PL = 2, PD = 0;
      for (;;) {
        if (qq >= xlim) { wt = 3; break; }
        if (rec && (PL == 2 || PL < z.lazy)) {
          rd_last = qq;
          if (PL != 2 && PL >= z.good && rd_ey == ~0u) rd_ey = qq;
        }
        const uint64_t e64 = ring[qq & (RING_SLOW - 1)];
        const uint32_t ex = (uint32_t)e64, ey = (uint32_t)(e64 >> 32);
        bool hv = qq + 3u <= n && (ey & 1u);
        if (!noslide && hv) {   // hash_head == S is NIL after a slide (only right after one)
          const uint32_t Sq = S_iter(Sb, qq);
          if (Sq != 0 && qq - Sq <= maxd) {
            const uint32_t si = sidx[qq];
            hv = (bpos[si] & BUCKET_FIRST) || (bpos[si - 1] & ~BUCKET_FIRST) != Sq;
          }
        }
        if (PL == 2) {   // first iteration of the walk (qq == x)
          const uint32_t len = ex >> 23, dist = (ex >> 8) & 0x7fffu;
          if (hv && len > w_len) w_len = len;
          uint32_t ML = hv && len > 2 ? len : 2u;
          if (ML == 3 && dist > 4096) ML = 2;   // TOO_FAR
          if (ML == 2) { wt = 1; nxt = x + 1; break; }
          PL = ML; PD = dist; qq++;
          continue;
        }
        if (PL < z.lazy && hv) {
          const uint32_t ev = PL >= z.good ? ey : ex;
          const uint32_t len = ev >> 23;
          if (len > w_len) w_len = len;
          if (len > PL) { if (PL > w_imp) w_imp = PL; PL = len; PD = (ev >> 8) & 0x7fffu; c++; qq++; continue; }
        }
        wt = 2; L = PL; D = PD; nxt = qq - 1 + PL;
        break;
      }
    }
    // ---- follow the parse path through the window
    const uint64_t Am = __ballot(wt == 1), Nm = __ballot(wt == 3);
    t1 = STEP_CLOCK(); csec[1] += t1 - t0; t0 = t1;
    const uint32_t rel = wt == 1 ? run_end_rel(Am, lane) : wt == 2 ? nxt - wb : 0xffffu;
    const WinPath wp = follow_path(rel, Nm, n - wb < 64 ? n - wb : 64u);
    bool onp;
    uint32_t mab;
    path_lane(wp, Am, ma, lane, onp, mab);
    need = wp.need;
    const uint32_t qn = wb + wp.end;
    if (onp && (wt == 1 || wt == 2)) {   // the parse's own walks (diagnostics for level equivalence)
      run_len = w_len > run_len ? w_len : run_len;
      run_imp = w_imp > run_imp ? w_imp : run_imp;
    }
    if (rec && onp && (wt == 1 || wt == 2))   // the walk's reads: x full-budget, then by PL
      for (uint32_t i = x; i <= rd_last; i++) {
        const uint64_t e64 = ring[i & (RING_SLOW - 1)];
        rtab[i] = (i == x || i < rd_ey) ? ((e64 & 0xffffff00ull) | 1ull) : ((e64 & 0xffffff0000000000ull) | (1ull << 32));
      }
    // pending literal at qn: after a run yes, after a match no
    const uint32_t man = wp.H ? (uint32_t)((Am >> (63 - __builtin_clzll(wp.H))) & 1ull) : ma;
    // ---- tally the path's symbols: node x emits [literal x-1 if pending], literals x..m-1, match
    t1 = STEP_CLOCK(); csec[2] += t1 - t0; t0 = t1;
    const uint32_t cnt = onp ? mab + (wt == 2 ? c + 1u : 0u) : 0u;
    const uint64_t ltm = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t T;
    const uint32_t o = wave_excl_sum(cnt, ltm, T);
    z.nsym += T;
    uint32_t base = 0;
    while (base < T) {
      const uint32_t room = z.lbs - 1u - z.last_lit;
      const uint32_t seg_end = T - base < room ? T : base + room;
      const uint32_t klo = o > base ? 0u : base - o;
      const uint32_t khi = o + cnt < seg_end ? cnt : (seg_end > o ? seg_end - o : 0u);
      for (uint32_t k = klo; k < khi; k++) {
        const uint32_t j = k - mab;   // k == 0 with mab: literal x-1
        uint32_t v;
        if (mab && k == 0) v = lane == 0 ? prevb : (uint32_t)ring[(x - 1) & (RING_SLOW - 1)] & 0xffu;
        else if (j < c) v = (uint32_t)ring[(x + j) & (RING_SLOW - 1)] & 0xffu;
        else v = 0x80000000u | (D << 8) | (L - 3u);
        if (v & 0x80000000u) {
          v &= 0x7fffffffu;
          __hip_atomic_fetch_add(&s.f.lfreq2[(257u + len_code(L - 3u)) >> 1], 1u << (16 * ((257u + len_code(L - 3u)) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(&s.f.dfreq2[(dist_code(D - 1u)) >> 1], 1u << (16 * ((dist_code(D - 1u)) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          __hip_atomic_fetch_add(&s.f.lfreq2[(v) >> 1], 1u << (16 * ((v) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        syms[(saving || MW ? sbase : 0u) + z.last_lit + (o + k - base)] = v;
      }
      z.last_lit += seg_end - base;
      if (z.last_lit == z.lbs - 1u) {
        // flush after symbol seg_end - 1: strstart = its iteration + 1 for a literal (the
        // literal of y is tallied at iteration y + 1), match end for a match (tallied at m + 1)
        const uint32_t g = seg_end - 1u;
        const bool own = cnt && o <= g && g < o + cnt;
        uint32_t fp = 0, fit = 0;
        if (own) {
          const uint32_t k = g - o, j = k - mab;
          if (mab && k == 0) { fp = x; fit = x; }
          else if (j < c) { fp = x + j + 1u; fit = fp; }
          else { fp = x + c + L; fit = x + c + 1u; }
        }
        const uint64_t om = __ballot(own);
        const int ol = (int)__builtin_ctzll(om);
        z.p = (uint32_t)__builtin_amdgcn_readlane((int)fp, ol);
        z.S = S_iter(Sb, (uint32_t)__builtin_amdgcn_readlane((int)fit, ol));
        state = FLUSH0();
        if (state != ~0u) break;
      }
      base = seg_end;
    }
    t1 = STEP_CLOCK(); csec[3] += t1 - t0;
    if (state != ~0u) break;
    if (need) { state = TR_NEED_R; z.p = qn; break; }
    prevb = qn > 0 ? (uint32_t)ring[(qn - 1u) & (RING_SLOW - 1)] & 0xffu : 0u;   // read when man: qn - 1 < wb + 64
    q = qn;
    ma = man;
  }
  if (state == ~0u) {
    // end of input: the pending literal goes into the final block without a flush check
    if (ma) {
      const uint32_t v = prevb;
      saved_flags |= 2;
      if (lane == 0) {
        syms[(saving || MW ? sbase : 0u) + z.last_lit] = v;
        __hip_atomic_fetch_add(&s.f.lfreq2[(v) >> 1], 1u << (16 * ((v) & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      z.last_lit++;
      z.nsym++;
    }
    z.p = n;
    z.S = S_iter(Sb, n);
  }
  }

  // the final block, the trailer and the final gates (main.cpp:632-681); multi-wave: the last block's
  // hand-over
  __device__ __forceinline__ void end_parse() {
  if (MW && state == ~0u) {
    // the final gates run on the last block's flusher; a refused hand-over (the trial was decided or
    // skipped first) leaves the last block's symbols out of sbase, so the sequence is not complete
    if (publish(1)) saved_flags |= 1;   // every symbol tallied: a saving trial's sequence is complete
    else state = TR_DECIDED;
  } else if (state == ~0u) {
    saved_flags |= 1;   // every symbol tallied: a saving trial's sequence is complete
    FLUSH(1);
    // adler32 trailer
    uint32_t ad = A.adler[tr.stream];
    uint32_t be = ((ad >> 24) & 0xff) | ((ad >> 8) & 0xff00) | ((ad << 8) & 0xff0000) | (ad << 24);
    put_bits(b, stg, be, 32, lane);   // after the last block: the ring is no longer read
    flush_bits_bytes(b, stg, lane);
    // final gates (main.cpp:632-681)
    if (b.overflow) state = TR_OVERFLOW;
    else if (full_needed) state = TR_FULL;
    else {
      uint64_t thr = A.o.shortcut_len - A.o.recomp_tresh;
      uint64_t L = b.pos;
      int64_t dd = (int64_t)(L - b.clen);
      uint64_t ad2 = (uint64_t)(dd < 0 ? -dd : dd);
      if (b.shortcut && b.eq_sc < thr) state = TR_SHORTCUT;
      else if (ad2 > A.o.sizediff_tresh) state = TR_SIZEDIFF;
      else state = TR_FULL;
    }
    spec_stop(s, A, tr.best_ident, state, uni(b.eq_all), uni(b.clen), lane);
  }
  if constexpr (MW) {   // no more blocks: flushers waiting past the last one stop; TR_NEED_R abandons the rest
    LDS MWCtl& ctl = (*(LDS MWPart*)&shm.mw).ctl;
    if (lane == 0) ctl.nblocks = nblk;
    st_rel(ctl.parse_done, 1u, lane);
    if (state == TR_NEED_R) st_rel(ctl.stop, 1u, lane);
  }
  }

  // the flushers' outcome (multi-wave) and the trial's result
  __device__ __forceinline__ void finish() {
  if constexpr (MW) {
    __syncthreads();   // every flusher has stopped
    if (wave != 0) return;
    LDS MWPart& mw = *(LDS MWPart*)&shm.mw;
    const uint32_t cs = uni(mw.ctl.state);
    // a flusher's decision stands (it is final); TR_NEED_R only when none was reached
    if (state != TR_NEED_R || cs != ~0u) state = cs;
    hazard |= uni(mw.ctl.hazard);
    if (lane == 0) {
      for (int f = 0; f < MW_F; f++) {
        b.cyc_tree += mw.fl[f].cyc_tree; b.cyc_emit += mw.fl[f].cyc_emit;
        b.cyc_heap += mw.fl[f].cyc_heap; b.cyc_scan += mw.fl[f].cyc_scan;
      }
    }
  }
  uint32_t rmax = (run_imp << 16) | run_len;   // both < 2^16: per-field maxima by two reductions
  {
    uint32_t a = run_imp, bl = run_len;
    for (int d = 32; d >= 1; d >>= 1) {
      const uint32_t oa = __shfl_xor(a, d, 64), ob = __shfl_xor(bl, d, 64);
      a = a > oa ? a : oa; bl = bl > ob ? bl : ob;
    }
    rmax = (a << 16) | bl;
  }
  if (lane == 0) {
    TrialRes r;
    r.state = state;
    r.flags = hazard | (b.shortcut ? 2u : 0u);
    r.out_len = b.pos;
    r.ident = b.eq_all;
    r.symbols = z.nsym;
    r.parsed = z.p;
    r.fallbacks = fallbacks;
    r.cyc_total = clock64() - cstart;
    r.cyc_tree = b.cyc_tree;
    r.cyc_emit = b.cyc_emit;
    r.blocks = b.blocks;
    r.cyc_heap = b.cyc_heap;
    r.cyc_scan = b.cyc_scan;
    r.cyc_send = b.cyc_send;
    for (int i = 0; i < 4; i++) r.cyc_sec[i] = csec[i];
    r.cyc_fallback = cyc_fb;
    r.saved_syms = sbase;
    r.saved_flags = saved_flags;
    r.reads_max = rmax;
    r.rt0 = rtstart;
    r.rt1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    A.res[t] = r;
  }
  }

  __device__ __forceinline__ void run() {
    if constexpr (MW) {
      LDS MWPart& mw = *(LDS MWPart*)&shm.mw;
      if (wave == 0) {
        if (lane < MW_F) { mw.slot[lane].seq = 0; mw.fl[lane].cyc_tree = 0; mw.fl[lane].cyc_emit = 0;
                          mw.fl[lane].cyc_heap = 0; mw.fl[lane].cyc_scan = 0; }
        if (lane == 0) {
          mw.ctl.next_emit = 0; mw.ctl.stop = 0; mw.ctl.parse_done = 0; mw.ctl.nblocks = 0;
          mw.ctl.state = ~0u; mw.ctl.hazard = 0;
        }
        spec_init(s, A, tr, lane);
        // decided before any flusher starts: the parse stops at its first hand-over (a separate
        // no-parse path would cost the kernel 25 VGPRs)
        if (spec_stopped(s) && lane == 0) { mw.ctl.state = TR_SKIPPED; mw.ctl.stop = 1; }
      }
      __syncthreads();
      if (wave != 0)
        trial_flusher(A, s, mw, tr, (const GLOBAL uint32_t*)syms, (const GLOBAL uint8_t*)in, z.level, z.lbs, full_needed,
                      wave - 1, lane);
    }
    if constexpr (!MW) spec_init(s, A, tr, lane);   // (checked at each block flush: FLUSH0)
    if (wave == 0) {   // the parse; every wave of a single-wave trial
      parse_setup();
      if constexpr (KIND == 0) parse_stored();
      else if (replay) parse_replay();
      else if constexpr (KIND == 1) parse_fast();
      else parse_slow();
      end_parse();
    }
    finish();
  }
};

template <int KIND, typename SH>
__device__ void trial_body(const SweepArgs& A, SH& shm, int lane) {
  if constexpr (!HasMW<SH>::value) {
    // a single-wave trial whose stream an earlier trial of the round has stopped ends before any set-up
    // (kept out of TrialRun: a path there costs the parse registers; multi-wave ones decide on wave 0)
    const Trial& tr = A.trials[blockIdx.x];
    const uint32_t j = uni(tr.spec_j);
    if (A.stopj && j &&
        uni(__hip_atomic_load((const GLOBAL uint32_t*)A.stopj + uni(tr.stream), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < j) {
      if (lane == 0) {
        TrialRes r = {};
        r.state = TR_SKIPPED;
        A.res[blockIdx.x] = r;
      }
      return;
    }
  }
  TrialRun<KIND, SH> run(A, shm, lane);
  run.run();
}

#ifndef TRIAL_SLOW_WAVES
#define TRIAL_SLOW_WAVES 4   // waves per SIMD the trial kernels (and flush_block, which they share) are register-capped for:
                             // the slow kind's 10 KB of LDS allows 16 waves per CU
#endif
__global__ __launch_bounds__(64, TRIAL_SLOW_WAVES) void k_trial_stored(SweepArgs A) {
  __shared__ struct { TrialShared t; uint64_t ring[(STAGE_WORDS + 1) / 2]; } shm;   // ring: staging only
  trial_body<0>(A, shm, threadIdx.x);
}
template <uint32_t INS>
__global__ __launch_bounds__(64, TRIAL_SLOW_WAVES) void k_trial_fast(SweepArgs A) {
  __shared__ TrialSharedFast<INS> shm;
  trial_body<1>(A, shm, threadIdx.x);
}
__global__ __launch_bounds__(64, TRIAL_SLOW_WAVES) void k_trial_slow(SweepArgs A) {
  __shared__ TrialSharedSlow shm;
  trial_body<2>(A, shm, threadIdx.x);
}
// multi-wave trials (small blocks): wave 0 parses, waves 1..MW_F flush
static constexpr uint32_t MW_THREADS = 64 * (1 + MW_F);
template <uint32_t INS>
__global__ __launch_bounds__(MW_THREADS, TRIAL_SLOW_WAVES) void k_trial_fast_mw(SweepArgs A) {
  __shared__ TrialSharedFastMW<INS> shm;
  trial_body<1>(A, shm, (int)(threadIdx.x & 63));
}
__global__ __launch_bounds__(MW_THREADS, TRIAL_SLOW_WAVES) void k_trial_slow_mw(SweepArgs A) {
  __shared__ TrialSharedSlowMW shm;
  trial_body<2>(A, shm, (int)(threadIdx.x & 63));
}

}  // namespace atz
