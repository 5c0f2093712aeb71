// Micro-benchmarks of serial wave-uniform code on gfx950 (one wave alone on a CU): cycles per
// iteration of dependent chains that the decoder / parse loops are built from.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }

// 0: dependent SALU adds/xor/shift (4 ops per iteration)
// 1: readlane chain: idx = readlane(v, idx & 63)
// 2: v_cmp -> ballot -> s_ff1 -> readlane chain (canonical decode core)
// 3: data-dependent uniform branch (taken ~50%)
// 4: ds_read_u8 dependent chain (LDS latency)
// 5: s_brev + shift + v_lshrrev + v_sub + v_cmp + s_ff1 + v_add + readlane (decode step)
__global__ __launch_bounds__(64) void k_ub(const uint32_t* in, uint64_t* out, int which) {
  __shared__ uint8_t lds[4096];
  const int lane = threadIdx.x;
  for (int i = lane; i < 4096; i += 64) lds[i] = (uint8_t)(in[i & 1023] & 255);
  __syncthreads();
  uint32_t v = in[lane];
  uint32_t s = __builtin_amdgcn_readfirstlane(in[100]);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (which == 0) {
    for (int i = 0; i < ITERS; i++) { s = (s ^ (s >> 3)) + 0x9e3779b9u; s = (s << 1) | (s >> 31); }
  } else if (which == 1) {
    for (int i = 0; i < ITERS; i++) s = rl(v, s & 63) + s;
  } else if (which == 2) {
    for (int i = 0; i < ITERS; i++) {
      uint64_t m = __ballot((v ^ s) & 1);
      uint32_t L = m ? (uint32_t)__ffsll((unsigned long long)m) - 1 : 0;
      s = rl(v, L) + s;
    }
  } else if (which == 3) {
    for (int i = 0; i < ITERS; i++) {
      if ((s * 0x9e3779b9u) >> 31) s = s * 3 + 1; else s = (s >> 1) ^ 0x1234;
    }
  } else if (which == 4) {
    for (int i = 0; i < ITERS; i++) {
      uint32_t x = lds[(s + lane) & 4095];
      s = __builtin_amdgcn_readfirstlane(x) + s * 5;
    }
  } else if (which == 5) {
    const uint32_t lsh = (lane >= 1 && lane <= 15) ? (uint32_t)(15 - lane) : 31u;
    const uint32_t first = v & 0x7fff, count = (lane >= 1 && lane <= 15) ? (v >> 20) : 0;
    for (int i = 0; i < ITERS; i++) {
      const uint32_t r = __builtin_bitreverse32(s) >> 17;
      const uint32_t c = r >> lsh;
      const uint64_t m = __ballot((c - first) < count);
      const uint32_t L = m ? (uint32_t)__ffsll((unsigned long long)m) - 1 : 1;
      const uint32_t idx = rl(c + v, L);
      s = (s >> L) + idx;
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[0] = t1 - t0; out[1] = s; }
}

int main() {
  uint32_t* d_in; uint64_t* d_out;
  hipMalloc(&d_in, 4096 * 4); hipMalloc(&d_out, 16);
  uint32_t h[4096];
  for (int i = 0; i < 4096; i++) h[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
  hipMemcpy(d_in, h, sizeof h, hipMemcpyHostToDevice);
  const char* names[] = {"salu 4-op chain", "readlane chain", "ballot+ff1+readlane", "uniform branch 50%", "ds_read_u8 chain",
                         "canonical decode step"};
  for (int w = 0; w < 6; w++) {
    uint64_t o[2];
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(k_ub, dim3(1), dim3(64), 0, 0, d_in, d_out, w);
      hipMemcpy(o, d_out, 16, hipMemcpyDeviceToHost);
    }
    printf("%-24s %7.1f cyc/iter\n", names[w], (double)o[0] / ITERS);
  }
  return 0;
}
