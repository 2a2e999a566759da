// Throughput microbenchmark of the blend kernels' noise generator on one MI355X:
// Philox4x32 blocks/s (10 and 7 rounds; 64-bit multiply vs separate hi/lo multiplies) and
// Box-Muller normals/s, every lane busy, result folded into one store per thread.
//   hipcc -O3 --offload-arch=gfx950 -o tools/philox_bench tools/philox_bench.hip && tools/philox_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../pertrenderer_amd/csrc/pr_common.h"

using pr::U4;

template <int R>
__device__ __forceinline__ U4 philox_r(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

template <int R>
__device__ __forceinline__ U4 philox_hilo(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// MODE 0: philox-10 (64-bit mul), 1: philox-10 hi/lo, 2: philox-7, 3: philox-10 + gauss4,
// 4: gauss4 on a cheap hash (Box-Muller alone), 5: philox-7 + gauss4
template <int MODE>
__global__ void __launch_bounds__(256) bench_kernel(float* out, int iters, uint64_t key) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  uint32_t ax = 0;
  float af = 0.f;
  for (int i = 0; i < iters; ++i) {
    const U4 c{t, (uint32_t)i, 7u, pr::kTagAgg};
    U4 u;
    if constexpr (MODE == 0 || MODE == 3) u = philox_r<10>(c, k0, k1);
    else if constexpr (MODE == 1) u = philox_hilo<10>(c, k0, k1);
    else if constexpr (MODE == 2 || MODE == 5) u = philox_r<7>(c, k0, k1);
    else {
      const uint32_t h = (t * 0x9E3779B9u) ^ ((uint32_t)i * 0x85EBCA6Bu);
      u = U4{h, h ^ 0x68E31DA4u, h * 3u, h ^ 0xB5297A4Du};
    }
    if constexpr (MODE >= 3) {
      float e[4];
      pr::gauss4(u, e);
      af += (e[0] + e[1]) + (e[2] + e[3]);
    } else {
      ax ^= u.x ^ u.y ^ u.z ^ u.w;
    }
  }
  out[t] = af + (float)ax;
}

int main() {
  const int threads = 256, blocks = 256 * 32, iters = 1024;
  const double n = (double)threads * blocks * iters;
  float* d;
  hipMalloc(&d, sizeof(float) * threads * blocks);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"philox10 mad_u64", "philox10 hi/lo", "philox7 mad_u64", "philox10 + gauss4",
                         "gauss4 (hash input)", "philox7 + gauss4"};
  for (int m = 0; m < 6; ++m) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0);
      switch (m) {
        case 0: bench_kernel<0><<<blocks, threads>>>(d, iters, 0x1234567890ull); break;
        case 1: bench_kernel<1><<<blocks, threads>>>(d, iters, 0x1234567890ull); break;
        case 2: bench_kernel<2><<<blocks, threads>>>(d, iters, 0x1234567890ull); break;
        case 3: bench_kernel<3><<<blocks, threads>>>(d, iters, 0x1234567890ull); break;
        case 4: bench_kernel<4><<<blocks, threads>>>(d, iters, 0x1234567890ull); break;
        default: bench_kernel<5><<<blocks, threads>>>(d, iters, 0x1234567890ull); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-22s %8.3f ms  %7.1f G blocks/s  %7.1f G normals/s (if 4 per block)\n", names[m], best,
           n / (best * 1e-3) / 1e9, 4 * n / (best * 1e-3) / 1e9);
  }
  hipFree(d);
  return 0;
}
