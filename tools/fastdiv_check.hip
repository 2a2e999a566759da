// Round-4 experiment record (profiles/r4_experiments.txt, "rast_fwd with correctly rounded reciprocal
// divisions"): bitwise check of the division helpers that variant used (div_rn / rcp_rn; not in the
// product, which kept the IEEE divisions) against IEEE division on the GPU.  rcp_rn: every significand at exponents -30..32 (all-ones significands are
// the reported exception).  div_rn with y = IEEE 1/b: random significands over the exponent ranges
// the forward admits (|b| in [2^-30, 2^32], quotients in (2^-92, 2^30]) plus quotients next to
// rounding midpoints.  Build / run:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o fastdiv_check tools/fastdiv_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ float div_rn(float a, float b, float y) {
  float q = a * y;
  float r = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(r, y, q);
  r = __builtin_fmaf(-b, q, a);
  return __builtin_fmaf(r, y, q);
}
__device__ float rcp_rn(float b, bool& ok) {
  const float y = __builtin_amdgcn_rcpf(b);
  ok = (__float_as_uint(b) & 0x7fffffu) != 0x7fffffu;
  return __builtin_fmaf(__builtin_fmaf(-b, y, 1.f), y, y);
}
__device__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}

// counters: [0] rcp mismatches (ok), [1] rcp mismatches (all-ones), [2] div mismatches with |a| >= 2^-100
// (the callers' range), [3] tests, [4] / [5] biased exponents of the smallest |a| / largest quotient among
// all mismatches, [6] all mismatches (operands below the callers' range included)
__global__ void rcp_check(int e0, unsigned long long* cnt) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (1u << 23)) return;
  const int e = e0 + (int)blockIdx.y;
  for (int sgn = 0; sgn < 2; ++sgn) {
    const float b = __uint_as_float(((uint32_t)sgn << 31) | ((uint32_t)(e + 127) << 23) | m);
    bool ok;
    const float y = rcp_rn(b, ok);
    if (__float_as_uint(y) != __float_as_uint(1.f / b)) atomicAdd(&cnt[ok ? 0 : 1], 1ull);
  }
}

__global__ void div_check(uint64_t seed, int iters, unsigned long long* cnt) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long bad = 0, cnt_all = 0;
  for (int i = 0; i < iters; ++i) {
    const uint64_t k = (seed + t) * 0x9e3779b97f4a7c15ull + (uint64_t)i * 0x632be59bd9b4e019ull;
    const uint32_t r0 = mix(k), r1 = mix(k + 1), r2 = mix(k + 2);
    const int eb = (int)(r2 % 63u) - 30;          // |b| in [2^-30, 2^33)
    const int eq = (int)((r2 >> 8) % 121u) - 91;  // quotient exponent in [-91, 29]
    const float b = __uint_as_float(((r2 >> 31) << 31) | ((uint32_t)(eb + 127) << 23) | (r0 & 0x7fffffu));
    float a;
    if (i & 1) {  // a = RN(b * q) for a random q: quotients next to representable values / midpoints
      const float q = __uint_as_float(((uint32_t)(eq + 127) << 23) | (r1 & 0x7fffffu));
      a = b * q;
      const uint32_t d = (r1 >> 23) % 5u;
      a = __uint_as_float(__float_as_uint(a) + d - 2u);
    } else {
      const int ea = eq + eb;
      a = __uint_as_float(((r1 >> 31) << 31) | ((uint32_t)(ea + 127) << 23) | (r1 & 0x7fffffu));
    }
    const float y = 1.f / b;
    if (__float_as_uint(div_rn(a, b, y)) != __float_as_uint(a / b)) {
      // the exponent of the smallest |a| and the largest |a / b| that missed
      atomicMin((unsigned*)&cnt[4], (__float_as_uint(a) >> 23) & 0xffu);
      atomicMax((unsigned*)&cnt[5], (__float_as_uint(a / b) >> 23) & 0xffu);
      bad += fabsf(a) >= 0x1p-100f;  // inside the callers' operand range
      ++cnt_all;
    }
  }
  if (bad) atomicAdd(&cnt[2], bad);
  if (cnt_all) atomicAdd(&cnt[6], cnt_all);
  atomicAdd(&cnt[3], (unsigned long long)iters);
}

int main() {
  unsigned long long* d;
  unsigned long long h[7] = {0, 0, 0, 0, 0xffffffffull, 0, 0};
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipLaunchKernelGGL(rcp_check, dim3((1u << 23) / 256, 63), dim3(256), 0, 0, -30, d);
  for (int s = 0; s < 16; ++s) hipLaunchKernelGGL(div_check, dim3(4096), dim3(256), 0, 0, (uint64_t)s << 40, 512, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  printf("rcp_rn: %llu significands x 63 exponents x 2 signs: mismatches %llu (ok) %llu (all-ones, reported)\n",
         1ull << 23, h[0], h[1]);
  printf("div_rn: %llu quotients (|b| in [2^-30, 2^33), |a / b| in [2^-91, 2^30)): mismatches %llu with |a| >= 2^-100, "
         "%llu in all (smallest |a| 2^%d, largest |a / b| 2^%d)\n",
         h[3], h[2], h[6], h[6] ? (int)h[4] - 127 : 0, h[6] ? (int)h[5] - 127 : 0);
  return (h[0] || h[2]) ? 2 : 0;
}
