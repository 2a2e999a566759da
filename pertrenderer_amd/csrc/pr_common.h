// Shared device helpers for libpertrender (gfx950 / CDNA4, wave64).
//
// * Philox4x32-10 counter-based generator (Salmon et al., SC'11): keyed by a
//   64-bit seed, counter = (pixel, slot, sample-group, stream tag).  One call
//   yields 4 words = 4 Monte-Carlo samples of one (pixel, slot), so forward and
//   backward regenerate identical noise without storing it.
// * Gaussian samples by Box-Muller on the hardware transcendentals
//   (v_log_f32 = log2, v_sqrt_f32, v_sin/cos_f32 taking revolutions); Cauchy
//   samples as tan(pi (u - 1/2)) on the same sin/cos.
// * Error plumbing for the C ABI (thread-local message).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/pertrender.h"

#define PR_DEV __device__ __forceinline__
#define PR_HD __host__ __device__ __forceinline__

namespace pr {

constexpr int kThreads = 256;  // 4 waves per workgroup

// stream tags (4th counter word) so the two draws never share a counter
constexpr uint32_t kTagRast = 0x52415354u;  // "RAST"
constexpr uint32_t kTagAgg = 0x41474752u;   // "AGGR"
constexpr uint32_t kTagTail = 0x5441494Cu;  // "TAIL": joint draw of a pixel's masked agg slots

struct U4 {
  uint32_t x, y, z, w;
};

// Philox4x32-R (Salmon et al., SC'11).  The noise streams use R = PR_PHILOX_ROUNDS = 7 (round 6):
// Salmon et al. report Philox4x32 Crush-resistant (TestU01 BigCrush) from 7 rounds, Random123's
// default 10 keeps a safety margin.  The blend kernels are bound by their generator at large S, so
// 7 rounds measured cfg 2 3588 -> 3680 and cfg 4 998 -> 1060 frames/s (DESIGN.md §4 Noise).  The
// round function is pinned by Random123's 10-round known-answer vectors through pr_philox(rounds 10).
#ifndef PR_PHILOX_ROUNDS
#define PR_PHILOX_ROUNDS 7
#endif
constexpr int kPhiloxRounds = PR_PHILOX_ROUNDS;
template <int R>
PR_DEV U4 philox4x32(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
PR_DEV U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) { return philox4x32<10>(c, k0, k1); }

// uniform in (0,1): odd 24-bit integer * 2^-24, exact in fp32, never 0 or 1
PR_DEV float u01(uint32_t r) { return (float)((r >> 8) | 1u) * 5.9604644775390625e-08f; }

PR_DEV uint32_t word(const U4& u, int i) {
  return i == 0 ? u.x : (i == 1 ? u.y : (i == 2 ? u.z : u.w));
}

// 4 N(0,1) samples from one Philox block: two Box-Muller pairs.
PR_DEV void gauss4(const U4& u, float e[4]) {
  const float r0 = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(u.x)));
  const float a0 = u01(u.y);
  const float r1 = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(u.z)));
  const float a1 = u01(u.w);
  e[0] = r0 * __builtin_amdgcn_cosf(a0);
  e[1] = r0 * __builtin_amdgcn_sinf(a0);
  e[2] = r1 * __builtin_amdgcn_cosf(a1);
  e[3] = r1 * __builtin_amdgcn_sinf(a1);
}

// 4 standard Cauchy samples tan(pi (u - 1/2)) from one Philox block, on the hardware
// sin/cos (revolutions: angle pi (u - 1/2) = 2 pi t with t = (u - 1/2) / 2), clamped
// to +-1e7 as the reference clamps its draws (smoothrast.py:24, smoothagg.py:27).
PR_DEV void cauchy4(const U4& u, float e[4]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float t = (u01(w[i]) - 0.5f) * 0.5f;
    const float c = __builtin_amdgcn_sinf(t) * __builtin_amdgcn_rcpf(__builtin_amdgcn_cosf(t));
    e[i] = fminf(fmaxf(c, -1e7f), 1e7f);
  }
}

// score function d/d eps (-log density): eps (Gaussian) or 2 eps / (1 + eps^2) (Cauchy)
PR_DEV float noise_score(float e, bool cauchy) { return cauchy ? (2.f * e) / (1.f + e * e) : e; }

PR_DEV U4 philox_block(uint64_t seed, uint32_t pixel, uint32_t slot, uint32_t group, uint32_t tag) {
  return philox4x32<kPhiloxRounds>(U4{pixel, slot, group, tag}, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// k-th index of [0, n) in centre-out order (n/2, n/2-1, n/2+1, ...): workgroups over
// image rows are dispatched from the middle outwards, so the rows of a centred object
// (the expensive ones) start first and the cheap border rows fill the tail.
PR_DEV uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// pr_seed_advance's update of a device key base (DeviceSeed.advance)
PR_DEV uint64_t seed_next(uint64_t s) { return mix64(s + 0x9E3779B97F4A7C15ull); }

PR_DEV int centre_out(int k, int n) { return (k & 1) ? n / 2 - 1 - (k >> 1) : n / 2 + (k >> 1); }

// --------------------------------------------------------------------- math
PR_DEV float heaviside1(float x) { return x >= 0.f ? 1.f : 0.f; }  // torch.heaviside(x, 1)


template <typename T>
PR_DEV T ld(const T* p) { return *p; }

}  // namespace pr

// ------------------------------------------------------------------- errors
namespace pr {
int set_error(int code, const std::string& msg);
int check_launch(const char* what);
// live per-kernel timing (pr_ktimer_arm): which = 0 before the dominant kernel's launch, 1 after
void ktimer_mark(int which, const char* kernel, hipStream_t st);

// PR_BLEND_SOFT: the deterministic SoftRast + SoftAgg blend (pr_softblend.hip)
size_t soft_blend_workspace(const PRBlendParams& p);
int soft_blend_fwd(const PRBlendFwdArgs& a, hipStream_t st);
int soft_blend_bwd(const PRBlendBwdArgs& a, hipStream_t st);

// Deterministic ordered scatter-add (pr_detsum.hip), the PR_DETERMINISTIC mode of the passes
// that scatter with float atomics: out[k] = sum of the C components of the entries with key k,
// in entry order.  Caller: detsum_layout on a workspace of detsum_workspace bytes, fill
// keys[0..n) (keys >= M are dropped), detsum_sort, then write each entry's components at its
// sorted position (vals_sorted[i * C + c] for the entry idx_sorted[i]) -- or fill vals in entry
// order and detsum_gather -- and detsum_reduce.  chunk <= 0: one sequential pass per key (the
// order of a serial loop); chunk > 0: sequential chunk sums of `chunk` entries, then the chunk
// sums in order (long segments).
struct DetSum {
  int64_t n = 0, M = 0;
  int C = 0, end_bit = 0;
  uint32_t* keys = nullptr;
  uint32_t* keys_sorted = nullptr;
  uint32_t* idx = nullptr;
  uint32_t* idx_sorted = nullptr;
  float* vals = nullptr;
  float* vals_sorted = nullptr;
  uint32_t* start = nullptr;
  uint32_t* end = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
};
size_t detsum_workspace(int64_t n, int64_t M, int C);
int detsum_layout(void* ws, size_t bytes, int64_t n, int64_t M, int C, DetSum& d);
int detsum_sort(const DetSum& d, hipStream_t st);
int detsum_gather(const DetSum& d, hipStream_t st);
int detsum_reduce(const DetSum& d, float* out, int64_t chunk, bool accumulate, hipStream_t st);
// one sequential pass per key; first: out = the batch's sums (0 for keys without entries), else the
// chains continue from out (keys without entries keep it)
int detsum_reduce_chain(const DetSum& d, float* out, bool first, hipStream_t st);
// entries per batch of the deterministic-mode scatters (bounds their workspace: ~90 B per entry);
// PR_DET_BATCH overrides (tests drive the batched path on small frames; read per call)
int64_t det_batch();
}  // namespace pr
