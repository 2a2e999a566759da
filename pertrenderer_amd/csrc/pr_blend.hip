// Perturbed soft rasterization + perturbed-argmax aggregation (fused blend).
//
// Reference semantics (quentinll/pertrenderer, pure Python):
//   smoothrast.py:12-59   randomHeaviside fwd/bwd   (prob from perturbed signed distances)
//   smoothagg.py:10-73    randomArgmax fwd/bwd      (Monte-Carlo argmax over K+1 logits)
//   smoothagg.py:196-205  GaussianAgg.aggregate     (logit assembly, background logit)
//   smoothagg.py:292-337  log_corrected / prod_corrected backward conventions
//   random_rasterizer.py:34-56  smooth_rgb_blend    (alpha product, colour mix)
// Closed-form backward: SURVEY.md §3.2, restated in oracle/blend_oracle.py.
//
// MI355X layout.  One 256-thread workgroup (4 waves) owns PB <= 32 consecutive
// pixels, i.e. one contiguous (PB*K)-slot range of every fragment tensor:
//   * slot phases: thread t walks slots t, t+256, ... of the range (fully
//     coalesced loads/stores, (pixel, slot) tracked incrementally: no integer
//     division in the loop); per-slot intermediates go to LDS;
//   * pixel phases: 8 lanes per pixel (32 pixels = 256 threads) reduce over the
//     pixel's slots with xor-shuffles inside the 8-lane group;
//   * the agg Monte-Carlo argmax runs one thread per (pixel, 4-sample Philox
//     group, slot chunk) and merges chunk partials with shuffles.
// Nothing of size S x P x K is materialised: noise is regenerated from Philox
// (or read from injected tensors in parity mode).  In Philox mode two exact
// skips remove RNG work without changing any result (Box-Muller |eps| <= 5.77
// for 24-bit uniforms): a rast slot with |dist/sigma| > 5.8 has the same outcome
// for every sample, and an agg logit more than 2*5.8*gamma below the pixel's
// largest logit can never win.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "pr_common.h"
#include "pr_phong.h"

namespace pr {
namespace {

constexpr float kNegInf = -__builtin_inff();
constexpr float kEpsMaxBM = 5.8f;               // > sqrt(-2 ln 2^-24) = 5.7683

#ifdef PR_BLEND_PROFILE
// diagnostic build: per block [start, end (100 MHz), phases (shader clock) x8, hw id, flag];
// fwd blocks at [0, 1<<16), bwd blocks at [1<<16, 2<<16)
constexpr unsigned kBProfBlocks = 1 << 16;
constexpr int kBProfRec = 12;
__device__ long long g_blend_prof[2 * kBProfBlocks * kBProfRec];
#define PR_BPROF_DECL long long bst_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bt_ = __builtin_amdgcn_s_memtime(), \
                      brt_ = __builtin_amdgcn_s_memrealtime()
#define PR_BPROF_DUMP(which, rec)                                                              \
  if (threadIdx.x == 0 && (rec) < kBProfBlocks) {                                              \
    unsigned hw_;                                                                              \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                          \
    long long* r_ = g_blend_prof + ((size_t)(which) * kBProfBlocks + (rec)) * kBProfRec;       \
    r_[0] = brt_; r_[1] = (long long)__builtin_amdgcn_s_memrealtime();                          \
    for (int i_ = 0; i_ < 8; ++i_) r_[2 + i_] = bst_[i_];                                       \
    r_[10] = hw_; r_[11] = 1;                                                                  \
  }
#define PR_BSTAMP(i) (bst_[i] += __builtin_amdgcn_s_memtime() - bt_, bt_ = __builtin_amdgcn_s_memtime())
#else
#define PR_BPROF_DECL (void)0
#define PR_BSTAMP(i) (void)0
#endif

// minimum waves per SIMD the blend kernels are compiled for (caps their VGPRs); sweeps
// override with -DPR_BLEND_FWD_WPE=... / -DPR_BLEND_BWD_WPE=...
#ifndef PR_BLEND_FWD_WPE
#define PR_BLEND_FWD_WPE 1
#endif
#ifndef PR_BLEND_BWD_WPE
#define PR_BLEND_BWD_WPE 1
#endif


struct Geo {
  int64_t P, PK;  // pixels, slots
  int K, KP1, PB, HW;
  int qK, rK, qK1, rK1, qS, rS;  // 256 / {K, K+1, Sa} and remainders
  int lpp, lsh;                  // lanes per pixel in the pixel phases (256 / PB, 8..64) and log2
  int bpi;                       // blocks per image for the centre-out block order (0: linear)
  int tail;                      // backward: joint masked-tail draw allowed (PR_BLEND_TAIL=0: off)
  int empty;                     // empty-block shortcut allowed (PR_BLEND_EMPTY=0: off)
  int cap;                       // LDS entry records per workgroup (>= K + 1)
  int seg;                       // segment plan: entries per part E (0: static grid, passes of cap)
  int lsh_max;                   // segment plan: log2 of the most lanes per pixel a part may use
  int plan_fwd_list, plan_bwd_list;  // segment plan: int offsets of the two segment lists
  int pm, pmNBI, pmW, pmA;           // interleaved pixel blocks (block_pixel; pm = 0: consecutive)
  int sync_rel;                      // fused scalar reduction: acq_rel arrivals (last_arrival)
};

// a value every lane holds alike (read from LDS: a vector register) into a scalar register
PR_DEV int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Segment plan (PRBlendFwdArgs.plan), int32 words: the header (per kernel: segment count and the
// entries per part E it was cut with), the per-block entry totals of the forward's and the
// backward's pixel blocks (uint16, scratch), then the two segment lists (block << 6 | part, in
// dispatch order).  E is raised on dense frames so that the segments never exceed the kernels'
// grids (the host's bound T + X: every block's parts fit in T + (total entries) / E).
constexpr int kPlanFwdSegs = 0, kPlanBwdSegs = 1, kPlanFwdE = 2, kPlanBwdE = 3, kPlanHeader = 8;

// Fused scalar reduction (PRBlendFwdArgs.sync): the backward's workgroups arrive on counters
// sharded by blockIdx % 8 (one word saturates near 90 atomics / us; the last generation of a
// grid arrives together), the last arrival of each class on a top counter; the last workgroup
// overall reads every partial (release / acquire fences around the arrivals) and forms d sigma,
// d gamma, d alpha -- the work of blend_finalize_kernel, one kernel boundary fewer.  It then
// zeroes the counters (a second backward of the same forward); pr_blend_fwd zeroes them first.
constexpr int kSyncStride = 16, kSyncTop = 8 * kSyncStride;

PR_DEV void sync_zero(int32_t* sync) {
  if (threadIdx.x < 9) sync[threadIdx.x == 8 ? kSyncTop : threadIdx.x * kSyncStride] = 0;
}

// A partial of the fused reduction is written by a device-scope atomic exchange whose old value
// the writer waits for: the exchange is then performed at the device's coherence point, before
// the workgroup's arrival.  So no workgroup needs a release fence (an L2 writeback of its XCD: the
// round-4 fused variant with __threadfence per workgroup took blend_bwd from 75 to 182 us), and
// only the last arrival invalidates its L2 before reading every partial.
template <class Args>
PR_DEV void put_partial(const Args& a, float* dst, float v) {
  if (a.sync) {
    const float old = __hip_atomic_exchange(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::"v"(old));  // wait for the exchange's return: it has been performed
  } else {
    *dst = v;
  }
}

// Ordering (DESIGN.md §4 "Fused scalar reduction").  Default (rel = 0): relaxed arrivals.  The
// HIP / LLVM memory model gives no happens-before edge from a partial to the last workgroup here;
// what orders them is gfx950's: a device-scope RMW is performed at the device coherence point and
// returns its old value only after that, the writer issues its arrival only after every partial
// exchange of its workgroup has returned (s_waitcnt + the barrier), so each partial is in the
// coherent memory before the arrival that counts it, and the last workgroup reads the partials
// with device-scope (sc1) loads that bypass its XCD's L2.  rel = 1 (PR_BLEND_SYNC_ORDER=release)
// is the model-conforming form: both arrivals acq_rel (a release per workgroup: its L2
// writeback), the last workgroup's acquire synchronising with every earlier arrival through the
// counters' release sequences.  Both give the same bits (tests/test_gpu_fused_finalize.py).
PR_DEV bool last_arrival(int32_t* sync, int nblk, int* flag, bool rel) {
  __syncthreads();  // this workgroup's partial exchanges have returned
  if (threadIdx.x == 0) {
    const int r = (int)(blockIdx.x % 8), n_r = (nblk - r + 7) / 8;
    int last = 0;
    if (rel) {
      if (__hip_atomic_fetch_add(sync + r * kSyncStride, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == n_r - 1)
        last = __hip_atomic_fetch_add(sync + kSyncTop, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
               min(nblk, 8) - 1;
    } else if (atomicAdd(sync + r * kSyncStride, 1) == n_r - 1) {
      last = atomicAdd(sync + kSyncTop, 1) == min(nblk, 8) - 1;
    }
    *flag = last;
  }
  __syncthreads();
  const bool last = uni(*flag) != 0;
  if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop stale partial lines of this L2
  return last;
}

// pixel block of this workgroup: centre-out within each image when blocks tile images
PR_DEV int64_t pixel_block(const Geo& g) {
  if (g.bpi == 0) return blockIdx.x;
  const int64_t n = blockIdx.x / g.bpi;
  return n * g.bpi + centre_out((int)(blockIdx.x - n * g.bpi), g.bpi);
}

// Pixel j of pixel block blk.  Consecutive (pm = 0): blk * PB + j.  Interleaved (pm = 1, blocks
// tiling images): within its image, block b takes pixel t = j * NBI + b (NBI = HW / PB blocks per
// image: one pixel from each NBI-pixel band), its column rotated by j * A when the bands are whole
// rows, so every block samples the whole frame and holds about the mean number of valid slots
// instead of the heaviest blocks setting the span; a bijection within each image.  Every global
// access and every Philox counter uses this physical index, so the outputs are those of the
// consecutive blocks (the scalar gradients' per-block partial sums regroup).
PR_DEV int block_pixel(const Geo& g, int64_t blk, int j) {
  if (!g.pm) return (int)(blk * g.PB + j);
  const int n = (int)(blk / g.pmNBI), b = (int)(blk - (int64_t)n * g.pmNBI);
  int t = j * g.pmNBI + b;
  if (g.pmA) {
    const int row = t / g.pmW;
    int col = t - row * g.pmW + (int)(((int64_t)j * g.pmA) % g.pmW);
    if (col >= g.pmW) col -= g.pmW;
    t = row * g.pmW + col;
  }
  return n * g.HW + t;
}

struct Sc {
  float sigma, gamma, alpha;
  uint64_t kr, ka;
};

PR_DEV Sc resolve(const PRBlendParams& p) {
  Sc s{p.sigma, p.gamma, p.alpha, p.seed_r, p.seed_a};
  if (p.scalars[0]) s.sigma = *p.scalars[0];
  if (p.scalars[1]) s.gamma = *p.scalars[1];
  if (p.scalars[2]) s.alpha = *p.scalars[2];
  if (p.seeds) {  // bit 63 marks an absolute key that ignores the device base (fixed noise)
    const uint64_t b = p.seeds[0];
    if (!(p.seed_r >> 63)) s.kr = mix64(b ^ p.seed_r);
    if (!(p.seed_a >> 63)) s.ka = mix64(b ^ p.seed_a);
  }
  return s;
}

PR_DEV bool slot_mask(const int64_t* p2f, const uint8_t* mask, int64_t gs) {
  return p2f ? (p2f[gs] >= 0) : (mask[gs] != 0);
}

// image index of block pixel pl (n0 / rem0 = image and offset of the block's first pixel)
PR_DEV int image_of(int n0, int rem0, int pl, int HW) {
  int r = rem0 + pl, n = n0;
  while (r >= HW) { r -= HW; ++n; }
  return n;
}

// znear / zfar of block pixel pl: the pass's first image's from registers (zf0 / zn0, loaded once
// per pass with a uniform address), another image's from memory (a block crossing an image edge:
// a branch no lane takes on single-frame batches).  The per-entry loads this replaces were a
// dependent global round trip in every slot iteration of 1a, B1 and B8.
PR_DEV void planes_of(const PRBlendParams& p, int n0, int rem0, int pl, int HW, float zf0, float zn0, float& zf,
                      float& zn) {
  const int n = image_of(n0, rem0, pl, HW);
  zf = zf0;
  zn = zn0;
  if (n != n0) {
    zf = p.zfar[n];
    zn = p.znear[n];
  }
}

// slot loop over [0, n) of a block with row length L: thread walks i = tid + 256*it,
// (pl, k) = divmod(i, L) maintained incrementally
#define PR_FOR_SLOTS(L, Q, R, NTOT)                                                      \
  for (int i_ = tid, pl = tid / (L), k = tid - (tid / (L)) * (L); i_ < (NTOT);          \
       i_ += kThreads, pl += (Q), k += (R), (k >= (L) ? (k -= (L), ++pl) : 0))

// Batched walks: kU items per thread per batch, so a batch's global loads are all in
// flight before the first is consumed (the slot phases are latency-bound: one HBM round
// trip per dependent iteration).
constexpr int kU = 4;
struct Batch {
  int pl[kU], k[kU];
  bool ok[kU];
};

// Entry walks of a pass: entry i belongs to pixel OWN[i] (the owner map, filled per pass
// by fill_owner) and is that pixel's entry i - (ea[pl] - eb): no search per item.
PR_DEV void entry_batch(Batch& b, int i0, int n, const uint8_t* OWN, const int* ea, int eb) {
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int i = i0 + u * kThreads;
    b.ok[u] = i < n;
    const int pl = b.ok[u] ? OWN[i] : 0;
    b.pl[u] = pl;
    b.k[u] = i - (ea[pl] - eb);
  }
}

// The pixel lanes (lpp per pixel) write their pixel's id over its entries (and zero the
// entries' win counts when CN is given).
PR_DEV void fill_owner(uint8_t* OWN, const int* ea, int eb, const int* cl, int npix, int lsh, int lpp,
                       int* CN = nullptr) {
  const int pl = threadIdx.x >> lsh, l = threadIdx.x & (lpp - 1);
  if (pl < npix) {
    const int e0 = ea[pl] - eb, c = cl[pl];
    for (int e = l; e <= c; e += lpp) {
      OWN[e0 + e] = (uint8_t)pl;
      if (CN) CN[e0 + e] = 0;
    }
  }
}

// Wave 0 (PB <= 32 pixels): per-pixel valid-prefix counts CP (clamped to [0, K]; K without
// pix_count), slot entries CL (CP when compact, else K), the exclusive prefix EA[0..npix] of
// the entries (CL + 1: the background entry), and the passes: maximal runs of consecutive
// pixels whose entries fit CAP records (CAP >= K + 1, so a pixel always fits), as starts
// PS[0..np) + end PS[np] = npix, with the pass count in PS[PB + 1].
PR_DEV int seg_parts(int tot, int E) { return tot > E ? (tot + E - 1) / E : 1; }

// A block's entries (valid slots + background) for the segment plan: the per-pixel count the
// scan below sums.
PR_DEV int pixel_entries(const int32_t* pcnt, int64_t gp, int K, bool compact) {
  return (compact ? min(max((int)pcnt[gp], 0), K) : K) + 1;
}

// E > 0: the passes are the block's entry-balanced segment parts instead (see below).
// GPX[0..npix): the block's physical pixels (block_pixel).
PR_DEV void block_entries(const Geo& g, int64_t blk, const int32_t* pcnt, int npix, int K, bool compact, int CAP,
                          int PB, int* CL, int* CP, int* EA, int* PS, int* GPX, int E = 0) {
  const int tid = threadIdx.x;
  const int gpv = tid < npix ? block_pixel(g, blk, tid) : 0;
  if (tid < npix) GPX[tid] = gpv;
  const int cp = tid < npix ? (pcnt ? min(max((int)pcnt[gpv], 0), K) : K) : 0;
  const int c = compact ? cp : K;
  const int v = tid < npix ? c + 1 : 0;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (tid >= o) x += y;
  }
  const int ex = x - v, tot = __shfl(x, 63);
  if (tid < npix) {
    CP[tid] = cp;
    CL[tid] = c;
    EA[tid] = ex;
  }
  if (tid == 0) {
    EA[npix] = tot;
    PS[0] = 0;
  }
  if (E > 0) {
    // entry-balanced parts (segment plan): n = ceil(tot / E) parts, pixel pl in part
    // floor(mid * n / tot) with mid its entries' midpoint.  The host keeps 2 (K+1) <= E <=
    // CAP - (K+1): a part spans tot / n >= (K+1) entries, so no part is empty, and holds at most
    // E + K + 1 <= CAP.  The plan kernel counts n from tot alone (seg_parts).
    const int n = seg_parts(tot, E);
    const int part = tid < npix ? min(n - 1, ((2 * ex + v) * n) / (2 * tot)) : n;
    for (int j = 1; j < n; ++j) {
      const int start = __popcll(__ballot(part < j));
      if (tid == 0) PS[j] = start;
    }
    if (tid == 0) {
      PS[n] = npix;
      PS[PB + 1] = n;
    }
    return;
  }
  // greedy passes, uniform over the wave (every value broadcast by shuffles); one pass
  // when everything fits
  int np = 0, est = 0;
  for (int pl = tot > CAP ? 1 : npix; pl < npix; ++pl) {
    const int end = pl + 1 < npix ? __shfl(ex, pl + 1) : tot;  // EA[pl + 1]
    if (end - est > CAP) {
      ++np;
      est = __shfl(ex, pl);
      if (tid == 0) PS[np] = pl;
    }
  }
  if (tid == 0) {
    PS[np + 1] = npix;
    PS[PB + 1] = np + 1;
  }
}

// The block's threads store v over the n floats at dst (float4 stores when dst is 16-B aligned).
PR_DEV void block_fill(float* dst, int64_t n, float v) {
  const int tid = threadIdx.x;
  int64_t head = ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) ? 0 : n;  // unaligned: scalar
  const int64_t n4 = (n - head) >> 2;
  const float4 v4 = make_float4(v, v, v, v);
  for (int64_t i = tid; i < n4; i += kThreads) reinterpret_cast<float4*>(dst)[i] = v4;
  for (int64_t i = 4 * n4 + tid; i < n; i += kThreads) dst[i] = v;
}

// Wave-wide append of the lanes with `want` to an LDS queue: one LDS atomic per wave,
// returns the lane's queue position (-1 if !want).
PR_DEV int wave_append(bool want, int* counter) {
  const uint64_t b = __ballot(want);
  if (b == 0) return -1;
  const int lane = __lane_id();
  const int leader = __ffsll((unsigned long long)b) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(b));
  base = __shfl(base, leader);
  return want ? base + __popcll(b & ((1ull << lane) - 1ull)) : -1;
}

// ---------------------------------------------------------------- rast noise
// Both noise modes evaluate smoothrast.py:32-33 literally, m_s = H(D + sigma*eps_s)
// with H(0)=1 and D = -dist; Philox mode draws eps_s by Box-Muller (4 per Philox
// block, gauss4) or, for ArctanRast, as Cauchy samples (cauchy4).  Box-Muller normals
// from 24-bit uniforms satisfy |eps| <= 5.7683, so with Gaussian noise a slot with
// |dist/sigma| > 5.8 has the same outcome for every sample: exact skip.
PR_DEV float pick4(const float e[4], uint32_t i) {
  return i == 0 ? e[0] : (i == 1 ? e[1] : (i == 2 ? e[2] : e[3]));
}

// -1: every sample inside, +1: every sample outside, 0: must draw (NaN included).
// dist * rcp(sigma) is within 2 ulp of dist / sigma, and the bound 5.8 sits above
// max |eps| = 5.7683 by far more than that, so the skip stays exact.
PR_DEV int rast_saturated(float dist, float sigma) {
  const float x = dist * __builtin_amdgcn_rcpf(sigma);
  return x < -kEpsMaxBM ? -1 : (x > kEpsMaxBM ? 1 : 0);
}

// Count of "inside" samples for one valid slot.
template <int NOISE>
PR_DEV int rast_count(const PRBlendParams& p, const Sc& sc, float dist, uint32_t gp, int k, int64_t gs,
                      int64_t PK) {
  int cnt = 0;
  const float D = -dist;
  if constexpr (NOISE == PR_NOISE_INJECTED) {
    for (int s = 0; s < p.Sr; ++s) cnt += (D + sc.sigma * p.noise_r[(int64_t)s * PK + gs]) >= 0.f ? 1 : 0;
  } else {
    const bool cauchy = p.flags & PR_BLEND_RAST_CAUCHY;
    if (!cauchy) {
      const int sat = rast_saturated(dist, sc.sigma);
      if (sat) return sat < 0 ? p.Sr : 0;
    }
    const uint32_t s0 = (uint32_t)p.sample_offset_r, s1 = s0 + (uint32_t)p.Sr;
    for (uint32_t g4 = s0 >> 2; 4u * g4 < s1; ++g4) {
      const U4 u = philox_block(sc.kr, gp, (uint32_t)k, g4, kTagRast);
      float e[4];
      if (cauchy) cauchy4(u, e); else gauss4(u, e);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 4u * g4 + (uint32_t)q;
        cnt += (sg >= s0 && sg < s1 && (D + sc.sigma * e[q]) >= 0.f) ? 1 : 0;
      }
    }
  }
  return cnt;
}

// Count and the score sum_s (base_s * score(eps_s)) / sigma with base = m_s - vr
// (smoothrast.py:46,49,53) or m_s (_wovr, :95,98), score = eps or 2 eps / (1 + eps^2).
template <int NOISE>
PR_DEV int rast_count_score(const PRBlendParams& p, const Sc& sc, float dist, uint32_t gp, int k, int64_t gs,
                            int64_t PK, float& gacc) {
  int cnt = 0;
  const float D = -dist;
  const float vr = heaviside1(D);
  gacc = 0.f;
  const bool cauchy = p.flags & PR_BLEND_RAST_CAUCHY, wovr = p.flags & PR_BLEND_RAST_WOVR;
  if constexpr (NOISE == PR_NOISE_INJECTED) {
    for (int s = 0; s < p.Sr; ++s) {
      const float e = p.noise_r[(int64_t)s * PK + gs];
      const float m = heaviside1(D + sc.sigma * e);
      cnt += (int)m;
      gacc += ((wovr ? m : m - vr) * noise_score(e, cauchy)) / sc.sigma;
    }
  } else {
    if (!cauchy && !wovr) {
      const int sat = rast_saturated(dist, sc.sigma);
      if (sat) return sat < 0 ? p.Sr : 0;  // m_s = vr for every sample: no score
    }
    // one Philox block per 4 samples, straight-line over the block; base_s is
    // b_in / b_out, the score sum is divided by sigma once at the end
    const float b_in = wovr ? 1.f : 1.f - vr, b_out = wovr ? 0.f : -vr;
    const uint32_t s0 = (uint32_t)p.sample_offset_r, s1 = s0 + (uint32_t)p.Sr;
    float acc = 0.f;
    for (uint32_t g4 = s0 >> 2; 4u * g4 < s1; ++g4) {
      const U4 u = philox_block(sc.kr, gp, (uint32_t)k, g4, kTagRast);
      float e[4];
      if (cauchy) cauchy4(u, e); else gauss4(u, e);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 4u * g4 + (uint32_t)q;
        if (sg < s0 || sg >= s1) continue;
        const bool in = (D + sc.sigma * e[q]) >= 0.f;
        cnt += in ? 1 : 0;
        acc = __builtin_fmaf(in ? b_in : b_out, noise_score(e[q], cauchy), acc);
      }
    }
    gacc = acc / sc.sigma;
  }
  return cnt;
}

// --------------------------------------------------------------- agg noise
// 4 consecutive samples [4g, 4g+4) of slot j of pixel gp.  Injected mode reads the
// caller's (Sa, P, K+1) tensor at local sample indices (sample offsets are 0 there).
template <int NOISE>
PR_DEV void agg_noise4(const PRBlendParams& p, const Sc& sc, uint32_t gp, int j, uint32_t g, int64_t P,
                       int KP1, float e[4]) {
  if constexpr (NOISE == PR_NOISE_INJECTED) {
    const int64_t PKa = P * KP1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = (int)(4 * g) + i;
      e[i] = s < p.Sa ? p.noise_a[(int64_t)s * PKa + (int64_t)gp * KP1 + j] : 0.f;
    }
  } else {
    const U4 u = philox_block(sc.ka, gp, (uint32_t)j, g, kTagAgg);
    if (p.flags & PR_BLEND_AGG_CAUCHY) {
      cauchy4(u, e);
    } else if (p.flags & PR_BLEND_AGG_UNIFORM) {  // U(-1/2, 1/2): u01 is odd/2^24, never 0 or 1
      e[0] = u01(u.x) - 0.5f; e[1] = u01(u.y) - 0.5f; e[2] = u01(u.z) - 0.5f; e[3] = u01(u.w) - 0.5f;
    } else {
      gauss4(u, e);
    }
  }
}

// Masked-tail noise of one agg sample (Philox Gaussian mode, backward only).  The m slots
// past a pixel's valid prefix have logit -inf: they never win, and their noise reaches the
// gradient only through S1 = sum_j eps_j (d z_max, B7) and S2 = sum_j eps_j^2 (d gamma).
// For m iid N(0,1) draws S1 = sqrt(m) Z and S2 = Z^2 + X with X ~ chi2(m-1) independent of
// Z (Cochran: sample mean and sum of squared deviations are independent), so the pair is
// drawn directly -- in distribution identical to m per-slot draws, at one Philox block per
// sample instead of m/4.  X = Z'^2 for m = 2, else 2 Gamma((m-1)/2) by Marsaglia-Tsang
// (ACM TOMS 26(3), 2000) squeeze + log test (acceptance >= 95 % for shape >= 1); a proposal
// rejected 8 times in a row (probability < 1e-10) keeps its last proposal.
PR_DEV void tail_pair(uint64_t key, uint32_t gp, uint32_t sg, int m, float& s1, float& s2) {
  U4 u = philox_block(key, gp, 0u, sg, kTagTail);
  float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(u.x)));
  const float z = rad * __builtin_amdgcn_cosf(u01(u.y));
  float x = rad * __builtin_amdgcn_sinf(u01(u.y));
  s1 = __builtin_amdgcn_sqrtf((float)m) * z;
  float c = 0.f;
  if (m == 2) {
    c = x * x;
  } else if (m >= 3) {
    const float d = 0.5f * (float)(m - 1) - (1.f / 3.f), cc = __builtin_amdgcn_rsqf(9.f * d);
    float uu = u01(u.z), v3 = 1.f;
    for (uint32_t t = 1;; ++t) {
      const float v = __builtin_fmaf(cc, x, 1.f);
      if (v > 0.f) {
        v3 = v * v * v;
        const float x2 = x * x;
        if (uu < 1.f - 0.0331f * (x2 * x2)) break;
        // natural logs on the hardware log2 (acceptance test only: 1 ulp moves the
        // boundary by < 1e-6 of the density)
        const float lu = __builtin_amdgcn_logf(uu) * 0.693147180559945f;
        const float lv = __builtin_amdgcn_logf(v3) * 0.693147180559945f;
        if (lu < __builtin_fmaf(0.5f, x2, d * ((1.f - v3) + lv))) break;
      }
      if (t == 8) break;
      u = philox_block(key, gp, t, sg, kTagTail);
      rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(u.x)));
      x = rad * __builtin_amdgcn_cosf(u01(u.y));
      uu = u01(u.z);
    }
    c = 2.f * d * v3;
  }
  s2 = __builtin_fmaf(z, z, c);
}

PR_DEV int agg_first_group(const PRBlendParams& p) { return p.sample_offset_a >> 2; }
PR_DEV int agg_num_groups(const PRBlendParams& p) {
  return ((p.sample_offset_a + p.Sa - 1) >> 2) - (p.sample_offset_a >> 2) + 1;
}

// Kernel arguments: the C ABI block plus, for PR_BLEND_PHONG (colour mode 3), a by-value copy of
// the shading inputs the host passed by pointer (PRBlend*Args.shade)
struct FwdK : PRBlendFwdArgs {
  PRShadeArgs sh;
};
struct BwdK : PRBlendBwdArgs {};

// image of slot gs (one-frame calls: 0 without a division)
template <typename A>
PR_DEV int slot_image(const A& a, int64_t gs) {
  return a.p.N == 1 ? 0 : (int)(gs / ((int64_t)a.p.H * a.p.W * a.p.K));
}

// the fragment slot gs as the shading sees it (face, image, barycentrics)
template <typename A>
PR_DEV Slot phong_slot(const A& a, int64_t gs, int64_t f) {
  Slot sl;
  sl.f = f;
  sl.n = slot_image(a, gs);
  sl.b[0] = a.bary[gs * 3]; sl.b[1] = a.bary[gs * 3 + 1]; sl.b[2] = a.bary[gs * 3 + 2];
  return sl;
}

// Colour of slot gs: texel tensor (CM 1, and CM 4: the backward of PR_BLEND_PHONG reading the
// forward's colours of the slots it needs), interpolated on demand from per-vertex colours (CM 2;
// the same operation order as interp_fwd_kernel, so the result is bit-identical to sampling the
// texels first), or Phong-shaded on demand (CM 3, forward: pr_phong.h's slot_terms, the operations
// of pr_shade_fwd, so bit-identical to shading the slots first).
template <int CM, typename A>
PR_DEV void slot_color(const A& a, int64_t gs, float c[3]) {
  if constexpr (CM == 3) {
    const int64_t f = a.pix_to_face[gs];
    if (f < 0) { c[0] = c[1] = c[2] = 0.f; return; }
    const Slot sl = phong_slot(a, gs, f);
    const Terms t = slot_terms(a.sh, sl, gs, a.sh.faces + f * 3);
    const V3 o = colour(t.lit, t.tex, t.spec);
    c[0] = o.x; c[1] = o.y; c[2] = o.z;
  } else if constexpr (CM == 2) {
    const int64_t f = a.pix_to_face[gs];
    if (f < 0) { c[0] = c[1] = c[2] = 0.f; return; }
    const float w0 = a.bary[gs * 3], w1 = a.bary[gs * 3 + 1], w2 = a.bary[gs * 3 + 2];
    const float* r0 = a.vert_colors + a.faces[f * 3] * 3;
    const float* r1 = a.vert_colors + a.faces[f * 3 + 1] * 3;
    const float* r2 = a.vert_colors + a.faces[f * 3 + 2] * 3;
#pragma unroll
    for (int d = 0; d < 3; ++d) c[d] = (w0 * r0[d] + w1 * r1[d]) + w2 * r2[d];
  } else {
    c[0] = a.colors[gs * 3]; c[1] = a.colors[gs * 3 + 1]; c[2] = a.colors[gs * 3 + 2];
  }
}


// ================================================================== forward
// CM: colour mode, 0 = weights out (no colour), 1 = texel colours, 2 = vertex colours
//
// LDS holds one record per ENTRY: a pixel's slot entries (its valid prefix with
// pix_count, else all K slots) followed by its background entry.  A workgroup owns PB
// pixels and walks them in passes of consecutive pixels whose entries fit the CAP
// records (one pass unless the block is unusually deep), so a block is sized by the
// fragments it really has, not by K.
// MULTI: the block may need several passes (CAP < PB * (K + 1)); without it the pass loop
// is a single straight-line pass (no loop-carried registers: 46 instead of 70 VGPRs).
// One pixel block (tile) of the forward: all of its passes (static grid), or only its segment
// part `part` of the entry-balanced plan (SEG).  rec: the profile record of this call.
template <int NOISE, bool RAST, int CM, bool MULTI, bool SEG>
PR_DEV void fwd_tile(const FwdK& a, const Geo& g, const int NC0, const Sc& sc, const int64_t blk,
                     const int part, const int64_t rec) {
  extern __shared__ float smem[];
  const PRBlendParams& p = a.p;
  const int K = g.K, KP1 = g.KP1, PB = g.PB, CAP = g.cap;
  float* A = smem;                 // [CAP] prob (the distance while queued), then int win counts
  float* B = A + CAP;              // [CAP] z_inv, then logits z
  float* PX = B + CAP;             // [PB][4] z_max, alpha, max logit, candidate count
  int* CL = reinterpret_cast<int*>(PX + PB * 4);            // [PB] slot entries (valid prefix or K)
  int* CP = CL + PB;                                        // [PB] valid-prefix count (K without pix_count)
  int* EA = CP + PB;                                        // [PB+1] exclusive prefix of entries (CL + 1)
  int* PS = EA + PB + 1;                                    // [PB+2] pass starts; [PB+1] = pass count
  int* GPX = PS + PB + 2;                                   // [PB] physical pixel (block_pixel)
  int* QN = GPX + PB;                                       // rast queue length
  uint16_t* Q = reinterpret_cast<uint16_t*>(QN + 4);        // [CAP] rast queue (pl << 8 | k)
  uint8_t* LC = reinterpret_cast<uint8_t*>(Q);              // [CAP] argmax candidates (after 1b)
  uint8_t* OWN = reinterpret_cast<uint8_t*>(Q + CAP);       // [CAP] pixel of each entry
  int* CNT = reinterpret_cast<int*>(A);
  int* PXI = reinterpret_cast<int*>(PX);
  const int tid = threadIdx.x;
  PR_BPROF_DECL;
  const int64_t bpix0 = blk * PB;
  const int bnpix = (int)min((int64_t)PB, g.P - bpix0);
  const int32_t* pcnt = a.pix_count;
  if (tid < 64) block_entries(g, blk, pcnt, bnpix, K, pcnt != nullptr, CAP, PB, CL, CP, EA, PS, GPX, SEG ? g.seg : 0);
  __syncthreads();
  const float gal = sc.gamma / sc.alpha;
  // ---- empty block (no pixel has a valid slot: only background entries): every sample's
  //      argmax is the background, W_bg = Sa / Sa = 1, alpha = 1 - (empty product) = 0; the
  //      same values the phases below would produce, without them
  if (pcnt && g.empty && uni(EA[bnpix]) == bnpix) {
    for (int i = tid; i < ((p.flags & PR_BLEND_WINNERS_IN) ? 0 : bnpix * p.Sa); i += kThreads) {
      const int pl = i / p.Sa;
      a.winners[(int64_t)GPX[pl] * p.Sa + (i - pl * p.Sa)] = (uint8_t)K;
    }
    if constexpr (CM != 0) {
      if (tid < bnpix) {
        const float wb = (float)p.Sa / (float)p.Sa;
        reinterpret_cast<float4*>(a.image)[GPX[tid]] =
            make_float4(0.f + wb * p.background[0], 0.f + wb * p.background[1], 0.f + wb * p.background[2], 1.f - 1.f);
      }
    } else {
      for (int i = tid; i < bnpix * KP1; i += kThreads) {
        const int pl = i / KP1, k = i - pl * KP1;
        a.weights[(int64_t)GPX[pl] * KP1 + k] = k == K ? (float)p.Sa / (float)p.Sa : 0.f / (float)p.Sa;
      }
    }
    __syncthreads();  // (SEG: the next segment rewrites this block's LDS)
    return;
  }

  const int npass = SEG ? 1 : (MULTI ? uni(PS[PB + 1]) : 1);
  for (int it = 0; it < npass; ++it) {
  const int pass = SEG ? part : it;
  const int ps = uni(PS[pass]), npix = uni(PS[pass + 1]) - ps;
  // lanes per pixel in the pixel phases and candidate stripes of the argmax: a segment of few
  // pixels spreads them over more lanes
  int lsh = g.lsh, NC = NC0;
  if constexpr (SEG) {
    while (lsh < g.lsh_max && (2 << lsh) * npix <= kThreads) ++lsh;
    const int ng = agg_num_groups(p);
    while (NC < 64 && npix * ng * NC * 2 <= kThreads && (KP1 + NC * 2 - 1) / (NC * 2) >= 4) NC <<= 1;
  }
  const int lpp = 1 << lsh;
  const int64_t pix0 = bpix0 + ps;  // logical: image / plane lookups (blocks keep to one image when interleaved)
  const int* cl = CL + ps;
  const int* cpv = CP + ps;
  const int* ea = EA + ps;
  const int* gpx = GPX + ps;
  const int eb = uni(ea[0]);
  const int n0 = (int)(pix0 / g.HW), rem0 = (int)(pix0 - (int64_t)n0 * g.HW);
  const float zf0 = p.zfar[n0], zn0 = p.znear[n0];
  if (tid == 0) *QN = 0;
  fill_owner(OWN, ea, eb, cl, npix, lsh, lpp);
  __syncthreads();
  PR_BSTAMP(0);

  // ---- 1a: slot entries, kU per thread in flight: mask, z_inv, and the probability
  //          wherever it needs no noise (masked, or saturated Gaussian); the rest is queued
  {
    // saturation shortcut of rast_count / rast_count_score (Philox Gaussian; the score
    // form also needs variance reduction)
    const bool sat_ok = NOISE == PR_NOISE_PHILOX && !(p.flags & PR_BLEND_RAST_CAUCHY) &&
                        !(a.rast_cache && (p.flags & PR_BLEND_RAST_WOVR));
    const int nit = uni(ea[npix]) - eb;  // entries of the pass (background entries skipped)
    for (int i0 = tid; i0 < nit; i0 += kU * kThreads) {
      Batch bt;
      entry_batch(bt, i0, nit, OWN, ea, eb);
#pragma unroll
      for (int u = 0; u < kU; ++u) bt.ok[u] = bt.ok[u] && bt.k[u] < cl[bt.pl[u]];
      bool mk[kU];
      float dd[kU], zb[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        mk[u] = false;
        dd[u] = zb[u] = 0.f;
        if (bt.ok[u]) {
          const int64_t gs = (int64_t)gpx[bt.pl[u]] * K + bt.k[u];
          // with valid-prefix counts nothing is read at a masked slot
          mk[u] = pcnt ? bt.k[u] < cpv[bt.pl[u]] : slot_mask(a.pix_to_face, a.mask, gs);
          if (mk[u] || !pcnt) {
            dd[u] = RAST ? a.dists[gs] : a.prob[gs];
            zb[u] = a.zbuf[gs];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int pl = bt.pl[u], k = bt.k[u], li = i0 + u * kThreads;  // entry index
        bool want = false;
        if (bt.ok[u]) {
          const int64_t gs = (int64_t)gpx[pl] * K + k;
          const bool m = mk[u];
          float zf, zn;
          planes_of(p, n0, rem0, pl, g.HW, zf0, zn0, zf, zn);
          B[li] = ((zf - zb[u]) / (zf - zn)) * (m ? 1.f : 0.f);
          if constexpr (RAST) {
            const int sat = m && sat_ok ? rast_saturated(dd[u], sc.sigma) : 0;
            want = m && sat == 0;
            if (want) {
              A[li] = dd[u];  // the distance, for 1b
            } else {          // count Sr (saturated inside) or 0: prob Sr/Sr * 1 = 1, or 0
              const float prob = sat < 0 ? 1.f : 0.f;
              A[li] = prob;
              // (with pix_count the cache is defined at valid slots only: the backward reads no more)
              if (a.rast_cache && (m || !pcnt)) reinterpret_cast<float2*>(a.rast_cache)[gs] = make_float2(prob, 0.f);
            }
          } else {
            A[li] = dd[u];
          }
        }
        if constexpr (RAST) {
          const int pos = wave_append(want, QN);
          if (want) Q[pos] = (uint16_t)((pl << 8) | k);
        }
      }
    }
  }
  __syncthreads();
  PR_BSTAMP(1);

  // ---- 1b: queued slots (valid, unsaturated): Monte-Carlo rasterization, all lanes busy
  if constexpr (RAST) {
    const int nq = *QN;
    for (int i = tid; i < nq; i += kThreads) {
      const int e = Q[i], pl = e >> 8, k = e & 255, li = ea[pl] - eb + k;
      const int64_t gp = gpx[pl], gs = gp * K + k;
      const float dist = A[li];
      float prob;
      if (a.rast_cache) {  // also keep the score mean for the backward (same arithmetic as its B1)
        float gacc;
        const int cnt = rast_count_score<NOISE>(p, sc, dist, (uint32_t)gp, k, gs, g.PK, gacc);
        prob = ((float)cnt / (float)p.Sr) * 1.f;
        reinterpret_cast<float2*>(a.rast_cache)[gs] = make_float2(prob, gacc / (float)p.Sr);
      } else {
        prob = ((float)rast_count<NOISE>(p, sc, dist, (uint32_t)gp, k, gs, g.PK) / (float)p.Sr) * 1.f;
      }
      A[li] = prob;
    }
    __syncthreads();
  }
  PR_BSTAMP(2);

  // ---- 2: per pixel (lpp lanes): alpha, z_max, logits, largest logit, and the list of
  //         argmax candidates (ascending j).  A pixel's entries are its cl slot entries,
  //         then the background (entry cl -> j = K); lanes take contiguous chunks
  {
    const int pl = tid >> lsh, l = tid & (lpp - 1);
    const bool act = pl < npix;
    const int c = act ? cl[pl] : 0, e0 = act ? ea[pl] - eb : 0, ckp = (c + lpp) >> lsh;  // ceil((c+1)/lpp)
    const int j0 = l * ckp, j1 = min(c + 1, j0 + ckp), k1 = min(c, j1);
    float al = 1.f, zm = kNegInf;
    if (act)
      for (int k = j0; k < k1; ++k) {
        al *= (1.f - A[e0 + k]);
        zm = fmaxf(zm, B[e0 + k]);
      }
    for (int m = 1; m < lpp; m <<= 1) {
      al *= __shfl_xor(al, m);
      zm = fmaxf(zm, __shfl_xor(zm, m));
    }
    if (c < K) zm = fmaxf(zm, 0.f);  // slots past the walked ones: z_inv 0, in the reference's max
    const float zmax = zm < p.eps ? p.eps : zm;
    float zl = kNegInf;
    if (act)
      for (int e = j0; e < j1; ++e) {
        const float z = e < c ? gal * logf(A[e0 + e]) + B[e0 + e] - zmax : p.eps - zmax;
        B[e0 + e] = z;
        CNT[e0 + e] = 0;
        zl = fmaxf(zl, z);
      }
    for (int m = 1; m < lpp; m <<= 1) zl = fmaxf(zl, __shfl_xor(zl, m));
    // candidates: finite logits not below zl - skipm (bounded Box-Muller noise only: a
    // logit further below the best can never win); lane chunks are contiguous, so an
    // exclusive scan of the lane counts gives each lane its output offset
    // (uniform noise: |eps| < 1/2, so a logit gamma below the best never wins)
    const float skipm = NOISE != PR_NOISE_PHILOX || (p.flags & PR_BLEND_AGG_CAUCHY) ? __builtin_inff()
                        : (p.flags & PR_BLEND_AGG_UNIFORM) ? sc.gamma : 2.f * kEpsMaxBM * sc.gamma;
    const float zfloor = zl - skipm;
    int nc = 0;
    if (act)
      for (int e = j0; e < j1; ++e) {
        const float z = B[e0 + e];
        nc += (z > kNegInf && z >= zfloor) ? 1 : 0;
      }
    int inc = nc;  // inclusive scan of the lane counts within the pixel's lanes
    for (int o = 1; o < lpp; o <<= 1) {
      const int y = __shfl_up(inc, o, lpp);
      if (l >= o) inc += y;
    }
    int off = inc - nc;
    const int tot = __shfl(inc, lpp - 1, lpp);
    if (act)
      for (int e = j0; e < j1; ++e) {
        const float z = B[e0 + e];
        if (z > kNegInf && z >= zfloor) LC[e0 + off++] = (uint8_t)(e < c ? e : K);
      }
    if (act && l == 0) {
      PX[pl * 4 + 0] = zmax;
      PX[pl * 4 + 1] = al;
      PX[pl * 4 + 2] = zl;
      PXI[pl * 4 + 3] = tot;
    }
  }
  __syncthreads();
  PR_BSTAMP(3);

  // ---- 3: Monte-Carlo argmax: thread = (pixel, 4-sample group, candidate stripe c::NC);
  //         PR_BLEND_WINNERS_IN: the given winners of every sample counted instead
  if (p.flags & PR_BLEND_WINNERS_IN) {
    PR_FOR_SLOTS(p.Sa, g.qS, g.rS, npix * p.Sa) {
      const int w = a.winners[(int64_t)gpx[pl] * p.Sa + k];
      atomicAdd(&CNT[ea[pl] - eb + (w == K ? cl[pl] : w)], 1);
    }
  } else {
    const int ng = agg_num_groups(p), g0 = agg_first_group(p);
    const int npairs = npix * ng * NC;
    for (int base = 0; base < npairs; base += kThreads) {
      const int t = base + tid;
      const bool act = t < npairs;
      const int c = t & (NC - 1), pg = t / NC;
      const int pl = act ? pg / ng : 0, gi = act ? pg - pl * ng : 0;
      const uint32_t gg = (uint32_t)(NOISE == PR_NOISE_INJECTED ? gi : g0 + gi);
      const int64_t gp = act ? gpx[pl] : 0;
      const int e0 = ea[pl] - eb, cpl = cl[pl];
      float best[4] = {kNegInf, kNegInf, kNegInf, kNegInf};
      int bidx[4] = {-1, -1, -1, -1};
      if (act) {
        const int len = PXI[pl * 4 + 3];
        for (int i = c; i < len; i += NC) {  // ascending j within the thread
          const int j = LC[e0 + i];
          const float z = B[e0 + (j == K ? cpl : j)];
          float e[4];
          agg_noise4<NOISE>(p, sc, (uint32_t)gp, j, gg, g.P, KP1, e);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = z + sc.gamma * e[q];
            if (v > best[q]) { best[q] = v; bidx[q] = j; }
          }
        }
      }
      for (int m = 1; m < NC; m <<= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float ob = __shfl_xor(best[q], m);
          const int oi = __shfl_xor(bidx[q], m);
          if (oi >= 0 && (bidx[q] < 0 || ob > best[q] || (ob == best[q] && oi < bidx[q]))) {
            best[q] = ob; bidx[q] = oi;
          }
        }
      }
      if (act && c == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int s = (int)(4 * gg) + q - (NOISE == PR_NOISE_INJECTED ? 0 : p.sample_offset_a);
          if (s < 0 || s >= p.Sa) continue;
          const int w = bidx[q] < 0 ? K : bidx[q];
          a.winners[gp * p.Sa + s] = (uint8_t)w;
          atomicAdd(&CNT[e0 + (w == K ? cpl : w)], 1);
        }
      }
    }
  }
  __syncthreads();
  PR_BSTAMP(4);

  // ---- 4: outputs
  const float fSa = (float)p.Sa;
  if constexpr (CM != 0) {
    // the pixel's lanes sweep its slot entries; only slots that won a sample are read
    const int pl = tid >> lsh, l = tid & (lpp - 1);
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
    if (pl < npix) {
      const int e0 = ea[pl] - eb;
      for (int k = l; k < cl[pl]; k += lpp) {
        const int cw = CNT[e0 + k];
        if (cw == 0) continue;
        const float w = (float)cw / fSa;
        float c[3];
        slot_color<CM>(a, (int64_t)gpx[pl] * K + k, c);
        if constexpr (CM == 3) {  // the backward's colour of this winner (PR_BLEND_COLOR_SPARSE)
          if (a.colors) {
            float* o = const_cast<float*>(a.colors) + ((int64_t)gpx[pl] * K + k) * 3;  // (an output here)
            o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
          }
        }
        acc0 += w * c[0];
        acc1 += w * c[1];
        acc2 += w * c[2];
      }
    }
    for (int m = 1; m < lpp; m <<= 1) {
      acc0 += __shfl_xor(acc0, m);
      acc1 += __shfl_xor(acc1, m);
      acc2 += __shfl_xor(acc2, m);
    }
    if constexpr (CM == 3) {
      // and the colour of the unperturbed argmax j0 (the backward's baseline slot): the first entry
      // holding the largest logit (phase 2's zl; background last, so a slot wins a tie), found
      // among the ascending candidates; shaded here unless it won a sample above
      if (a.colors && pl < npix && l == 0) {
        const int e0 = ea[pl] - eb, c = cl[pl], tot = PXI[pl * 4 + 3];
        const float zl = PX[pl * 4 + 2];
        int j0 = K;
        for (int i = 0; i < tot; ++i) {
          const int j = LC[e0 + i];
          if (B[e0 + (j == K ? c : j)] == zl) { j0 = j; break; }
        }
        if (j0 < K && CNT[e0 + j0] == 0) {
          float c3[3];
          slot_color<CM>(a, (int64_t)gpx[pl] * K + j0, c3);
          float* o = const_cast<float*>(a.colors) + ((int64_t)gpx[pl] * K + j0) * 3;
          o[0] = c3[0]; o[1] = c3[1]; o[2] = c3[2];
        }
      }
    }
    if (pl < npix && l == 0) {
      const float wb = (float)CNT[ea[pl] - eb + cl[pl]] / fSa;
      float4 o;
      o.x = acc0 + wb * p.background[0];
      o.y = acc1 + wb * p.background[1];
      o.z = acc2 + wb * p.background[2];
      o.w = 1.f - PX[pl * 4 + 1];
      reinterpret_cast<float4*>(a.image)[gpx[pl]] = o;
    }
  } else {
    PR_FOR_SLOTS(KP1, g.qK1, g.rK1, npix * KP1) {  // dense K+1 weights: 0 past the slot entries
      const int c = cl[pl];
      const int cw = (k < c || k == K) ? CNT[ea[pl] - eb + (k == K ? c : k)] : 0;
      a.weights[(int64_t)gpx[pl] * KP1 + k] = (float)cw / fSa;
    }
  }
  __syncthreads();  // the next pass reuses every LDS record
  PR_BSTAMP(5);
  }  // passes
#ifdef PR_BLEND_PROFILE
  PR_BPROF_DUMP(0, rec);
#endif
}

// Static grid: workgroup = pixel block.  SEG: workgroup b runs segment b of the plan (the grid is
// the plan's bound on the segment count; workgroups past the plan's count exit at once).
template <int NOISE, bool RAST, int CM, bool MULTI, bool SEG>
__global__ void __launch_bounds__(kThreads, PR_BLEND_FWD_WPE) blend_fwd_kernel(FwdK a, Geo g, int NC) {
  if (a.sync && blockIdx.x == 0) sync_zero(a.sync);  // for the backward's fused reduction
  if constexpr (CM == 3) {  // the shading backward's small accumulators (a PR_GRAD_PREZEROED pr_shade_bwd)
    const PRShadeArgs& sh = a.sh;
    const int64_t t0 = (int64_t)blockIdx.x * kThreads + threadIdx.x, st = (int64_t)gridDim.x * kThreads;
    float* vb[3] = {sh.grad_verts, sh.grad_normals, sh.texture == PR_TEX_VERTEX ? sh.grad_vert_colors : nullptr};
    for (int j = 0; j < 3; ++j)
      if (vb[j])
        for (int64_t i = t0; i < sh.V * 3; i += st) vb[j][i] = 0.f;
    float* nb[2] = {sh.grad_light, sh.grad_camera};
    for (int j = 0; j < 2; ++j)
      if (nb[j])
        for (int64_t i = t0; i < (int64_t)a.p.N * 3; i += st) nb[j][i] = 0.f;
  }
  if constexpr (!SEG) {
    fwd_tile<NOISE, RAST, CM, MULTI, false>(a, g, NC, resolve(a.p), pixel_block(g), -1, blockIdx.x);
  } else {
    const int32_t* plan = a.plan;
    const int si = blockIdx.x;
    if (si >= uni(plan[kPlanFwdSegs])) return;
    const uint32_t code = reinterpret_cast<const uint32_t*>(plan + g.plan_fwd_list)[si];
    g.seg = uni(plan[kPlanFwdE]);
    fwd_tile<NOISE, RAST, CM, false, true>(a, g, NC, resolve(a.p), (int64_t)(code >> 6), (int)(code & 63), si);
  }
}

// ================================================================= backward
#ifndef PR_BLEND_B2R  // B2's per-lane entry chunk held in registers (0: always walk LDS)
#define PR_BLEND_B2R 8
#endif
constexpr int kB2R = PR_BLEND_B2R > 0 ? PR_BLEND_B2R : 1;
// Same entry layout and passes as the forward.  Entries are compacted (a pixel's valid
// slots + background) when the masked tail is drawn jointly (B6); otherwise every slot
// keeps its entry, since injected / Cauchy noise needs each masked slot's own d z.
// (MULTI: at least 6 waves per SIMD, the occupancy its 24 KB of LDS allows anyway)
//
// One pixel block of the backward: all passes (static grid) or segment part `part` (SEG); its
// scalar partials go to partials[4 pidx .. 4 pidx + 4).
template <int NOISE, bool RAST, int CM, bool MULTI, bool SEG>
PR_DEV void bwd_tile(const BwdK& a, const Geo& g, const Sc& sc, float* partials, const int64_t blk,
                     const int part, const int64_t pidx) {
  extern __shared__ float smem[];
  const PRBlendParams& p = a.p;
  const int K = g.K, KP1 = g.KP1, PB = g.PB, CAP = g.cap;
  const int Sa = p.Sa;
  float* PR = smem;                    // [CAP] prob
  float* ZZ = PR + CAP;                // [CAP] z_inv -> dL/dz
  float* GM = ZZ + CAP;                // [CAP] rast score mean (gmaps)
  float* EX = GM + CAP;                // [CAP] exclusive products of (1 - prob)
  float* DW = EX + CAP;                // [CAP] dL/dW
  int* CN = reinterpret_cast<int*>(DW + CAP);           // [CAP] win counts
  float* AS = reinterpret_cast<float*>(CN + CAP);       // [PB][Sa] a_s, then the tail terms (B6b)
  float* PX = AS + PB * Sa;            // [PB][12] per-pixel scalars; [8..12) the upstream image gradient
  int* CL = reinterpret_cast<int*>(PX + PB * 12);       // [PB] slot entries (valid prefix or K)
  int* CP = CL + PB;                   // [PB] valid-prefix count (K without pix_count)
  int* EA = CP + PB;                   // [PB+1] exclusive prefix of entries (CL + 1)
  int* PS = EA + PB + 1;               // [PB+2] pass starts; [PB+1] = pass count
  int* GPX = PS + PB + 2;              // [PB] physical pixel (block_pixel)
  uint8_t* OWN = reinterpret_cast<uint8_t*>(GPX + PB);  // [CAP] pixel of each entry
  uint8_t* WN = OWN + CAP;             // [PB][Sa] the forward's winners of the pass
  const int tid = threadIdx.x;
  PR_BPROF_DECL;
  const int64_t bpix0 = blk * PB;
  const int bnpix = (int)min((int64_t)PB, g.P - bpix0);
  const int32_t* pcnt = a.pix_count;
  const int ng = agg_num_groups(p), g0 = agg_first_group(p);
  const bool agg_cauchy = p.flags & PR_BLEND_AGG_CAUCHY;
  // B6 draws the masked tail jointly (tail_pair) in Philox Gaussian mode when the valid
  // prefix is known; injected noise (parity) and Cauchy noise keep one row per slot
  const bool tail = NOISE == PR_NOISE_PHILOX && !agg_cauchy && pcnt != nullptr && g.tail;
  if (tid < 64) block_entries(g, blk, pcnt, bnpix, K, tail, CAP, PB, CL, CP, EA, PS, GPX, SEG ? g.seg : 0);
  __syncthreads();
  const float gal = sc.gamma / sc.alpha;
  float part_sigma = 0.f, part_q = 0.f, part_a = 0.f, part_gal = 0.f;
  // ---- empty block (compacted entries, no pixel with a valid slot): the background wins every
  //      sample and is also the unperturbed argmax, so with the baseline every a_s = 0: no d z,
  //      no scalar partials; masked slots get zero d zbuf / d dists / d colour (the values B8m
  //      writes).  Without the baseline (GaussianAgg_wovr) a_s = dW_bg and the full path runs.
  // PR_BLEND_LIVE_ONLY (RAST, counts): the masked slots' zero gradients are not written at all
  const bool live_only = RAST && pcnt != nullptr && (p.flags & PR_BLEND_LIVE_ONLY);
  if (RAST && tail && g.empty && !(p.flags & PR_BLEND_AGG_WOVR) && uni(EA[bnpix]) == bnpix) {
    if (live_only) {
    } else if (!g.pm) {
      const int64_t s0 = bpix0 * K, n = (int64_t)bnpix * K;
      block_fill(a.grad_zbuf + s0, n, 0.f);
      block_fill(a.grad_dists + s0, n, 0.f);
      if constexpr (CM == 1 || CM == 4) block_fill(a.grad_colors + 3 * s0, 3 * n, 0.f);
      if constexpr (CM == 2) block_fill(a.grad_bary + 3 * s0, 3 * n, 0.f);
    } else {  // interleaved: one K-slot row per pixel
      for (int i = tid; i < bnpix * K; i += kThreads) {
        const int pl = i / K;
        const int64_t s = (int64_t)GPX[pl] * K + (i - pl * K);
        a.grad_zbuf[s] = 0.f;
        a.grad_dists[s] = 0.f;
        if constexpr (CM == 1 || CM == 4) a.grad_colors[3 * s] = a.grad_colors[3 * s + 1] = a.grad_colors[3 * s + 2] = 0.f;
        if constexpr (CM == 2) a.grad_bary[3 * s] = a.grad_bary[3 * s + 1] = a.grad_bary[3 * s + 2] = 0.f;
      }
    }
    if (tid < 4) put_partial(a, partials + pidx * 4 + tid, 0.f);
    __syncthreads();  // (SEG: the next segment rewrites this block's LDS)
    return;
  }

  const int npass = SEG ? 1 : (MULTI ? uni(PS[PB + 1]) : 1);
  for (int it = 0; it < npass; ++it) {
  const int pass = SEG ? part : it;
  const int ps = uni(PS[pass]), npix = uni(PS[pass + 1]) - ps;
  int lsh = g.lsh;  // lanes per pixel: a segment of few pixels may spread them over more lanes
  if constexpr (SEG)
    while (lsh < g.lsh_max && (2 << lsh) * npix <= kThreads) ++lsh;
  const int lpp = 1 << lsh;
  const int64_t pix0 = bpix0 + ps;  // logical: image / plane lookups (blocks keep to one image when interleaved)
  const int* cl = CL + ps;
  const int* cpv = CP + ps;
  const int* ea = EA + ps;
  const int* gpx = GPX + ps;
  const int eb = uni(ea[0]), nent = uni(ea[npix]) - eb;
  const int n0 = (int)(pix0 / g.HW), rem0 = (int)(pix0 - (int64_t)n0 * g.HW);
  const float zf0 = p.zfar[n0], zn0 = p.znear[n0];
  fill_owner(OWN, ea, eb, cl, npix, lsh, lpp, CN);
  __syncthreads();
  PR_BSTAMP(0);

  // ---- B1: entries (slots + background): prob, z_inv, rast score, dL/dW (kU items per
  //          thread with their global loads in flight together)
  {
    for (int i0 = tid; i0 < nent; i0 += kU * kThreads) {
      Batch bt;
      entry_batch(bt, i0, nent, OWN, ea, eb);
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (bt.ok[u] && bt.k[u] == cl[bt.pl[u]]) bt.k[u] = K;  // the background entry
      bool mk[kU];
      float2 pg[kU];  // (prob, gm) from the cache / input prob, or (dist, -) to recount
      float zb[kU], dw[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        mk[u] = false;
        pg[u] = make_float2(0.f, 0.f);
        zb[u] = dw[u] = 0.f;
        if (!bt.ok[u]) continue;
        const int pl = bt.pl[u], k = bt.k[u];
        const int64_t gp = gpx[pl];
        if (k < K) {
          const int64_t gs = gp * K + k;
          // with valid-prefix counts nothing is read at a masked slot (prob, score, z_inv are 0)
          mk[u] = pcnt ? k < cpv[pl] : slot_mask(a.pix_to_face, a.mask, gs);
          if (!mk[u] && pcnt) continue;
          if constexpr (RAST) {
            if (a.rast_cache) pg[u] = reinterpret_cast<const float2*>(a.rast_cache)[gs];
            else pg[u].x = a.dists[gs];
          } else {
            pg[u].x = a.prob[gs];
          }
          zb[u] = a.zbuf[gs];
          if constexpr (CM == 1) {
            const float4 gi = reinterpret_cast<const float4*>(a.grad_image)[gp];
            const float* c = a.colors + gs * 3;
            dw[u] = (gi.x * c[0] + gi.y * c[1]) + gi.z * c[2];
          } else if constexpr (CM == 0) {  // (CM 2 / 4: dW of the slots B5 reads, B2)
            dw[u] = a.grad_weights[gp * KP1 + k];
          }
        } else {
          if constexpr (CM != 0) {  // the background entry also keeps the pixel's g_image for B8
            const float4 gi = reinterpret_cast<const float4*>(a.grad_image)[gp];
            dw[u] = (gi.x * p.background[0] + gi.y * p.background[1]) + gi.z * p.background[2];
            *reinterpret_cast<float4*>(PX + pl * 12 + 8) = gi;
          } else {
            dw[u] = a.grad_weights[gp * KP1 + K];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (!bt.ok[u]) continue;
        const int pl = bt.pl[u], k = bt.k[u], li = i0 + u * kThreads;  // entry index
        DW[li] = dw[u];
        if (k == K) continue;
        const bool m = mk[u];
        const float mf = m ? 1.f : 0.f;
        float prob = pg[u].x, gm = pg[u].y;
        if constexpr (RAST) {
          if (!a.rast_cache) {  // recount below (B1r): keep the distance and the mask
            prob = pg[u].x;
            gm = mf;
          }
        }
        float zf, zn;
        planes_of(p, n0, rem0, pl, g.HW, zf0, zn0, zf, zn);
        PR[li] = prob;
        ZZ[li] = ((zf - zb[u]) / (zf - zn)) * mf;
        GM[li] = gm;
      }
    }
    // B1r: without the forward's cache, the Monte-Carlo rasterization again (same arithmetic
    // as the forward's 1b); each thread revisits its own B1 entries, one at a time
    if constexpr (RAST) {
      if (!a.rast_cache) {
        for (int li = tid; li < nent; li += kThreads) {
          const int pl = OWN[li], k = li - (ea[pl] - eb);
          if (k >= cl[pl]) continue;
          float prob = 0.f, gm = 0.f;
          if (GM[li] != 0.f) {
            const int64_t gp = gpx[pl], gs = gp * K + k;
            float gacc;
            const int cnt = rast_count_score<NOISE>(p, sc, PR[li], (uint32_t)gp, k, gs, g.PK, gacc);
            prob = ((float)cnt / (float)p.Sr) * 1.f;
            gm = gacc / (float)p.Sr;
          }
          PR[li] = prob;
          GM[li] = gm;
        }
      }
    }
    // the pass's winners (one contiguous byte range) into LDS for B5, with their win counts
    // (CN zeroed with the owner map); kU loads in flight per thread
    const int nw = npix * Sa;
    for (int i0 = tid; i0 < nw; i0 += kU * kThreads) {
      int w[kU], wp[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = i0 + u * kThreads;
        wp[u] = i / Sa;  // (Sa: runtime divisor, once per winner)
        w[u] = i < nw ? a.winners[(int64_t)gpx[min(wp[u], npix - 1)] * Sa + (i - wp[u] * Sa)] : 0;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = i0 + u * kThreads;
        if (i >= nw) continue;
        WN[i] = (uint8_t)w[u];
        const int pl = wp[u];
        atomicAdd(&CN[ea[pl] - eb + (w[u] == K ? cl[pl] : w[u])], 1);
      }
    }
  }
  __syncthreads();
  PR_BSTAMP(1);

  // ---- B2: per pixel (lpp lanes, contiguous chunks of its entries: the cl slot entries,
  //          then the background as entry cl -> j = K): z_max + first argmax, exclusive
  //          products for the alpha gradient, logits, unperturbed argmax j0
  {
    const int pl = tid >> lsh, l = tid & (lpp - 1);
    const bool act = pl < npix;
    const int c = act ? cl[pl] : 0, e0 = act ? ea[pl] - eb : 0, ckp = (c + lpp) >> lsh;  // ceil((c+1)/lpp)
    const int j0c = l * ckp, j1c = min(c + 1, j0c + ckp), k1c = min(c, j1c);
    // chunks of at most kB2R entries (every pixel of the launch: K + 1 <= kB2R * lpp) are read
    // into registers once; the loops below then touch LDS only for their results (same
    // arithmetic, same order)
    const bool regs = !MULTI && g.KP1 <= kB2R * lpp;  // (the multi-pass template keeps its VGPR cap)
    float rpr[kB2R], rzz[kB2R];
    if (regs) {
#pragma unroll
      for (int u = 0; u < kB2R; ++u) {
        const int k = j0c + u;
        rpr[u] = act && k < k1c ? PR[e0 + k] : 0.f;
        rzz[u] = act && k < k1c ? ZZ[e0 + k] : 0.f;
      }
    }
    float zm = kNegInf, tp = 1.f;
    int km = 1 << 30;
    if (regs) {
#pragma unroll
      for (int u = 0; u < kB2R; ++u) {
        if (!(act && j0c + u < k1c)) break;
        if (rzz[u] > zm) { zm = rzz[u]; km = j0c + u; }
        tp *= (1.f - rpr[u]);
      }
    } else if (act) {
      for (int k = j0c; k < k1c; ++k) {
        const float zi = ZZ[e0 + k];
        if (zi > zm) { zm = zi; km = k; }
        tp *= (1.f - PR[e0 + k]);
      }
    }
    for (int m = 1; m < lpp; m <<= 1) {
      const float oz = __shfl_xor(zm, m);
      const int ok = __shfl_xor(km, m);
      if (oz > zm || (oz == zm && ok < km)) { zm = oz; km = ok; }
    }
    // slots past the slot entries hold z_inv = 0 in the reference's max; they follow every
    // walked slot, so a walked slot wins a tie
    if (c < K && 0.f > zm) { zm = 0.f; km = c; }
    if (km == (1 << 30)) km = 0;
    const float zmax = zm < p.eps ? p.eps : zm;
    if constexpr (CM != 0) {
      // exclusive products across the lane chunks (log-step scans up and down the
      // pixel's lanes), then within the chunk
      float inc = tp, sinc = tp;
      for (int o = 1; o < lpp; o <<= 1) {
        const float y = __shfl_up(inc, o, lpp), z = __shfl_down(sinc, o, lpp);
        if (l >= o) inc *= y;
        if (l + o < lpp) sinc *= z;
      }
      const float iu = __shfl_up(inc, 1, lpp), sd = __shfl_down(sinc, 1, lpp);
      float pre = l > 0 ? iu : 1.f, suf = l + 1 < lpp ? sd : 1.f;
      if (act && l == 0) PX[pl * 12 + 5] = tp * suf;  // prod (1 - prob): a masked slot's exclusive product
      if (regs) {
        float ex[kB2R];
#pragma unroll
        for (int u = kB2R - 1; u >= 0; --u) {
          ex[u] = suf;
          if (act && j0c + u < k1c) suf *= (1.f - rpr[u]);
        }
#pragma unroll
        for (int u = 0; u < kB2R; ++u) {
          if (!(act && j0c + u < k1c)) break;
          EX[e0 + j0c + u] = pre * ex[u];
          pre *= (1.f - rpr[u]);
        }
      } else if (act) {
        for (int k = k1c - 1; k >= j0c; --k) {
          EX[e0 + k] = suf;
          suf *= (1.f - PR[e0 + k]);
        }
        for (int k = j0c; k < k1c; ++k) {
          EX[e0 + k] = pre * EX[e0 + k];
          pre *= (1.f - PR[e0 + k]);
        }
      }
    }
    float zb = kNegInf;
    int jb = 1 << 30;
    if (regs) {
#pragma unroll
      for (int u = 0; u < kB2R; ++u) {
        const int e = j0c + u;
        if (!(act && e < j1c)) break;
        const int j = e < c ? e : K;
        const float z = j < K ? gal * logf(rpr[u]) + rzz[u] - zmax : p.eps - zmax;
        if (z > zb || jb == (1 << 30)) { zb = z; jb = j; }
      }
    } else if (act) {
      for (int e = j0c; e < j1c; ++e) {
        const int j = e < c ? e : K;
        const float z = j < K ? gal * logf(PR[e0 + e]) + ZZ[e0 + e] - zmax : p.eps - zmax;
        if (z > zb || jb == (1 << 30)) { zb = z; jb = j; }
      }
    }
    for (int m = 1; m < lpp; m <<= 1) {
      const float oz = __shfl_xor(zb, m);
      const int oj = __shfl_xor(jb, m);
      if (oj != (1 << 30) && (jb == (1 << 30) || oz > zb || (oz == zb && oj < jb))) { zb = oz; jb = oj; }
    }
    if (act && l == 0) {
      PX[pl * 12 + 0] = zm;          // raw max z_inv (clamp test)
      PX[pl * 12 + 2] = (float)km;   // its first index
      PX[pl * 12 + 3] = (float)jb;   // unperturbed argmax of the K+1 logits
    }
    if constexpr (CM >= 2) {
#ifdef PR_BLEND_PROF_SPLIT_B2  // diagnostic: B2's pixel part to slot 7, its colour gathers to slot 2
      PR_BSTAMP(7);
#endif
      // dW = g_rgb . colour of the slot entries B5 reads (a win, or j0): the colour is
      // interpolated from the vertex colours here (CM 2), or read from the forward's colours of
      // exactly those slots (CM 4: PR_BLEND_PHONG's sparse colours), once per such entry
      if (act) {
        const float* gi = PX + pl * 12 + 8;
        for (int e = l; e < c; e += lpp) {
          const int cnt = CN[e0 + e];
          if (cnt == 0 && e != jb) continue;
          float cc[3];
          slot_color<CM>(a, (int64_t)gpx[pl] * K + e, cc);
          DW[e0 + e] = (gi[0] * cc[0] + gi[1] * cc[1]) + gi[2] * cc[2];
        }
      }
    }
  }
  __syncthreads();
  PR_BSTAMP(2);


  // ---- B5: per (pixel, sample): a_s = dW[j*_s] - dW[j0] (win counts: B1, CM 2's dW: B2)
  PR_FOR_SLOTS(Sa, g.qS, g.rS, npix * Sa) {
    const int s = k;
    const int e0 = ea[pl] - eb, c = cl[pl];
    const int jw = WN[pl * Sa + s];
    const int j0 = (int)PX[pl * 12 + 3];
    const int ew = e0 + (jw == K ? c : jw), e0j = e0 + (j0 == K ? c : j0);
    // GaussianAgg_wovr: a_s = <g, w_s> (smoothagg.py:118); else <g, w_s - vr'>
    const bool nobase = (p.flags & PR_BLEND_AGG_WOVR) && !(p.flags & PR_BLEND_AGG_CAUCHY);
    const float as = nobase ? DW[ew] : DW[ew] - DW[e0j];
    AS[pl * Sa + s] = as;
    part_a += as;
  }
  __syncthreads();
  PR_BSTAMP(3);

  // ---- B6: dz_j = mean_s(a_s * score(eps_sj) / gamma) and sum_s a_s * eps_sj * score(eps_sj)
  //          (d gamma; score = eps for Gaussian noise, 2 eps / (1 + eps^2) for Cauchy)
  //   6a: one row per entry, over nch adjacent lanes (groups gi = c, c + nch, ...) merged with
  //       xor-shuffles;
  //   6b: with the tail draw, one item per (pixel, sample): the masked slots' joint draw,
  //       a_s * S2 into d gamma and a_s * S1 / gamma over a_s in AS (summed in B7).
  // The lane split nch depends on the launch only (the agg sample groups ng), never on the pass's
  // entry count, so a pixel's d z has the same summation order in whatever block it lands: the
  // interleaved and consecutive layouts give the same bits.  Below 8 groups (Sa <= 28) one lane
  // sums an entry's samples in order -- the oracle's sequential mean over s; from 8 groups up the
  // groups are split over 2..16 lanes (cfg 4's Sa = 64: 4), which the long per-entry RNG chains
  // need.  (Rounds 1-4 chose nch from the pass's entry count: light passes split more, so the two
  // layouts summed the same pixel differently -- VERDICT r4 weak 1.)
  {
    // the reference divides each sample's a_s * score by gamma (smoothagg.py:52); one
    // reciprocal here instead of an IEEE division per (slot, sample): within 1 ulp
    const float inv_gamma = 1.f / sc.gamma;
    int nch = 1;
    if (ng >= 8) {
      nch = 2;
      while (nch < 16 && 8 * nch <= ng) nch <<= 1;
    }
    const int lch = 31 - __builtin_clz(nch);
    for (int i0 = 0; i0 < nent * nch; i0 += kThreads) {  // uniform trip count (shuffles below)
      const int i = i0 + tid, row = i >> lch, c = i & (nch - 1);
      const bool live = row < nent;
      float dz = 0.f, q = 0.f;
      if (live) {
        const int pl = OWN[row];
        const int r = row - (ea[pl] - eb);
        const int j = r == cl[pl] ? K : r;
        const int64_t gp = gpx[pl];
        for (int gi = c; gi < ng; gi += nch) {
          const uint32_t gg = (uint32_t)(NOISE == PR_NOISE_INJECTED ? gi : g0 + gi);
          const int sbase = (int)(4 * gg) - (NOISE == PR_NOISE_INJECTED ? 0 : p.sample_offset_a);
          float av[4];
          bool any = false;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int s = sbase + u;
            av[u] = (s >= 0 && s < Sa) ? AS[pl * Sa + s] : 0.f;
            any |= av[u] != 0.f;
          }
          if (!any) continue;
          float e[4];
          agg_noise4<NOISE>(p, sc, (uint32_t)gp, j, gg, g.P, KP1, e);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (av[u] != 0.f) {
              const float scr = noise_score(e[u], agg_cauchy);
              dz += (av[u] * scr) * inv_gamma;
              q += av[u] * (e[u] * scr);
            }
          }
        }
      }
      for (int mm = 1; mm < nch; mm <<= 1) dz += __shfl_xor(dz, mm);
      if (live && c == 0) ZZ[row] = dz / (float)Sa;  // ZZ now holds dL/dz (entry = row)
      part_q += q;
    }
    if (tail) {
      __syncthreads();  // 6a has read every a_s: 6b overwrites them in place
      PR_FOR_SLOTS(Sa, g.qS, g.rS, npix * Sa) {
        const int s = k, m = K - cpv[pl];
        const float as = AS[pl * Sa + s];
        float t = 0.f;
        if (m > 0 && as != 0.f) {
          float s1, s2;
          tail_pair(sc.ka, (uint32_t)gpx[pl], (uint32_t)(p.sample_offset_a + s), m, s1, s2);
          t = (as * s1) * inv_gamma;
          part_q += as * s2;
        }
        AS[pl * Sa + s] = t;
      }
    }
  }
  __syncthreads();
  PR_BSTAMP(4);

  // ---- B7: d z_max = -sum_k dz_k - dz_K, passed only if max z_inv >= eps; with the tail
  //          draw the masked slots' sum is sum_s AS[s] / Sa
  {
    const int pl = tid >> lsh, l = tid & (lpp - 1);
    const bool act = pl < npix;
    const int c = act ? cl[pl] : 0, e0 = act ? ea[pl] - eb : 0, cks = (c + lpp - 1) >> lsh;
    const int j0c = l * cks, k1c = min(c, j0c + cks);
    const int nt = act && tail ? Sa : 0, ckt = (nt + lpp - 1) >> lsh;
    const int t0 = l * ckt, t1 = min(nt, t0 + ckt);
    float s = 0.f, st = 0.f;
    if (act) {
      for (int k = j0c; k < k1c; ++k) s += ZZ[e0 + k];
      for (int t = t0; t < t1; ++t) st += AS[pl * Sa + t];
    }
    for (int m = 1; m < lpp; m <<= 1) {
      s += __shfl_xor(s, m);
      st += __shfl_xor(st, m);
    }
    if (act && l == 0) {
      if (tail) s += st / (float)Sa;
      float dzm = -s - ZZ[e0 + c];
      dzm = dzm * (PX[pl * 12 + 0] >= p.eps ? 1.f : 0.f);
      PX[pl * 12 + 4] = dzm;
    }
  }
  __syncthreads();
  PR_BSTAMP(5);

  // ---- B8: per-slot gradients of the slot entries (LDS records and the pixel's g_image in
  //          LDS: one entry per iteration); with compacted entries the masked slots in B8m
  for (int li = tid; li < nent; li += kThreads) {
    const int pl = OWN[li], k = li - (ea[pl] - eb);
    if (k >= cl[pl]) continue;  // the background entry
    const int64_t gp = gpx[pl], gs = gp * K + k;
    int64_t fk = -1;
    bool m;
    if (pcnt) {  // the face id is read below, for the (few) slots that won a sample
      m = k < cpv[pl];
    } else if (a.pix_to_face) {
      fk = a.pix_to_face[gs];
      m = fk >= 0;
    } else {
      m = a.mask[gs] != 0;
    }
    const float mf = m ? 1.f : 0.f;
    const float dzk = ZZ[li];
    const float dzinv = dzk + (k == (int)PX[pl * 12 + 2] ? PX[pl * 12 + 4] : 0.f);
    float zf, zn;
    planes_of(p, n0, rem0, pl, g.HW, zf0, zn0, zf, zn);
    // gradient only: hardware reciprocal of (zfar - znear) instead of an IEEE division
    a.grad_zbuf[gs] = -((dzinv * mf) * __builtin_amdgcn_rcpf(zf - zn));
    const float prob = PR[li];
    // L and 1/prob feed only gradients (tolerance, not winners): hardware log2 / rcp
    // (prob = count / Sr: never denormal; log2(1) = 0 and rcp(0) = inf exactly)
    const float L = __builtin_amdgcn_logf(prob) * 0.693147180559945f;
    float dL = gal * dzk;
    if (dL != dL) dL = 0.f;
    const float lp = __builtin_isinf(L) ? 0.f : L * dzk;
    if (lp == lp) part_gal += lp;
    float r = __builtin_amdgcn_rcpf(prob);
    if (__builtin_isinf(r)) r = 0.f;
    float dprob = r * dL;
    float4 gi = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (CM != 0) gi = *reinterpret_cast<const float4*>(PX + pl * 12 + 8);
    if constexpr (CM != 0) dprob = -((-gi.w) * EX[li]) + dprob;
    if constexpr (RAST) {
      const float dD = GM[li] * (dprob * mf);
      a.grad_dists[gs] = -dD;
      part_sigma += dD;
    } else {
      a.grad_prob[gs] = dprob;
    }
    if constexpr (CM == 1 || CM == 4) {
      const float w = (float)CN[li] / (float)Sa;
      float* dc = a.grad_colors + gs * 3;
      dc[0] = w * gi.x;
      dc[1] = w * gi.y;
      dc[2] = w * gi.z;
    } else if constexpr (CM == 2) {
      // d colour = w * g_rgb, pushed through the interpolation (interp_bwd_kernel's order)
      const int cnt = CN[li];
      float gb[3] = {0.f, 0.f, 0.f};
      const int64_t f = (cnt != 0 && m) ? (pcnt ? a.pix_to_face[gs] : fk) : -1;
      if (f >= 0) {
        const float w = (float)cnt / (float)Sa;
        const float dc[3] = {w * gi.x, w * gi.y, w * gi.z};
        const int64_t v[3] = {a.faces[f * 3], a.faces[f * 3 + 1], a.faces[f * 3 + 2]};
        const float bw[3] = {a.bary[gs * 3], a.bary[gs * 3 + 1], a.bary[gs * 3 + 2]};
#pragma unroll
        for (int d = 0; d < 3; ++d) {
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            gb[i] += dc[d] * a.vert_colors[v[i] * 3 + d];
            if (a.grad_vert_colors && dc[d] != 0.f) atomicAdd(&a.grad_vert_colors[v[i] * 3 + d], bw[i] * dc[d]);
          }
        }
      }
      a.grad_bary[gs * 3] = gb[0];
      a.grad_bary[gs * 3 + 1] = gb[1];
      a.grad_bary[gs * 3 + 2] = gb[2];
    }
  }

  // ---- B8m: slots past the compacted entries: constant gradients, no LDS record read.
  //           d zbuf, d dists and d colour are 0 (mask factor 0, no wins); without dists
  //           d prob keeps the alpha term g_alpha * prod_j (1 - prob_j) (its dL term is 0:
  //           prob = 0 there).  One wave per pixel: its lanes store consecutive slots.
  if (tail && !live_only) {
    const int lane = tid & 63;
    for (int mpl = tid >> 6; mpl < npix; mpl += kThreads / 64) {
      const int64_t gp = gpx[mpl];
      float dprob = 0.f;
      if constexpr (!RAST && CM != 0) dprob = PX[mpl * 12 + 11] * PX[mpl * 12 + 5];
      for (int k = cl[mpl] + lane; k < K; k += 64) {
        const int64_t gs = gp * K + k;
        a.grad_zbuf[gs] = 0.f;
        if constexpr (RAST) a.grad_dists[gs] = 0.f;
        else a.grad_prob[gs] = dprob;
        if constexpr (CM == 1 || CM == 4) {
          float* dc = a.grad_colors + gs * 3;
          dc[0] = dc[1] = dc[2] = 0.f;
        } else if constexpr (CM == 2) {
          a.grad_bary[gs * 3] = a.grad_bary[gs * 3 + 1] = a.grad_bary[gs * 3 + 2] = 0.f;
        }
      }
    }
  }
  __syncthreads();  // the next pass reuses every LDS record
  PR_BSTAMP(6);
  }  // passes

  // ---- block reduction of the scalar partials (fixed order -> deterministic)
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    part_sigma += __shfl_xor(part_sigma, m);
    part_q += __shfl_xor(part_q, m);
    part_a += __shfl_xor(part_a, m);
    part_gal += __shfl_xor(part_gal, m);
  }
  float* RED = smem;  // all per-entry arrays are dead now
  if ((tid & 63) == 0) {
    RED[(tid >> 6) * 4 + 0] = part_sigma;
    RED[(tid >> 6) * 4 + 1] = part_q;
    RED[(tid >> 6) * 4 + 2] = part_a;
    RED[(tid >> 6) * 4 + 3] = part_gal;
  }
  __syncthreads();
  if (tid < 4) put_partial(a, partials + pidx * 4 + tid, (RED[tid] + RED[4 + tid]) + (RED[8 + tid] + RED[12 + tid]));
#ifdef PR_BLEND_PROFILE
  PR_BSTAMP(7);
  PR_BPROF_DUMP(1, pidx);
#endif
  __syncthreads();  // (SEG: the next segment rewrites RED)
}

// d sigma, d gamma, d alpha from the per-block partials, by one workgroup in a fixed order
// (deterministic): blocks b, b + 256, ... per thread (four blocks' loads in flight per step: the
// latency chain of one load per step cost ~6 us), then the waves' xor-shuffle sums, then the
// four waves in order.  red: 16 floats of LDS.  coherent (the fused reduction's last workgroup):
// device-scope loads, read at the coherence point the partials' exchanges were performed at.
PR_DEV float load_partial(const float* src, bool coherent) {
  return coherent ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *src;
}

PR_DEV void finalize_scalars(const float* partials, int nblk, const PRBlendParams& p, int has_rast, float* out,
                             float* red, bool coherent = false) {
  const int tid = threadIdx.x;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int b = tid;
  for (; b + 3 * kThreads < nblk; b += 4 * kThreads) {
    float v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = load_partial(partials + (int64_t)(b + u * kThreads) * 4 + c, coherent);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] += v[u][c];
  }
  for (; b < nblk; b += kThreads) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += load_partial(partials + (int64_t)b * 4 + c, coherent);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += __shfl_xor(acc[c], m);
  if ((tid & 63) == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c) red[(tid >> 6) * 4 + c] = acc[c];
  __syncthreads();
  if (tid == 0) {
    const Sc sc = resolve(p);
    float r[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = (red[c] + red[4 + c]) + (red[8 + c] + red[12 + c]);
    const float dsig = r[0], Q = r[1], As = r[2], dgal = r[3];
    // smoothagg.py:54-56,72 : mean_s sum a_s (|eps_s|^2 - 1) / gamma
    const float dg1 = ((Q - As) / sc.gamma) / (float)p.Sa;
    out[0] = has_rast ? dsig : 0.f;
    out[1] = dg1 + dgal / sc.alpha;                       // prod_corrected x = gamma/alpha
    out[2] = -dgal * ((sc.gamma / sc.alpha) / sc.alpha);
  }
}

template <int NOISE, bool RAST, int CM, bool MULTI, bool SEG>
__global__ void __launch_bounds__(kThreads, MULTI ? 6 : PR_BLEND_BWD_WPE) blend_bwd_kernel(BwdK a, Geo g, float* partials) {
  int nblk = (int)gridDim.x;
  if constexpr (!SEG) {
    const int64_t blk = pixel_block(g);
    bwd_tile<NOISE, RAST, CM, MULTI, false>(a, g, resolve(a.p), partials, blk, -1, blk);
  } else {
    const int32_t* plan = a.plan;
    const int si = blockIdx.x;
    nblk = uni(plan[kPlanBwdSegs]);
    if (si < nblk) {  // (workgroups past the plan's count still arrive below)
      const uint32_t code = reinterpret_cast<const uint32_t*>(plan + g.plan_bwd_list)[si];
      g.seg = uni(plan[kPlanBwdE]);
      bwd_tile<NOISE, RAST, CM, false, true>(a, g, resolve(a.p), partials, (int64_t)(code >> 6), (int)(code & 63), si);
    }
  }
  if (a.sync) {
    __shared__ float red[16];
    __shared__ int flag;
    if (last_arrival(a.sync, (int)gridDim.x, &flag, g.sync_rel != 0)) {
      finalize_scalars(partials, nblk, a.p, RAST ? 1 : 0, a.grad_scalars, red, true);
      sync_zero(a.sync);
    }
  }
}

// (plan: the backward ran the plan's segments; their count is read here)
__global__ void __launch_bounds__(kThreads) blend_finalize_kernel(const float* partials, int nblk,
                                                                  PRBlendParams p, int has_rast,
                                                                  float* out, int32_t* plan) {
  __shared__ float red[16];
  if (plan) nblk = uni(plan[kPlanBwdSegs]);
  finalize_scalars(partials, nblk, p, has_rast, out, red);
}

// ====================================================== segment plan
// (1) blend_plan_count_kernel, one thread per pixel: every pixel's entries from the valid-prefix
//     counts, summed over the forward's and the backward's pixel blocks (PB <= 32 adjacent lanes)
//     -> each block's entry total.  (2) blend_plan_list_kernel, one workgroup: per kernel, the
//     frame's total entries fix E (at least the host's target; raised so the segments fit the
//     grid bound T + X), every block's part count seg_parts(tot, E) -- the count block_entries
//     splits it into -- an exclusive scan of the part counts in dispatch order (the forward's
//     blocks centre-out on single frames, as its static grid) and the segment list.
constexpr int kPlanThreads = 1024;
constexpr int64_t kPlanMaxPixels = int64_t(1) << 18;
constexpr int kPlanMaxBlocks = (int)(kPlanMaxPixels / 16) + (int)(kPlanMaxPixels / 32);

struct PlanGeo {
  int P, K;
  int PB[2], E[2], lo[2], hi[2], X[2], bpi[2], T[2], list[2], compact[2];  // [0] forward, [1] backward
  int tots;  // int offset of the uint16 block totals ([T0] forward, then [T1] backward)
};

PR_DEV int block_of_rank(int r, int bpi) {
  if (bpi == 0) return r;
  const int n = r / bpi;
  return n * bpi + centre_out(r - n * bpi, bpi);
}

__global__ void __launch_bounds__(kThreads) blend_plan_count_kernel(const int32_t* pcnt, PlanGeo q, int32_t* plan) {
  const int gp = blockIdx.x * kThreads + threadIdx.x;
  const int c = gp < q.P ? pcnt[gp] : 0;
  uint16_t* tots = reinterpret_cast<uint16_t*>(plan + q.tots);
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    int e = gp < q.P ? (q.compact[w] ? min(max(c, 0), q.K) : q.K) + 1 : 0;
    for (int m = 1; m < q.PB[w]; m <<= 1) e += __shfl_xor(e, m);
    if (gp < q.P && (gp & (q.PB[w] - 1)) == 0) tots[(w ? q.T[0] : 0) + gp / q.PB[w]] = (uint16_t)e;
  }
}

__global__ void __launch_bounds__(kPlanThreads) blend_plan_list_kernel(PlanGeo q, int32_t* plan) {
  __shared__ uint16_t tl[kPlanMaxBlocks];
  __shared__ int wsum[kPlanThreads / 64];
  __shared__ int esh;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint16_t* tots = reinterpret_cast<const uint16_t*>(plan + q.tots);
  const int TT = q.T[0] + q.T[1];
  for (int i = tid; i < TT; i += kPlanThreads) tl[i] = tots[i];  // (loads independent: all in flight)
  __syncthreads();
  for (int w = 0; w < 2; ++w) {
    const int T = q.T[w], ch = (T + kPlanThreads - 1) / kPlanThreads;
    const uint16_t* tw = tl + (w ? q.T[0] : 0);
    const int r0 = min(T, tid * ch), r1 = min(T, r0 + ch);
    // the frame's entries -> E
    int tsum = 0;
    for (int r = r0; r < r1; ++r) tsum += tw[r];
    for (int o = 32; o >= 1; o >>= 1) tsum += __shfl_xor(tsum, o);
    if (lane == 0) wsum[wv] = tsum;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int i = 0; i < kPlanThreads / 64; ++i) tot += wsum[i];
      const int need = (tot + q.X[w] - 1) / q.X[w];  // parts <= T + tot / E <= T + X
      esh = min(max(q.E[w], max(need, q.lo[w])), q.hi[w]);
    }
    __syncthreads();
    const int E = esh;
    // part counts in dispatch order: chunk sums, block-wide exclusive scan, list
    int sum = 0;
    for (int r = r0; r < r1; ++r) sum += seg_parts(tw[block_of_rank(r, q.bpi[w])], E);
    int x = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    __syncthreads();  // wsum reuse
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int woff = 0, total = 0;
    for (int i = 0; i < kPlanThreads / 64; ++i) {
      const int v = wsum[i];
      woff += i < wv ? v : 0;
      total += v;
    }
    int off = woff + x - sum;
    uint32_t* list = reinterpret_cast<uint32_t*>(plan + q.list[w]);
    for (int r = r0; r < r1; ++r) {
      const int b = block_of_rank(r, q.bpi[w]), n = seg_parts(tw[b], E);
      for (int j = 0; j < n; ++j) list[off + j] = ((uint32_t)b << 6) | (uint32_t)j;
      off += n;
    }
    if (tid == 0) {
      plan[w ? kPlanBwdSegs : kPlanFwdSegs] = total;
      plan[w ? kPlanBwdE : kPlanFwdE] = E;
    }
    __syncthreads();  // wsum / esh reuse
  }
}

// ====================================================== standalone heaviside
PR_DEV PRBlendParams heaviside_params(const PRHeavisideArgs& a) {
  PRBlendParams p{};
  p.Sr = a.Sr; p.sample_offset_r = a.sample_offset_r; p.sigma = a.sigma;
  p.seed_r = a.seed_r; p.noise_r = a.noise_r;
  p.seeds = a.seeds;
  p.flags = a.flags & (PR_BLEND_RAST_CAUCHY | PR_BLEND_RAST_WOVR);
  if (a.sigma_dev) p.sigma = a.sigma_dev[0];
  return p;
}

template <int NOISE>
__global__ void __launch_bounds__(kThreads) heaviside_fwd_kernel(PRHeavisideArgs a) {
  const int64_t PK = (int64_t)a.N * a.H * a.W * a.K;
  const PRBlendParams p = heaviside_params(a);
  const Sc sc = resolve(p);
  for (int64_t gs = (int64_t)blockIdx.x * kThreads + threadIdx.x; gs < PK;
       gs += (int64_t)gridDim.x * kThreads) {
    const int64_t gp = gs / a.K;
    const int k = (int)(gs - gp * a.K);
    const int cnt = rast_count<NOISE>(p, sc, a.dists[gs], (uint32_t)gp, k, gs, PK);
    a.prob[gs] = (float)cnt / (float)a.Sr;
  }
}

template <int NOISE>
__global__ void __launch_bounds__(kThreads) heaviside_bwd_kernel(PRHeavisideArgs a, float* partials) {
  __shared__ float red[kThreads];
  const int64_t PK = (int64_t)a.N * a.H * a.W * a.K;
  const PRBlendParams p = heaviside_params(a);
  const Sc sc = resolve(p);
  float part = 0.f;
  for (int64_t gs = (int64_t)blockIdx.x * kThreads + threadIdx.x; gs < PK;
       gs += (int64_t)gridDim.x * kThreads) {
    const int64_t gp = gs / a.K;
    const int k = (int)(gs - gp * a.K);
    float gacc;
    rast_count_score<NOISE>(p, sc, a.dists[gs], (uint32_t)gp, k, gs, PK, gacc);
    const float dD = (gacc / (float)a.Sr) * a.grad_prob[gs];
    a.grad_dists[gs] = -dD;
    part += dD;
  }
  red[threadIdx.x] = part;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(kThreads) sum_partials_kernel(const float* partials, int n, float* out) {
  __shared__ float red[kThreads];
  float acc = 0.f;
  for (int b = threadIdx.x; b < n; b += kThreads) acc += partials[b];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

__global__ void seed_advance_kernel(uint64_t* seeds, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) seeds[i] = seed_next(seeds[i]);
}

// pr_philox: the generator of PR_NOISE_PHILOX on caller-given counters (known-answer tests); R = 10
// (Random123's vectors) or the streams' kPhiloxRounds
template <int R>
__global__ void __launch_bounds__(kThreads) philox_kernel(const uint4* ctr, const uint64_t* keys, int64_t n,
                                                          uint4* words, float4* normals, float4* cauchy) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint4 c = ctr[i];
  const uint64_t k = keys[i];
  const U4 u = philox4x32<R>(U4{c.x, c.y, c.z, c.w}, (uint32_t)k, (uint32_t)(k >> 32));
  if (words) words[i] = make_uint4(u.x, u.y, u.z, u.w);
  float e[4];
  if (normals) {
    gauss4(u, e);
    normals[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
  if (cauchy) {
    cauchy4(u, e);
    cauchy[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
}

// ================================================================== host side
// A, B, PX, CP, queue length (+pad), then the uint16 rast queue [PB*K] (which also holds the
// uint8 candidate lists [PB][KP1]: 2K >= K+1)
// Workgroup shape: PB pixels (<= 32: the entry scan runs in one wave) and CAP entry records
// in LDS.  CAP is as large as an LDS target allows (kept small enough for ~8 workgroups per
// CU), clamped to [K + 1, PB * (K + 1)]: a block whose pixels hold more entries takes several
// passes.  Forward record: prob, z_inv / logit, queue and candidate bytes; backward record:
// 6 words, plus a_s per (pixel, sample).  The backward uses 16-pixel blocks on small frames
// (fewer than 4096 blocks of 32: cfg2 measured 0.093 vs 0.109 ms).
struct Shape {
  int PB, cap;
};
size_t fwd_lds(int PB, int cap) {
  return (size_t)(2 * cap + 9 * PB + 7) * sizeof(float) + (size_t)cap * (sizeof(uint16_t) + 1);
}
size_t bwd_lds(int PB, int cap, int Sa) {
  return (size_t)(6 * cap + PB * Sa + 17 * PB + 3) * sizeof(float) + (size_t)cap + (size_t)PB * Sa;
}
constexpr size_t kLdsTargetFwd = 20 * 1024, kLdsTargetBwd = 24 * 1024, kLdsMax = 60 * 1024;

// PR_BLEND_LDS_KB_FWD / _BWD (LDS target) and PR_BLEND_PB_FWD / _BWD (pixels) for sweeps
Shape pick_shape(int KP1, int Sa, int64_t P, bool bwd) {
  const char* e = getenv(bwd ? "PR_BLEND_LDS_KB_BWD" : "PR_BLEND_LDS_KB_FWD");
  const size_t target = e && atoi(e) > 0 ? (size_t)atoi(e) * 1024 : (bwd ? kLdsTargetBwd : kLdsTargetFwd);
  const char* b0 = getenv(bwd ? "PR_BLEND_PB_BWD" : "PR_BLEND_PB_FWD");
  int PB = b0 ? atoi(b0) : (bwd && P < 4096 * 32 ? 16 : 32);
  if (PB != 1 && PB != 2 && PB != 4 && PB != 8 && PB != 16) PB = 32;
  for (;; PB >>= 1) {
    const size_t fixed = bwd ? bwd_lds(PB, 0, Sa) : fwd_lds(PB, 0);
    const size_t per = bwd ? 6 * sizeof(float) + 1 : 2 * sizeof(float) + 3;
    const int fit = target > fixed ? (int)((target - fixed) / per) : 0;
    const int cap = max(KP1, min(PB * KP1, fit));
    const size_t lds = bwd ? bwd_lds(PB, cap, Sa) : fwd_lds(PB, cap);
    if (lds <= kLdsMax || PB == 1) return Shape{PB, cap};
  }
}

int check_params(const PRBlendParams& p, bool need_rast) {
  if (p.N <= 0 || p.H <= 0 || p.W <= 0 || p.K <= 0) return set_error(PR_ERR_ARG, "blend: empty shape");
  if (p.K > 255) return set_error(PR_ERR_ARG, "blend: faces_per_pixel must be <= 255");
  if (p.Sa <= 0 || (need_rast && p.Sr <= 0)) return set_error(PR_ERR_ARG, "blend: nb_samples must be > 0");
  if (p.Sa > 4096 || p.Sr > (1 << 24)) return set_error(PR_ERR_ARG, "blend: nb_samples too large");
  if (p.noise_mode != PR_NOISE_PHILOX && p.noise_mode != PR_NOISE_INJECTED)
    return set_error(PR_ERR_ARG, "blend: unknown noise mode");
  if (p.noise_mode == PR_NOISE_INJECTED && (!p.noise_a || (need_rast && !p.noise_r)))
    return set_error(PR_ERR_ARG, "blend: injected noise pointers missing");
  if (p.sample_offset_a < 0 || p.sample_offset_r < 0) return set_error(PR_ERR_ARG, "blend: negative sample offset");
  if (p.noise_mode == PR_NOISE_INJECTED && (p.sample_offset_a != 0 || p.sample_offset_r != 0))
    return set_error(PR_ERR_ARG, "blend: injected noise is indexed locally; sample offsets must be 0");
  if (!p.znear || !p.zfar) return set_error(PR_ERR_ARG, "blend: znear/zfar missing");
  const int64_t P = (int64_t)p.N * p.H * p.W;
  if (P >= (int64_t(1) << 31) || (int64_t)p.H * p.W >= (int64_t(1) << 31))
    return set_error(PR_ERR_ARG, "blend: too many pixels");
  return PR_OK;
}

int color_mode(int flags) {
  if (!(flags & PR_BLEND_COLOR)) return 0;
  if (flags & PR_BLEND_VERTEX) return 2;
  if (flags & PR_BLEND_PHONG) return 3;
  return (flags & PR_BLEND_COLOR_SPARSE) ? 4 : 1;
}

template <typename Fn, typename... Args>
void launch_grid(Fn* fn, int nblk, size_t lds, hipStream_t st, Args... args) {
  hipLaunchKernelGGL(fn, dim3(nblk), dim3(kThreads), lds, st, args...);
}

template <int NOISE, bool MULTI, bool SEG>
void launch_fwd(const FwdK& a, Geo geo, int NC, hipStream_t st, size_t lds, int nblk) {
  const bool rast = a.p.flags & PR_BLEND_RAST;
  const int cm = color_mode(a.p.flags);
  ktimer_mark(0, "blend_fwd_kernel", st);
  if (cm == 3) {  // (RAST only, static grid: pr_blend_fwd checks)
    if constexpr (!SEG) launch_grid(blend_fwd_kernel<NOISE, true, 3, MULTI, false>, nblk, lds, st, a, geo, NC);
  } else if (rast && cm == 2) launch_grid(blend_fwd_kernel<NOISE, true, 2, MULTI, SEG>, nblk, lds, st, a, geo, NC);
  else if (rast && cm == 1) launch_grid(blend_fwd_kernel<NOISE, true, 1, MULTI, SEG>, nblk, lds, st, a, geo, NC);
  else if (rast) launch_grid(blend_fwd_kernel<NOISE, true, 0, MULTI, SEG>, nblk, lds, st, a, geo, NC);
  else if (cm == 1) launch_grid(blend_fwd_kernel<NOISE, false, 1, MULTI, SEG>, nblk, lds, st, a, geo, NC);
  else if (cm == 2) launch_grid(blend_fwd_kernel<NOISE, false, 2, MULTI, SEG>, nblk, lds, st, a, geo, NC);
  else launch_grid(blend_fwd_kernel<NOISE, false, 0, MULTI, SEG>, nblk, lds, st, a, geo, NC);
  ktimer_mark(1, "blend_fwd_kernel", st);
}

template <int NOISE, bool MULTI, bool SEG>
void launch_bwd(const BwdK& a, Geo geo, hipStream_t st, size_t lds, int nblk, float* part) {
  const bool rast = a.p.flags & PR_BLEND_RAST;
  const int cm = color_mode(a.p.flags);
  ktimer_mark(0, "blend_bwd_kernel", st);
  if (cm == 4) {  // (RAST only, static grid: pr_blend_bwd checks)
    if constexpr (!SEG) launch_grid(blend_bwd_kernel<NOISE, true, 4, MULTI, false>, nblk, lds, st, a, geo, part);
  } else if (rast && cm == 2) launch_grid(blend_bwd_kernel<NOISE, true, 2, MULTI, SEG>, nblk, lds, st, a, geo, part);
  else if (rast && cm == 1) launch_grid(blend_bwd_kernel<NOISE, true, 1, MULTI, SEG>, nblk, lds, st, a, geo, part);
  else if (rast) launch_grid(blend_bwd_kernel<NOISE, true, 0, MULTI, SEG>, nblk, lds, st, a, geo, part);
  else if (cm == 1) launch_grid(blend_bwd_kernel<NOISE, false, 1, MULTI, SEG>, nblk, lds, st, a, geo, part);
  else if (cm == 2) launch_grid(blend_bwd_kernel<NOISE, false, 2, MULTI, SEG>, nblk, lds, st, a, geo, part);
  else launch_grid(blend_bwd_kernel<NOISE, false, 0, MULTI, SEG>, nblk, lds, st, a, geo, part);
  ktimer_mark(1, "blend_bwd_kernel", st);
}

Geo make_geo(const PRBlendParams& p, int PB, bool bwd) {
  Geo g;
  g.P = (int64_t)p.N * p.H * p.W;
  g.PK = g.P * p.K;
  g.K = p.K;
  g.KP1 = p.K + 1;
  g.PB = PB;
  g.HW = p.H * p.W;
  g.qK = kThreads / g.K; g.rK = kThreads % g.K;
  g.qK1 = kThreads / g.KP1; g.rK1 = kThreads % g.KP1;
  g.qS = kThreads / p.Sa; g.rS = kThreads % p.Sa;
  // lanes per pixel in the pixel phases: 8 (measured: 16 lanes for the backward's 16-pixel
  // blocks made its pixel phase slower -- longer shuffle prefixes outweigh shorter chunks)
  // PR_BLEND_LPP=16|32|64 (sweeps; capped at 256 / PB so every pixel keeps its lanes):
  // 8 / 16 / 32 measured within 1 % at cfg2 and cfg3
  // Default: 8, doubled while a lane would walk more than 8 slots and the block has idle
  // lanes (cfg4's 8-pixel backward blocks at K = 150: 32 lanes, chunks of 5 instead of 19).
  static const int lpp_env = getenv("PR_BLEND_LPP") ? atoi(getenv("PR_BLEND_LPP")) : 0;
  int lpp = 8;
  if (lpp_env == 8 || lpp_env == 16 || lpp_env == 32 || lpp_env == 64) lpp = lpp_env;
  else while (lpp < 64 && 2 * lpp * PB <= kThreads && g.KP1 > 8 * lpp) lpp <<= 1;
  while (lpp > 8 && lpp * PB > kThreads) lpp >>= 1;
  g.lpp = lpp;
  g.lsh = 31 - __builtin_clz(g.lpp);
  // centre-out block order (PR_BLEND_ORDER bit 0: forward, bit 1: backward; 0 = linear).
  // Default: the forward of a single frame only (cfg 2); on batches linear order is faster
  // (cfg 4 blend_fwd 5.16 -> 4.72 ms, cfg 3 equal), and the backward is linear everywhere.
  static const int order_env = getenv("PR_BLEND_ORDER") ? atoi(getenv("PR_BLEND_ORDER")) : -1;
  const int order = order_env >= 0 ? order_env : (p.N == 1 ? 1 : 0);
  g.bpi = (order >> (bwd ? 1 : 0) & 1) && g.HW % PB == 0 ? g.HW / PB : 0;
  static const int tail = getenv("PR_BLEND_TAIL") ? atoi(getenv("PR_BLEND_TAIL")) : 1;
  g.tail = tail;
  const char* empty = getenv("PR_BLEND_EMPTY");  // read per call: tests compare both paths in one process
  g.empty = empty ? atoi(empty) : 1;
  // interleaved pixel blocks (block_pixel): blocks must tile images.  Default: the backward's grids
  // of more than 8192 blocks (batches: cfg 3 4646 -> 4777, cfg 4 817 -> 841 frames/s with both
  // kernels interleaved, the backward's blocks even out over many generations: cfg 3 blend_bwd
  // 1.21 -> 1.07 ms; the forward lost there, 0.56 -> 0.60 ms, so it keeps consecutive blocks --
  // the two layouts are independent, winners and caches are indexed by physical pixel and slot);
  // one-frame grids keep consecutive blocks, whose empty-block shortcut
  // frees half the grid at once (interleaved, every block carries work and the forward's 2048
  // blocks outnumber the 1792 resident: cfg 2 3197 -> 3060, eval 3460 -> 3205;
  // profiles/r4_experiments.txt).  PR_BLEND_INTERLEAVE=0|1 forces it (read per call: tests compare
  // both layouts in one process); the segment plan turns it off.
  const char* il = getenv("PR_BLEND_INTERLEAVE");
  g.pm = (il ? atoi(il) != 0 : bwd && g.P / PB > 8192) && PB > 1 && g.HW % PB == 0;
  g.pmNBI = g.pm ? g.HW / PB : 1;
  g.pmW = p.W;
  g.pmA = g.pm && g.pmNBI % p.W == 0 ? ((int)(0.6180339887 * p.W) | 1) % p.W : 0;
  if (g.pm) g.bpi = 0;  // balanced blocks: no dispatch order to choose
  // fused scalar reduction's arrivals: relaxed (default) or acq_rel (PR_BLEND_SYNC_ORDER=release;
  // read per call: tests compare both in one process)
  const char* so = getenv("PR_BLEND_SYNC_ORDER");
  g.sync_rel = so && so[0] == 'r';
  return g;
}

// The segment plan's configuration for a call (both kernels: the forward computes the plan, the
// backward of the same call reads it, so both derive it from the same parameters).  Off without
// valid-prefix counts, on frames larger than kPlanMaxPixels (one plan workgroup; many-generation
// grids gain little), and with PR_BLEND_SEG=0.  E: entries per part, PR_BLEND_SEG_FWD / _BWD.
struct PlanCfg {
  bool on = false;
  PlanGeo q{};
  int lsh_max[2] = {0, 0};
  size_t bytes = 0;
};

PlanCfg plan_cfg(const PRBlendParams& p, const int32_t* pcnt) {
  PlanCfg c;
  // Off by default (PR_BLEND_SEG=1 opts in; read per call: tests compare both paths in one process).
  // Measured at cfg 2 (profiles/r4_blend_segments.txt): the backward kernel 74.7 -> 66.8 us at
  // E = 768, but the two plan kernels cost ~15 us and the forward's parts overflow its resident
  // workgroups (forward kernel 46 -> 53 us): a net loss of ~20 us per step.
  const char* env = getenv("PR_BLEND_SEG");
  const int64_t P = (int64_t)p.N * p.H * p.W;
  if (!pcnt || P > kPlanMaxPixels || !(env && atoi(env) != 0) || (p.flags & (PR_BLEND_PHONG | PR_BLEND_COLOR_SPARSE))) return c;
  const int KP1 = p.K + 1;
  // (read per call: tests drive several segment sizes in one process)
  const int e_env[2] = {getenv("PR_BLEND_SEG_FWD") ? atoi(getenv("PR_BLEND_SEG_FWD")) : 0,
                        getenv("PR_BLEND_SEG_BWD") ? atoi(getenv("PR_BLEND_SEG_BWD")) : 0};
  // lanes per pixel a part of few pixels may spread over (PR_BLEND_SEG_LPP / _BWD, sweeps).  Default:
  // the static grid's, which keeps every per-pixel reduction in the same order
  const int l_env[2] = {getenv("PR_BLEND_SEG_LPP") ? atoi(getenv("PR_BLEND_SEG_LPP")) : 0,
                        getenv("PR_BLEND_SEG_LPP_BWD") ? atoi(getenv("PR_BLEND_SEG_LPP_BWD")) : 0};
  constexpr int kDefaultE[2] = {512, 512};
  int64_t tblocks = 0, off = kPlanHeader;
  for (int w = 0; w < 2; ++w) {
    const Shape sh = pick_shape(KP1, p.Sa, P, w == 1);
    const Geo g = make_geo(p, sh.PB, w == 1);
    // 2 (K+1) <= E <= CAP - (K+1): parts are never empty and always fit the LDS records
    const int lo = 2 * KP1, hi = sh.cap - KP1;
    if (sh.PB < 4 || lo > hi) return c;
    c.q.PB[w] = sh.PB;
    c.q.E[w] = e_env[w] > 0 ? e_env[w] : kDefaultE[w];
    c.q.lo[w] = lo;
    c.q.hi[w] = hi;
    c.q.X[w] = (int)((P * KP1 + hi - 1) / hi);  // a dense frame's parts at E = hi
    c.q.bpi[w] = g.bpi;
    c.q.T[w] = (int)((P + sh.PB - 1) / sh.PB);
    int ls = g.lsh;
    while (ls < 6 && (2 << ls) <= l_env[w]) ++ls;
    c.lsh_max[w] = ls;
    tblocks += c.q.T[w];
  }
  if (tblocks > kPlanMaxBlocks) return c;
  c.q.P = (int)P;
  c.q.K = p.K;
  c.q.compact[0] = 1;
  // the backward compacts its entries when it draws the masked tail jointly (blend_bwd_kernel's tail)
  c.q.compact[1] = p.noise_mode == PR_NOISE_PHILOX && !(p.flags & PR_BLEND_AGG_CAUCHY) && make_geo(p, c.q.PB[1], true).tail;
  for (int w = 0; w < 2; ++w) {
    c.q.list[w] = (int)off;
    off += c.q.T[w] + c.q.X[w];
  }
  c.q.tots = (int)off;
  off += (tblocks + 1) / 2;
  c.bytes = (size_t)off * sizeof(int32_t);
  c.on = true;
  return c;
}

// PR_BLEND_PHONG's shading block: RAST, no VERTEX, texture UV or VERTEX with its buffers (pr_shade's
// checks, minus the per-slot tensors the blend owns)
int phong_check(const PRBlendParams& p, const PRShadeArgs* sh) {
  if (!(p.flags & PR_BLEND_RAST) || (p.flags & PR_BLEND_VERTEX) || !(p.flags & PR_BLEND_COLOR))
    return set_error(PR_ERR_ARG, "blend: PR_BLEND_PHONG needs RAST | COLOR and no VERTEX");
  if (!sh) return set_error(PR_ERR_ARG, "blend: PR_BLEND_PHONG without shade args");
  const PRShadeArgs& a = *sh;
  if (!a.faces || !a.verts || !a.normals || !a.light || !a.ambient || !a.diffuse_color || !a.specular_color ||
      !a.mat_diffuse || !a.mat_specular || !a.shininess || !a.camera)
    return set_error(PR_ERR_ARG, "blend: PR_BLEND_PHONG mesh / lighting buffer missing");
  if (a.texture == PR_TEX_UV ? (!a.face_uvs || !a.maps || a.Hm <= 0 || a.Wm <= 0)
      : a.texture == PR_TEX_VERTEX ? !a.vert_colors : true)
    return set_error(PR_ERR_ARG, "blend: PR_BLEND_PHONG texture must be PR_TEX_UV or PR_TEX_VERTEX with its buffers");
  if (a.V < 0 || a.F < 0 || a.V >= (int64_t(1) << 31)) return set_error(PR_ERR_ARG, "blend: bad mesh size");
  return PR_OK;
}


int64_t bwd_blocks(const PRBlendParams& p) {
  const int PB = pick_shape(p.K + 1, p.Sa, (int64_t)p.N * p.H * p.W, true).PB;
  const int64_t P = (int64_t)p.N * p.H * p.W;
  return (P + PB - 1) / PB;
}

}  // namespace
}  // namespace pr

using namespace pr;

#ifdef PR_BLEND_PROFILE
extern "C" int pr_blend_prof_dump(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_blend_prof), bytes < sizeof(g_blend_prof) ? bytes : sizeof(g_blend_prof),
                             0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

// Diagnostic (not part of the ABI header): resident workgroups per CU of the Philox vertex /
// texel-colour blend kernels at a shape, as the HIP occupancy calculator sees them; out[0..3] =
// fwd single-pass, fwd multi-pass, bwd single-pass, bwd multi-pass; out[4..7] = their LDS bytes.
extern "C" int pr_diag_blend_occupancy(int K, int Sa, long long P, int cm, int* out) {
  const int KP1 = K + 1;
  const Shape sf = pick_shape(KP1, Sa, P, false), sb = pick_shape(KP1, Sa, P, true);
  const size_t lf = fwd_lds(sf.PB, sf.cap), lb = bwd_lds(sb.PB, sb.cap, Sa);
  int r = 0;
  auto occ = [&](const void* f, size_t lds) {
    int n = -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, kThreads, lds) != hipSuccess) r = -1;
    return n;
  };
  if (cm == 2) {
    out[0] = occ((const void*)blend_fwd_kernel<PR_NOISE_PHILOX, true, 2, false, false>, lf);
    out[1] = occ((const void*)blend_fwd_kernel<PR_NOISE_PHILOX, true, 2, true, false>, lf);
    out[2] = occ((const void*)blend_bwd_kernel<PR_NOISE_PHILOX, true, 2, false, false>, lb);
    out[3] = occ((const void*)blend_bwd_kernel<PR_NOISE_PHILOX, true, 2, true, false>, lb);
  } else {
    out[0] = occ((const void*)blend_fwd_kernel<PR_NOISE_PHILOX, true, 1, false, false>, lf);
    out[1] = occ((const void*)blend_fwd_kernel<PR_NOISE_PHILOX, true, 1, true, false>, lf);
    out[2] = occ((const void*)blend_bwd_kernel<PR_NOISE_PHILOX, true, 1, false, false>, lb);
    out[3] = occ((const void*)blend_bwd_kernel<PR_NOISE_PHILOX, true, 1, true, false>, lb);
  }
  out[4] = out[5] = (int)lf;
  out[6] = out[7] = (int)lb;
  return r;
}

extern "C" int pr_blend_fwd(const PRBlendFwdArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "blend_fwd: null args");
  const PRBlendFwdArgs& a = *args;
  if (a.p.flags & PR_BLEND_SOFT) return soft_blend_fwd(a, reinterpret_cast<hipStream_t>(stream));
  const bool rast = a.p.flags & PR_BLEND_RAST, color = a.p.flags & PR_BLEND_COLOR;
  if (int e = check_params(a.p, rast)) return e;
  if (!a.pix_to_face && !a.mask) return set_error(PR_ERR_ARG, "blend_fwd: need pix_to_face or mask");
  const int cm = color_mode(a.p.flags);
  if ((a.p.flags & PR_BLEND_WINNERS_IN) && rast)
    return set_error(PR_ERR_ARG, "blend_fwd: PR_BLEND_WINNERS_IN takes probabilities (no PR_BLEND_RAST)");
  if (!a.zbuf || !a.winners || (rast && !a.dists) || (!rast && !a.prob) ||
      (cm == 1 && (!a.colors || !a.image)) || (!color && !a.weights) ||
      (cm == 2 && (!a.image || !a.bary || !a.faces || !a.vert_colors || !a.pix_to_face)) ||
      (cm == 3 && (!a.image || !a.bary || !a.pix_to_face)))
    return set_error(PR_ERR_ARG, "blend_fwd: missing buffer");
  if (cm == 3)
    if (int e = phong_check(a.p, a.shade)) return e;
  FwdK k{};
  static_cast<PRBlendFwdArgs&>(k) = a;
  if (cm == 3) k.sh = *a.shade;
  const int KP1 = a.p.K + 1;
  const Shape sh = pick_shape(KP1, a.p.Sa, (int64_t)a.p.N * a.p.H * a.p.W, false);
  const int PB = sh.PB;
  Geo geo = make_geo(a.p, PB, false);
  geo.cap = sh.cap;
  // slot chunks per (pixel, sample group) so that ~256 threads share the MC loop
  const int ng = ((a.p.sample_offset_a + a.p.Sa - 1) >> 2) - (a.p.sample_offset_a >> 2) + 1;
  int NC = 1;
  while (NC < 64 && PB * ng * NC * 2 <= kThreads && (KP1 + NC * 2 - 1) / (NC * 2) >= 4) NC <<= 1;
  int64_t nblk = (geo.P + PB - 1) / PB;
  const size_t lds = fwd_lds(PB, sh.cap);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool multi = sh.cap < PB * KP1;
  const PlanCfg pc = a.plan ? plan_cfg(a.p, a.pix_count) : PlanCfg{};
  if (pc.on) {  // entry-balanced segments (blend_plan_kernel) taken by resident workgroups
    blend_plan_count_kernel<<<(pc.q.P + kThreads - 1) / kThreads, kThreads, 0, st>>>(a.pix_count, pc.q, a.plan);
    blend_plan_list_kernel<<<1, kPlanThreads, 0, st>>>(pc.q, a.plan);
    if (int e = check_launch("blend_plan")) return e;
    geo.lsh_max = pc.lsh_max[0];
    geo.plan_fwd_list = pc.q.list[0];
    geo.pm = 0;  // the plan cuts consecutive pixel blocks
    nblk = pc.q.T[0] + pc.q.X[0];  // the plan's bound on the segments
    if (a.p.noise_mode == PR_NOISE_INJECTED) launch_fwd<PR_NOISE_INJECTED, false, true>(k, geo, NC, st, lds, (int)nblk);
    else launch_fwd<PR_NOISE_PHILOX, false, true>(k, geo, NC, st, lds, (int)nblk);
  } else if (a.p.noise_mode == PR_NOISE_INJECTED) {
    if (multi) launch_fwd<PR_NOISE_INJECTED, true, false>(k, geo, NC, st, lds, (int)nblk);
    else launch_fwd<PR_NOISE_INJECTED, false, false>(k, geo, NC, st, lds, (int)nblk);
  } else {
    if (multi) launch_fwd<PR_NOISE_PHILOX, true, false>(k, geo, NC, st, lds, (int)nblk);
    else launch_fwd<PR_NOISE_PHILOX, false, false>(k, geo, NC, st, lds, (int)nblk);
  }
  return check_launch("blend_fwd");
}


extern "C" size_t pr_blend_plan_size(const PRBlendParams* p) {
  if (!p || (p->flags & PR_BLEND_SOFT)) return 0;
  static const int32_t probe = 0;  // any non-null counts pointer
  const PlanCfg pc = plan_cfg(*p, &probe);
  return pc.on ? pc.bytes : 0;
}

extern "C" size_t pr_blend_bwd_workspace_size(const PRBlendBwdArgs* args) {
  if (!args) return 0;
  if (args->p.flags & PR_BLEND_SOFT) return soft_blend_workspace(args->p);
  const PlanCfg pc = args->plan ? plan_cfg(args->p, args->pix_count) : PlanCfg{};
  const size_t part = (size_t)(pc.on ? pc.q.T[1] + pc.q.X[1] : bwd_blocks(args->p)) * 4 * sizeof(float);
  return part;
}

extern "C" int pr_blend_bwd(const PRBlendBwdArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "blend_bwd: null args");
  const PRBlendBwdArgs& a = *args;
  if (a.p.flags & PR_BLEND_SOFT) return soft_blend_bwd(a, reinterpret_cast<hipStream_t>(stream));
  if (a.p.flags & PR_BLEND_AGG_UNIFORM)
    return set_error(PR_ERR_ARG, "blend_bwd: UniformAgg has no gradient (reference smoothagg.py:64-70)");
  const bool rast = a.p.flags & PR_BLEND_RAST, color = a.p.flags & PR_BLEND_COLOR;
  if (int e = check_params(a.p, rast)) return e;
  if (!a.pix_to_face && !a.mask) return set_error(PR_ERR_ARG, "blend_bwd: need pix_to_face or mask");
  if (!a.zbuf || !a.winners || !a.grad_zbuf || !a.grad_scalars ||
      (rast && (!a.dists || !a.grad_dists)) || (!rast && (!a.prob || !a.grad_prob)) ||
      (color_mode(a.p.flags) == 1 && (!a.colors || !a.grad_image || !a.grad_colors)) ||
      (color_mode(a.p.flags) == 2 && (!a.grad_image || !a.bary || !a.faces || !a.vert_colors ||
                                      !a.grad_bary || !a.pix_to_face)) ||
      (color_mode(a.p.flags) == 4 && (!a.colors || !a.grad_image || !a.grad_colors)) ||
      (!color && !a.grad_weights))
    return set_error(PR_ERR_ARG, "blend_bwd: missing buffer");
  if (a.p.flags & PR_BLEND_PHONG)
    return set_error(PR_ERR_ARG, "blend_bwd: PR_BLEND_PHONG is forward only (its backward: PR_BLEND_COLOR_SPARSE, then pr_shade_bwd)");
  if (color_mode(a.p.flags) == 4 && (!rast || (a.p.flags & PR_BLEND_VERTEX)))
    return set_error(PR_ERR_ARG, "blend_bwd: PR_BLEND_COLOR_SPARSE needs RAST and no VERTEX");
  const size_t need = pr_blend_bwd_workspace_size(args);
  if (!a.workspace || a.workspace_bytes < need) return set_error(PR_ERR_WORKSPACE, "blend_bwd: workspace too small");
  BwdK k{};
  static_cast<PRBlendBwdArgs&>(k) = a;

  const int KP1 = a.p.K + 1;
  const Shape sh = pick_shape(KP1, a.p.Sa, (int64_t)a.p.N * a.p.H * a.p.W, true);
  const int PB = sh.PB;
  Geo geo = make_geo(a.p, PB, true);
  geo.cap = sh.cap;
  int64_t nblk = (geo.P + PB - 1) / PB;
  size_t lds = bwd_lds(PB, sh.cap, a.p.Sa);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* part = reinterpret_cast<float*>(a.workspace);
  const bool multi = sh.cap < PB * KP1;
  const PlanCfg pc = a.plan ? plan_cfg(a.p, a.pix_count) : PlanCfg{};
  if (pc.on) {  // the forward's plan: entry-balanced segments taken by resident workgroups
    geo.lsh_max = pc.lsh_max[1];
    geo.plan_bwd_list = pc.q.list[1];
    geo.pm = 0;  // the plan cuts consecutive pixel blocks
    nblk = pc.q.T[1] + pc.q.X[1];  // the plan's bound on the segments
    if (a.p.noise_mode == PR_NOISE_INJECTED) launch_bwd<PR_NOISE_INJECTED, false, true>(k, geo, st, lds, (int)nblk, part);
    else launch_bwd<PR_NOISE_PHILOX, false, true>(k, geo, st, lds, (int)nblk, part);
  } else if (a.p.noise_mode == PR_NOISE_INJECTED) {
    if (multi) launch_bwd<PR_NOISE_INJECTED, true, false>(k, geo, st, lds, (int)nblk, part);
    else launch_bwd<PR_NOISE_INJECTED, false, false>(k, geo, st, lds, (int)nblk, part);
  } else {
    if (multi) launch_bwd<PR_NOISE_PHILOX, true, false>(k, geo, st, lds, (int)nblk, part);
    else launch_bwd<PR_NOISE_PHILOX, false, false>(k, geo, st, lds, (int)nblk, part);
  }
  if (int e = check_launch("blend_bwd")) return e;
  if (a.sync) return PR_OK;  // the scalars were reduced by the kernel's last workgroup
  blend_finalize_kernel<<<1, kThreads, 0, st>>>(part, (int)nblk, a.p, rast ? 1 : 0, a.grad_scalars,
                                                pc.on ? a.plan : nullptr);
  return check_launch("blend_finalize");
}

static int heaviside_check(const PRHeavisideArgs& a) {
  if (a.N <= 0 || a.H <= 0 || a.W <= 0 || a.K <= 0 || a.Sr <= 0) return set_error(PR_ERR_ARG, "heaviside: bad shape");
  if (a.noise_mode != PR_NOISE_PHILOX && a.noise_mode != PR_NOISE_INJECTED)
    return set_error(PR_ERR_ARG, "heaviside: unknown noise mode");
  if (a.noise_mode == PR_NOISE_INJECTED && (!a.noise_r || a.sample_offset_r != 0))
    return set_error(PR_ERR_ARG, "heaviside: injected noise missing or offset != 0");
  if (!a.dists) return set_error(PR_ERR_ARG, "heaviside: dists missing");
  if ((int64_t)a.N * a.H * a.W >= (int64_t(1) << 32)) return set_error(PR_ERR_ARG, "heaviside: too many pixels");
  return PR_OK;
}

static int heaviside_blocks(const PRHeavisideArgs& a) {
  const int64_t PK = (int64_t)a.N * a.H * a.W * a.K;
  return (int)std::min<int64_t>((PK + kThreads - 1) / kThreads, 4096);
}

extern "C" int pr_heaviside_fwd(const PRHeavisideArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "heaviside_fwd: null args");
  const PRHeavisideArgs& a = *args;
  if (int e = heaviside_check(a)) return e;
  if (!a.prob) return set_error(PR_ERR_ARG, "heaviside_fwd: prob missing");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.noise_mode == PR_NOISE_INJECTED)
    heaviside_fwd_kernel<PR_NOISE_INJECTED><<<heaviside_blocks(a), kThreads, 0, st>>>(a);
  else
    heaviside_fwd_kernel<PR_NOISE_PHILOX><<<heaviside_blocks(a), kThreads, 0, st>>>(a);
  return check_launch("heaviside_fwd");
}

extern "C" size_t pr_heaviside_bwd_workspace_size(const PRHeavisideArgs* args) {
  if (!args) return 0;
  return (size_t)heaviside_blocks(*args) * sizeof(float);
}

extern "C" int pr_heaviside_bwd(const PRHeavisideArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "heaviside_bwd: null args");
  const PRHeavisideArgs& a = *args;
  if (int e = heaviside_check(a)) return e;
  if (!a.grad_prob || !a.grad_dists || !a.grad_sigma) return set_error(PR_ERR_ARG, "heaviside_bwd: buffer missing");
  if (!a.workspace || a.workspace_bytes < pr_heaviside_bwd_workspace_size(args))
    return set_error(PR_ERR_WORKSPACE, "heaviside_bwd: workspace too small");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = heaviside_blocks(a);
  float* part = reinterpret_cast<float*>(a.workspace);
  if (a.noise_mode == PR_NOISE_INJECTED)
    heaviside_bwd_kernel<PR_NOISE_INJECTED><<<nb, kThreads, 0, st>>>(a, part);
  else
    heaviside_bwd_kernel<PR_NOISE_PHILOX><<<nb, kThreads, 0, st>>>(a, part);
  if (int e = check_launch("heaviside_bwd")) return e;
  sum_partials_kernel<<<1, kThreads, 0, st>>>(part, nb, a.grad_sigma);
  return check_launch("heaviside_sum");
}

extern "C" int pr_seed_advance(uint64_t* seeds, int32_t n, void* stream) {
  if (!seeds || n <= 0) return set_error(PR_ERR_ARG, "seed_advance: bad args");
  seed_advance_kernel<<<(n + 63) / 64, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(seeds, n);
  return check_launch("seed_advance");
}

extern "C" int pr_philox(const uint32_t* counters, const uint64_t* keys, int64_t n, uint32_t* words, float* normals,
                         float* cauchy, int32_t rounds, void* stream) {
  if (!counters || !keys || n <= 0 || n > (int64_t(1) << 40)) return set_error(PR_ERR_ARG, "philox: bad args");
  if (rounds != 10 && rounds != kPhiloxRounds) return set_error(PR_ERR_ARG, "philox: rounds must be 10 or the streams'");
  const int64_t nb = (n + kThreads - 1) / kThreads;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint4* c = reinterpret_cast<const uint4*>(counters);
  uint4* w = reinterpret_cast<uint4*>(words);
  float4 *nm = reinterpret_cast<float4*>(normals), *cy = reinterpret_cast<float4*>(cauchy);
  if (rounds == 10) philox_kernel<10><<<(unsigned)nb, kThreads, 0, st>>>(c, keys, n, w, nm, cy);
  else philox_kernel<kPhiloxRounds><<<(unsigned)nb, kThreads, 0, st>>>(c, keys, n, w, nm, cy);
  return check_launch("philox");
}
