// Deterministic SoftRas blend: smooth_rgb_blend (random_rasterizer.py:34-56) with SoftRast
// (smoothrast.py:126-134, P = sigmoid(-d / sigma)) and SoftAgg (smoothagg.py:165-182, W =
// softmax(z / gamma) over the K face logits and the background logit) -- eval.py's default
// "softras" renderer (eval.py:70, :161-163).  PR_BLEND_SOFT selects it in pr_blend_fwd/bwd.
//
// One thread per pixel walks the pixel's valid slots (the rasterizer's valid-prefix counts,
// or every slot's pix_to_face >= 0 without them): masked slots have P = 0, logit -inf, weight
// exactly 0 and zero gradients, so they are never read.  For K <= 64 (eval.py's 50) the
// *_lanes kernels spread a pixel's slots over 16 lanes instead (coalesced rows; round 5).  The backward recomputes the forward
// in registers (nothing is saved between the passes) and reduces d sigma / d gamma / d alpha
// per workgroup in a fixed order (deterministic), summed by a one-workgroup finalize.
//
// Gradient conventions kept from the reference: log_corrected (1/P with inf -> 0),
// prod_corrected (the x-gradient as a nansum with y = -inf -> 0, twice: gamma/alpha times
// log P, and 1/gamma times the logits), torch.max's routing of d zmax to the first maximum
// (only when max >= eps: clamp(min=eps)), and torch.prod's exclusive-product backward.
#include "pr_common.h"

namespace pr {
namespace {

constexpr float kNegInf = -__builtin_inff();

struct SoftSc {
  float sigma, gamma, alpha;
};

PR_DEV SoftSc soft_scalars(const PRBlendParams& p) {
  SoftSc s{p.sigma, p.gamma, p.alpha};
  if (p.scalars[0]) s.sigma = *p.scalars[0];
  if (p.scalars[1]) s.gamma = *p.scalars[1];
  if (p.scalars[2]) s.alpha = *p.scalars[2];
  return s;
}

// per-pixel state shared by the two passes
struct SoftPix {
  int n;          // valid slots (a prefix when counts are given)
  float zmax;     // clamp(max z_inv, eps)
  int jmax;       // first argmax of z_inv over all K slots
  bool zmax_grad; // max z_inv >= eps: d zmax reaches z_inv[jmax]
  float ymax, ssum;
};

PR_DEV bool valid_slot(const PRBlendFwdArgs* f, const PRBlendBwdArgs* b, int64_t gs, int k, int cnt) {
  if (cnt >= 0) return k < cnt;
  const int64_t* p2f = f ? f->pix_to_face : b->pix_to_face;
  return p2f[gs] >= 0;
}

// sigmoid(-d / sigma) as torch: 1 / (1 + exp(-x)) with x = (-d) / sigma
PR_DEV float soft_prob(float d, float sigma, float& u) {
  u = (-d) / sigma;
  return 1.f / (1.f + expf(-u));
}

template <typename A>
PR_DEV void soft_color(const A& a, int64_t gs, float c[3]) {
  c[0] = a.colors[gs * 3]; c[1] = a.colors[gs * 3 + 1]; c[2] = a.colors[gs * 3 + 2];
}

// pass 1 (both kernels): zmax / first argmax over the pixel's K slots (masked slots have
// z_inv = 0), then the softmax max and normaliser over the K+1 logits
template <typename A>
PR_DEV SoftPix soft_pixel(const A& a, const PRBlendFwdArgs* fa, const PRBlendBwdArgs* ba, int64_t p, int cnt,
                          const SoftSc& sc, float zn, float zf, float inv_g, float gal) {
  const int K = a.p.K;
  const float den = zf - zn;
  SoftPix s;
  s.n = 0;
  float zm = kNegInf;
  int jm = 0;
  const int kend = cnt >= 0 ? cnt : K;
  for (int k = 0; k < kend; ++k) {
    const int64_t gs = p * K + k;
    if (!valid_slot(fa, ba, gs, k, cnt)) continue;
    const float zi = ((zf - a.zbuf[gs]) / den) * 1.f;
    if (zi > zm) { zm = zi; jm = k; }
    ++s.n;
  }
  // masked slots (z_inv = 0): the first one competes for the max at its own index
  if (cnt >= 0 ? cnt < K : s.n < K) {
    int jz = 0;
    if (cnt >= 0) jz = cnt;
    else
      for (int k = 0; k < K; ++k)
        if (!valid_slot(fa, ba, p * K + k, k, cnt)) { jz = k; break; }
    if (0.f > zm || (0.f == zm && jz < jm)) { zm = 0.f; jm = jz; }
  }
  s.jmax = jm;
  s.zmax_grad = zm >= a.p.eps;
  s.zmax = zm >= a.p.eps ? zm : a.p.eps;
  // softmax statistics of y_j = (1/gamma) z_j
  float ym = inv_g * (a.p.eps - s.zmax);  // background logit
  for (int k = 0; k < kend; ++k) {
    const int64_t gs = p * K + k;
    if (!valid_slot(fa, ba, gs, k, cnt)) continue;
    float u;
    const float P = soft_prob(a.dists[gs], sc.sigma, u);
    const float zi = (zf - a.zbuf[gs]) / den;
    const float z = (gal * logf(P) + zi) - s.zmax;
    ym = fmaxf(ym, inv_g * z);
  }
  s.ymax = ym;
  float ss = expf(inv_g * (a.p.eps - s.zmax) - ym);
  for (int k = 0; k < kend; ++k) {
    const int64_t gs = p * K + k;
    if (!valid_slot(fa, ba, gs, k, cnt)) continue;
    float u;
    const float P = soft_prob(a.dists[gs], sc.sigma, u);
    const float zi = (zf - a.zbuf[gs]) / den;
    const float z = (gal * logf(P) + zi) - s.zmax;
    ss += expf(inv_g * z - ym);
  }
  s.ssum = ss;
  return s;
}

__global__ void __launch_bounds__(kThreads) soft_fwd_kernel(PRBlendFwdArgs a, int64_t P, int HW) {
  const SoftSc sc = soft_scalars(a.p);
  const float inv_g = 1.f / sc.gamma, gal = sc.gamma / sc.alpha;
  const int K = a.p.K;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < P; p += (int64_t)gridDim.x * kThreads) {
    const int n = (int)(p / HW);
    const float zn = a.p.znear[n], zf = a.p.zfar[n], den = zf - zn;
    const int cnt = a.pix_count ? a.pix_count[p] : -1;
    const SoftPix s = soft_pixel(a, &a, (const PRBlendBwdArgs*)nullptr, p, cnt, sc, zn, zf, inv_g, gal);
    float rgb[3] = {0.f, 0.f, 0.f}, alpha = 1.f;
    const int kend = cnt >= 0 ? cnt : K;
    for (int k = 0; k < kend; ++k) {
      const int64_t gs = p * K + k;
      if (!valid_slot(&a, nullptr, gs, k, cnt)) continue;
      float u;
      const float Pk = soft_prob(a.dists[gs], sc.sigma, u);
      alpha *= 1.f - Pk;
      const float zi = (zf - a.zbuf[gs]) / den;
      const float z = (gal * logf(Pk) + zi) - s.zmax;
      const float w = expf(inv_g * z - s.ymax) / s.ssum;
      float c[3];
      soft_color(a, gs, c);
      rgb[0] += w * c[0]; rgb[1] += w * c[1]; rgb[2] += w * c[2];
    }
    const float wb = expf(inv_g * (a.p.eps - s.zmax) - s.ymax) / s.ssum;
    float* o = a.image + p * 4;
    o[0] = rgb[0] + wb * a.p.background[0];
    o[1] = rgb[1] + wb * a.p.background[1];
    o[2] = rgb[2] + wb * a.p.background[2];
    o[3] = 1.f - alpha;
  }
}

__global__ void __launch_bounds__(kThreads) soft_bwd_kernel(PRBlendBwdArgs a, int64_t P, int HW, float* partials) {
  __shared__ float red[kThreads * 3];
  const SoftSc sc = soft_scalars(a.p);
  const float inv_g = 1.f / sc.gamma, gal = sc.gamma / sc.alpha;
  const int K = a.p.K;
  float acc_sig = 0.f, acc_inv = 0.f, acc_gal = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < P; p += (int64_t)gridDim.x * kThreads) {
    const int n = (int)(p / HW);
    const float zn = a.p.znear[n], zf = a.p.zfar[n], den = zf - zn;
    const int cnt = a.pix_count ? a.pix_count[p] : -1;
    const SoftPix s = soft_pixel(a, (const PRBlendFwdArgs*)nullptr, &a, p, cnt, sc, zn, zf, inv_g, gal);
    const float* gi = a.grad_image + p * 4;
    const float gr[3] = {gi[0], gi[1], gi[2]}, gA = gi[3];
    const int kend = cnt >= 0 ? cnt : K;
    // sweep 1: weights, the softmax dot, the alpha product (zeros counted separately)
    const float wb = expf(inv_g * (a.p.eps - s.zmax) - s.ymax) / s.ssum;
    const float gWb = (gr[0] * a.p.background[0] + gr[1] * a.p.background[1]) + gr[2] * a.p.background[2];
    float dot = wb * gWb, prod_nz = 1.f, alpha = 1.f;
    int zeros = 0;
    for (int k = 0; k < kend; ++k) {
      const int64_t gs = p * K + k;
      if (!valid_slot(nullptr, &a, gs, k, cnt)) continue;
      float u;
      const float Pk = soft_prob(a.dists[gs], sc.sigma, u);
      const float f = 1.f - Pk;
      alpha *= f;
      if (f == 0.f) ++zeros; else prod_nz *= f;
      const float zi = (zf - a.zbuf[gs]) / den;
      const float z = (gal * logf(Pk) + zi) - s.zmax;
      const float w = expf(inv_g * z - s.ymax) / s.ssum;
      float c[3];
      soft_color(a, gs, c);
      dot += w * ((gr[0] * c[0] + gr[1] * c[1]) + gr[2] * c[2]);
    }
    // background logit z_K = eps - zmax
    const float gyb = wb * (gWb - dot);
    const float gzb = inv_g * gyb;
    acc_inv += (a.p.eps - s.zmax) * gyb;
    float gzmax = -gzb;
    // sweep 2: slot gradients; d z_inv of the first argmax gets d zmax afterwards
    float gz_at_jmax = 0.f;
    for (int k = 0; k < K; ++k) {
      const int64_t gs = p * K + k;
      const bool v = k < kend && valid_slot(nullptr, &a, gs, k, cnt);
      if (!v) {  // masked slot (the padded tail is not read): zero gradients
        a.grad_dists[gs] = 0.f; a.grad_zbuf[gs] = 0.f;
        a.grad_colors[gs * 3] = 0.f; a.grad_colors[gs * 3 + 1] = 0.f; a.grad_colors[gs * 3 + 2] = 0.f;
        continue;
      }
      float u;
      const float Pk = soft_prob(a.dists[gs], sc.sigma, u);
      const float zi = (zf - a.zbuf[gs]) / den;
      const float L = logf(Pk);
      const float z = (gal * L + zi) - s.zmax;
      const float w = expf(inv_g * z - s.ymax) / s.ssum;
      float c[3];
      soft_color(a, gs, c);
      a.grad_colors[gs * 3] = w * gr[0]; a.grad_colors[gs * 3 + 1] = w * gr[1]; a.grad_colors[gs * 3 + 2] = w * gr[2];
      const float gW = (gr[0] * c[0] + gr[1] * c[1]) + gr[2] * c[2];
      const float gy = w * (gW - dot);
      const float gz = inv_g * gy;
      if (z != kNegInf) acc_inv += z * gy;      // prod_corrected(1/gamma, z): inf -> 0, nansum
      gzmax -= gz;
      if (k == s.jmax) gz_at_jmax = gz;
      const float gL = gal * gz;                // prod_corrected(gamma/alpha, L)
      if (L != kNegInf) acc_gal += L * gz;
      // d P: log_corrected (1/P, inf -> 0) and the alpha product (exclusive product)
      const float rP = 1.f / Pk;
      float gP = gL * (isinf(rP) ? 0.f : rP);
      const float f = 1.f - Pk;
      const float excl = zeros == 0 ? alpha / f : (zeros == 1 && f == 0.f ? prod_nz : 0.f);
      gP += gA * excl;                          // d alpha_chan = -gA, d/dP (1-P) = -1
      // sigmoid(u), u = (-d) / sigma
      const float gu = gP * (Pk * (1.f - Pk));
      a.grad_dists[gs] = -(gu / sc.sigma);
      acc_sig += -gu * u / sc.sigma;
      a.grad_zbuf[gs] = -gz / den;              // d z_inv (d zmax added below)
    }
    // d zmax -> z_inv[jmax] (first maximum), only if max z_inv >= eps (clamp(min=eps))
    if (s.zmax_grad && gzmax != 0.f) {
      const int64_t gs = p * K + s.jmax;
      if (s.jmax < kend && valid_slot(nullptr, &a, gs, s.jmax, cnt))
        a.grad_zbuf[gs] = -(gz_at_jmax + gzmax) / den;
    }
  }
  red[threadIdx.x * 3] = acc_sig;
  red[threadIdx.x * 3 + 1] = acc_inv;
  red[threadIdx.x * 3 + 2] = acc_gal;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int c = 0; c < 3; ++c) red[threadIdx.x * 3 + c] += red[(threadIdx.x + s) * 3 + c];
    __syncthreads();
  }
  if (threadIdx.x < 3) partials[blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x];
}

__global__ void __launch_bounds__(kThreads) soft_finalize_kernel(const float* partials, int nblk, PRBlendParams p,
                                                                 float* out) {
  __shared__ float red[kThreads * 3];
  float acc[3] = {0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < nblk; b += kThreads)
    for (int c = 0; c < 3; ++c) acc[c] += partials[b * 3 + c];
  for (int c = 0; c < 3; ++c) red[threadIdx.x * 3 + c] = acc[c];
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int c = 0; c < 3; ++c) red[threadIdx.x * 3 + c] += red[(threadIdx.x + s) * 3 + c];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const SoftSc sc = soft_scalars(p);
    const float dsig = red[0], dinv = red[1], dgal = red[2];
    const float inv_g = 1.f / sc.gamma;
    out[0] = dsig;
    // gamma enters as gamma / alpha (prod_corrected) and as 1 / gamma (softmax temperature)
    out[1] = dgal / sc.alpha + (-dinv * (inv_g * inv_g));
    out[2] = -dgal * sc.gamma / (sc.alpha * sc.alpha);
  }
}

// ---- the backward with the pixel's slots across lanes (K <= 64): G = 16 lanes per pixel, slot
// k on lane k % 16, so a pixel's dists / zbuf / colours and its five gradient rows are read and
// written as contiguous runs (the one-thread-per-pixel walk strides them by K floats: ~5x the
// time at K = 50), the per-pixel maxima / sums / products are 16-lane butterflies.  Same
// arithmetic per slot as soft_bwd_kernel; the per-pixel sums and products associate in a
// different order (tests/test_gpu_softblend.py holds both against the reference at 1e-5).
constexpr int kSoftG = 16, kSoftS = 4;  // lanes per pixel, slots per lane (K <= 64)
constexpr int kSoftPix = kThreads / kSoftG;  // pixels per workgroup pass

PR_DEV float gmax(float v) {
#pragma unroll
  for (int o = kSoftG / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
PR_DEV float gsum(float v) {
#pragma unroll
  for (int o = kSoftG / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
PR_DEV float gprod(float v) {
#pragma unroll
  for (int o = kSoftG / 2; o > 0; o >>= 1) v *= __shfl_xor(v, o);
  return v;
}
PR_DEV int gisum(int v) {
#pragma unroll
  for (int o = kSoftG / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
PR_DEV int gimin(int v) {
#pragma unroll
  for (int o = kSoftG / 2; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

__global__ void __launch_bounds__(kThreads) soft_bwd_lanes_kernel(PRBlendBwdArgs a, int64_t P, int HW,
                                                                  float* partials) {
  __shared__ float red[kThreads * 3];
  const SoftSc sc = soft_scalars(a.p);
  const float inv_g = 1.f / sc.gamma, gal = sc.gamma / sc.alpha;
  const int K = a.p.K;
  const int g = threadIdx.x % kSoftG;
  float acc_sig = 0.f, acc_inv = 0.f, acc_gal = 0.f;
  for (int64_t p0 = (int64_t)blockIdx.x * kSoftPix; p0 < P; p0 += (int64_t)gridDim.x * kSoftPix) {
    const int64_t p = p0 + threadIdx.x / kSoftG;
    const bool live = p < P;  // group-uniform
    const int64_t pc = live ? p : P - 1;
    const int n = (int)(pc / HW);
    const float zn = a.p.znear[n], zf = a.p.zfar[n], den = zf - zn;
    const int cnt = a.pix_count ? a.pix_count[pc] : -1;
    // this lane's slots k = g + 16 j: validity, the sigmoid and the logit terms
    bool v[kSoftS];
    float d[kSoftS], zi[kSoftS], Pk[kSoftS], u[kSoftS], c[kSoftS][3];
    float zm = kNegInf;
    int jm = 1 << 30, nv = 0, jz = 1 << 30;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j) {
      const int k = g + kSoftG * j;
      const int64_t gs = pc * K + k;
      v[j] = live && k < K && (cnt >= 0 ? k < cnt : a.pix_to_face[gs] >= 0);
      if (live && k < K && !v[j]) jz = min(jz, k);
      d[j] = v[j] ? a.dists[gs] : 0.f;
      zi[j] = v[j] ? ((zf - a.zbuf[gs]) / den) * 1.f : 0.f;
      c[j][0] = v[j] ? a.colors[gs * 3] : 0.f;
      c[j][1] = v[j] ? a.colors[gs * 3 + 1] : 0.f;
      c[j][2] = v[j] ? a.colors[gs * 3 + 2] : 0.f;
      Pk[j] = v[j] ? soft_prob(d[j], sc.sigma, u[j]) : 0.f;
      if (!v[j]) u[j] = 0.f;
      if (v[j]) {
        ++nv;
        if (zi[j] > zm || (zi[j] == zm && k < jm)) { zm = zi[j]; jm = k; }
      }
    }
    // first argmax over the pixel: the largest z_inv, ties to the smaller slot
#pragma unroll
    for (int o = kSoftG / 2; o > 0; o >>= 1) {
      const float oz = __shfl_xor(zm, o);
      const int oj = __shfl_xor(jm, o);
      if (oz > zm || (oz == zm && oj < jm)) { zm = oz; jm = oj; }
    }
    nv = gisum(nv);
    jz = gimin(jz);
    if (jz < K) {  // a masked slot (z_inv = 0) competes at its own index (soft_pixel)
      if (!(nv > 0) || 0.f > zm || (0.f == zm && jz < jm)) { zm = 0.f; jm = jz; }
    }
    if (nv == 0 && jz >= K) jm = 0;
    const bool zmax_grad = zm >= a.p.eps;
    const float zmax = zm >= a.p.eps ? zm : a.p.eps;
    float L[kSoftS], z[kSoftS];
    float ym = kNegInf;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j) {
      L[j] = v[j] ? logf(Pk[j]) : 0.f;
      z[j] = v[j] ? (gal * L[j] + zi[j]) - zmax : 0.f;
      if (v[j]) ym = fmaxf(ym, inv_g * z[j]);
    }
    ym = fmaxf(gmax(ym), inv_g * (a.p.eps - zmax));
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j)
      if (v[j]) ss += expf(inv_g * z[j] - ym);
    ss = gsum(ss) + expf(inv_g * (a.p.eps - zmax) - ym);
    const float* gi = a.grad_image + pc * 4;
    const float gr[3] = {gi[0], gi[1], gi[2]}, gA = gi[3];
    const float wb = expf(inv_g * (a.p.eps - zmax) - ym) / ss;
    const float gWb = (gr[0] * a.p.background[0] + gr[1] * a.p.background[1]) + gr[2] * a.p.background[2];
    float w[kSoftS], gW[kSoftS];
    float dotl = 0.f, alpha = 1.f, prod_nz = 1.f;
    int zeros = 0;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j) {
      w[j] = v[j] ? expf(inv_g * z[j] - ym) / ss : 0.f;
      gW[j] = (gr[0] * c[j][0] + gr[1] * c[j][1]) + gr[2] * c[j][2];
      if (v[j]) {
        const float f = 1.f - Pk[j];
        alpha *= f;
        if (f == 0.f) ++zeros; else prod_nz *= f;
        dotl += w[j] * gW[j];
      }
    }
    const float dot = wb * gWb + gsum(dotl);
    alpha = gprod(alpha);
    prod_nz = gprod(prod_nz);
    zeros = gisum(zeros);
    const float gyb = wb * (gWb - dot);
    const float gzb = inv_g * gyb;
    float inv_l = live && g == 0 ? (a.p.eps - zmax) * gyb : 0.f;
    float gz_sum = 0.f, gz_jmax = 0.f;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j) {
      const int k = g + kSoftG * j;
      if (!live || k >= K) continue;
      const int64_t gs = pc * K + k;
      if (!v[j]) {
        a.grad_dists[gs] = 0.f; a.grad_zbuf[gs] = 0.f;
        a.grad_colors[gs * 3] = 0.f; a.grad_colors[gs * 3 + 1] = 0.f; a.grad_colors[gs * 3 + 2] = 0.f;
        continue;
      }
      a.grad_colors[gs * 3] = w[j] * gr[0]; a.grad_colors[gs * 3 + 1] = w[j] * gr[1];
      a.grad_colors[gs * 3 + 2] = w[j] * gr[2];
      const float gy = w[j] * (gW[j] - dot);
      const float gz = inv_g * gy;
      if (z[j] != kNegInf) inv_l += z[j] * gy;
      gz_sum += gz;
      if (k == jm) gz_jmax = gz;
      const float gL = gal * gz;
      if (L[j] != kNegInf) acc_gal += L[j] * gz;
      const float rP = 1.f / Pk[j];
      float gP = gL * (isinf(rP) ? 0.f : rP);
      const float f = 1.f - Pk[j];
      const float excl = zeros == 0 ? alpha / f : (zeros == 1 && f == 0.f ? prod_nz : 0.f);
      gP += gA * excl;
      const float gu = gP * (Pk[j] * (1.f - Pk[j]));
      a.grad_dists[gs] = -(gu / sc.sigma);
      acc_sig += -gu * u[j] / sc.sigma;
      a.grad_zbuf[gs] = -gz / den;
    }
    acc_inv += inv_l;
    // d zmax -> z_inv[jmax] (first maximum), only if max z_inv >= eps, and only a valid slot
    const float gzmax = -gzb - gsum(gz_sum);
    const float gzj = gsum(gz_jmax);
    if (live && g == (jm % kSoftG) && zmax_grad && gzmax != 0.f && jm < K) {
      const int64_t gs = pc * K + jm;
      const bool vj = cnt >= 0 ? jm < cnt : a.pix_to_face[gs] >= 0;
      if (vj) a.grad_zbuf[gs] = -(gzj + gzmax) / den;
    }
  }
  red[threadIdx.x * 3] = acc_sig;
  red[threadIdx.x * 3 + 1] = acc_inv;
  red[threadIdx.x * 3 + 2] = acc_gal;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int c = 0; c < 3; ++c) red[threadIdx.x * 3 + c] += red[(threadIdx.x + s) * 3 + c];
    __syncthreads();
  }
  if (threadIdx.x < 3) partials[blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x];
}

// the forward with the same lane layout (image only)
__global__ void __launch_bounds__(kThreads) soft_fwd_lanes_kernel(PRBlendFwdArgs a, int64_t P, int HW) {
  const SoftSc sc = soft_scalars(a.p);
  const float inv_g = 1.f / sc.gamma, gal = sc.gamma / sc.alpha;
  const int K = a.p.K;
  const int g = threadIdx.x % kSoftG;
  for (int64_t p0 = (int64_t)blockIdx.x * kSoftPix; p0 < P; p0 += (int64_t)gridDim.x * kSoftPix) {
    const int64_t p = p0 + threadIdx.x / kSoftG;
    const bool live = p < P;
    const int64_t pc = live ? p : P - 1;
    const int n = (int)(pc / HW);
    const float zn = a.p.znear[n], zf = a.p.zfar[n], den = zf - zn;
    const int cnt = a.pix_count ? a.pix_count[pc] : -1;
    bool v[kSoftS];
    float zi[kSoftS], Pk[kSoftS], c[kSoftS][3];
    float zm = kNegInf;
    int jm = 1 << 30, nv = 0, jz = 1 << 30;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j) {
      const int k = g + kSoftG * j;
      const int64_t gs = pc * K + k;
      v[j] = live && k < K && (cnt >= 0 ? k < cnt : a.pix_to_face[gs] >= 0);
      if (live && k < K && !v[j]) jz = min(jz, k);
      zi[j] = v[j] ? ((zf - a.zbuf[gs]) / den) * 1.f : 0.f;
      c[j][0] = v[j] ? a.colors[gs * 3] : 0.f;
      c[j][1] = v[j] ? a.colors[gs * 3 + 1] : 0.f;
      c[j][2] = v[j] ? a.colors[gs * 3 + 2] : 0.f;
      float u;
      Pk[j] = v[j] ? soft_prob(a.dists[gs], sc.sigma, u) : 0.f;
      if (v[j]) {
        ++nv;
        if (zi[j] > zm || (zi[j] == zm && k < jm)) { zm = zi[j]; jm = k; }
      }
    }
#pragma unroll
    for (int o = kSoftG / 2; o > 0; o >>= 1) {
      const float oz = __shfl_xor(zm, o);
      const int oj = __shfl_xor(jm, o);
      if (oz > zm || (oz == zm && oj < jm)) { zm = oz; jm = oj; }
    }
    nv = gisum(nv);
    jz = gimin(jz);
    if (jz < K && (!(nv > 0) || 0.f > zm || (0.f == zm && jz < jm))) zm = 0.f;
    const float zmax = zm >= a.p.eps ? zm : a.p.eps;
    float z[kSoftS];
    float ym = kNegInf;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j) {
      z[j] = v[j] ? (gal * logf(Pk[j]) + zi[j]) - zmax : 0.f;
      if (v[j]) ym = fmaxf(ym, inv_g * z[j]);
    }
    ym = fmaxf(gmax(ym), inv_g * (a.p.eps - zmax));
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j)
      if (v[j]) ss += expf(inv_g * z[j] - ym);
    ss = gsum(ss) + expf(inv_g * (a.p.eps - zmax) - ym);
    float rgb[3] = {0.f, 0.f, 0.f}, alpha = 1.f;
#pragma unroll
    for (int j = 0; j < kSoftS; ++j) {
      if (!v[j]) continue;
      alpha *= 1.f - Pk[j];
      const float w = expf(inv_g * z[j] - ym) / ss;
      rgb[0] += w * c[j][0]; rgb[1] += w * c[j][1]; rgb[2] += w * c[j][2];
    }
    rgb[0] = gsum(rgb[0]); rgb[1] = gsum(rgb[1]); rgb[2] = gsum(rgb[2]);
    alpha = gprod(alpha);
    if (live && g == 0) {
      const float wb = expf(inv_g * (a.p.eps - zmax) - ym) / ss;
      float* o = a.image + p * 4;
      o[0] = rgb[0] + wb * a.p.background[0];
      o[1] = rgb[1] + wb * a.p.background[1];
      o[2] = rgb[2] + wb * a.p.background[2];
      o[3] = 1.f - alpha;
    }
  }
}

int soft_blocks(int64_t P) { return (int)std::min<int64_t>((P + kThreads - 1) / kThreads, 4096); }
bool soft_lanes(const PRBlendParams& p) {
  static const bool off = getenv("PR_SOFT_LANES") && getenv("PR_SOFT_LANES")[0] == '0';
  return p.K <= kSoftG * kSoftS && !off;
}
int soft_bwd_blocks(const PRBlendParams& p) {
  const int64_t P = (int64_t)p.N * p.H * p.W;
  return soft_lanes(p) ? (int)std::min<int64_t>((P + kSoftPix - 1) / kSoftPix, 8192) : soft_blocks(P);
}

}  // namespace

size_t soft_blend_workspace(const PRBlendParams& p) {
  return (size_t)soft_bwd_blocks(p) * 3 * sizeof(float);
}

int soft_blend_fwd(const PRBlendFwdArgs& a, hipStream_t st) {
  const PRBlendParams& p = a.p;
  if (p.N <= 0 || p.H <= 0 || p.W <= 0 || p.K <= 0) return set_error(PR_ERR_ARG, "soft blend: empty shape");
  if (!(p.flags & PR_BLEND_RAST) || !(p.flags & PR_BLEND_COLOR) || (p.flags & PR_BLEND_VERTEX))
    return set_error(PR_ERR_ARG, "soft blend: needs RAST | COLOR with texel colours");
  if (!a.dists || !a.zbuf || !a.colors || !a.image || !a.pix_to_face || !p.znear || !p.zfar)
    return set_error(PR_ERR_ARG, "soft blend: missing buffer");
  const int64_t P = (int64_t)p.N * p.H * p.W;
  if (soft_lanes(p)) soft_fwd_lanes_kernel<<<soft_bwd_blocks(p), kThreads, 0, st>>>(a, P, p.H * p.W);
  else soft_fwd_kernel<<<soft_blocks(P), kThreads, 0, st>>>(a, P, p.H * p.W);
  return check_launch("soft_blend_fwd");
}

int soft_blend_bwd(const PRBlendBwdArgs& a, hipStream_t st) {
  const PRBlendParams& p = a.p;
  if (p.N <= 0 || p.H <= 0 || p.W <= 0 || p.K <= 0) return set_error(PR_ERR_ARG, "soft blend: empty shape");
  if (!(p.flags & PR_BLEND_RAST) || !(p.flags & PR_BLEND_COLOR) || (p.flags & PR_BLEND_VERTEX))
    return set_error(PR_ERR_ARG, "soft blend: needs RAST | COLOR with texel colours");
  if (!a.dists || !a.zbuf || !a.colors || !a.pix_to_face || !a.grad_image || !a.grad_dists || !a.grad_zbuf ||
      !a.grad_colors || !a.grad_scalars || !p.znear || !p.zfar)
    return set_error(PR_ERR_ARG, "soft blend: missing buffer");
  if (!a.workspace || a.workspace_bytes < soft_blend_workspace(p))
    return set_error(PR_ERR_WORKSPACE, "soft blend: workspace too small");
  const int64_t P = (int64_t)p.N * p.H * p.W;
  const int nb = soft_bwd_blocks(p);
  float* part = reinterpret_cast<float*>(a.workspace);
  if (soft_lanes(p)) soft_bwd_lanes_kernel<<<nb, kThreads, 0, st>>>(a, P, p.H * p.W, part);
  else soft_bwd_kernel<<<nb, kThreads, 0, st>>>(a, P, p.H * p.W, part);
  if (int e = check_launch("soft_blend_bwd")) return e;
  soft_finalize_kernel<<<1, kThreads, 0, st>>>(part, nb, p, a.grad_scalars);
  return check_launch("soft_blend_finalize");
}

}  // namespace pr
