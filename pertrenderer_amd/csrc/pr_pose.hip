// Pose ops of the pose-optimisation loop: SO(3) exponential map and the row-vector
// rotation of a point set, forward and backward (PyTorch3D 0.4.0 so3_exponential_map
// and Rotate.transform_points as used at experiments/eval.py:343-346).
//
// They are tiny (one 3-vector, a few thousand points), so the point of a native op
// is launch count: the torch composition is ~60 kernels per fwd+bwd step (hat
// assembly, bmm, elementwise, their autograd), each a separate graph node.  Here it
// is one kernel per direction; the R-gradient reduction is a fixed-order block
// reduction (deterministic).
#include "pr_common.h"

namespace pr {
namespace {

PR_DEV void hat3(const float w[3], float S[9]) {
  S[0] = 0.f;   S[1] = -w[2]; S[2] = w[1];
  S[3] = w[2];  S[4] = 0.f;   S[5] = -w[0];
  S[6] = -w[1]; S[7] = w[0];  S[8] = 0.f;
}

PR_DEV void mm3(const float A[9], const float B[9], float C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C[i * 3 + j] = (A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j]) + A[i * 3 + 2] * B[6 + j];
}

struct SO3Fac {
  float nrms, angle, inv, sn, cs, fac1, fac2;
};

PR_DEV SO3Fac so3_fac(const float w[3], float eps) {
  SO3Fac f;
  f.nrms = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
  f.angle = sqrtf(f.nrms > eps ? f.nrms : eps);
  f.inv = 1.f / f.angle;
  f.sn = sinf(f.angle);
  f.cs = cosf(f.angle);
  f.fac1 = f.inv * f.sn;
  f.fac2 = f.inv * f.inv * (1.f - f.cs);
  return f;
}

__global__ void so3_exp_fwd_kernel(PRSO3Args a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= a.N) return;
  const float w[3] = {a.log_rot[n * 3], a.log_rot[n * 3 + 1], a.log_rot[n * 3 + 2]};
  const SO3Fac f = so3_fac(w, a.eps);
  float S[9], S2[9];
  hat3(w, S);
  mm3(S, S, S2);
#pragma unroll
  for (int i = 0; i < 9; ++i) a.R[n * 9 + i] = (f.fac1 * S[i] + f.fac2 * S2[i]) + ((i % 4) == 0 ? 1.f : 0.f);
}

// autograd of the forward expression, term by term
__global__ void so3_exp_bwd_kernel(PRSO3Args a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= a.N) return;
  const float w[3] = {a.log_rot[n * 3], a.log_rot[n * 3 + 1], a.log_rot[n * 3 + 2]};
  const SO3Fac f = so3_fac(w, a.eps);
  float S[9], S2[9], G[9];
  hat3(w, S);
  mm3(S, S, S2);
  for (int i = 0; i < 9; ++i) G[i] = a.grad_R[n * 9 + i];
  float dfac1 = 0.f, dfac2 = 0.f;
  for (int i = 0; i < 9; ++i) { dfac1 += G[i] * S[i]; dfac2 += G[i] * S2[i]; }
  // S2 = S @ S: dS = G2 S^T + S^T G2 with G2 = fac2 * G
  float G2[9], St[9], A[9], B[9], dS[9];
  for (int i = 0; i < 9; ++i) G2[i] = f.fac2 * G[i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) St[i * 3 + j] = S[j * 3 + i];
  mm3(G2, St, A);
  mm3(St, G2, B);
  for (int i = 0; i < 9; ++i) dS[i] = f.fac1 * G[i] + (A[i] + B[i]);
  const float dinv = dfac1 * f.sn + dfac2 * (2.f * f.inv * (1.f - f.cs));
  const float dang = dfac1 * f.inv * f.cs + dfac2 * f.inv * f.inv * f.sn - dinv * f.inv * f.inv;
  const float dc = dang * 0.5f / f.angle;
  const float dn = f.nrms >= a.eps ? dc : 0.f;  // clamp(min=eps) passes the gradient where nrms >= eps
  a.grad_log_rot[n * 3 + 0] = 2.f * w[0] * dn + (dS[7] - dS[5]);
  a.grad_log_rot[n * 3 + 1] = 2.f * w[1] * dn + (dS[2] - dS[6]);
  a.grad_log_rot[n * 3 + 2] = 2.f * w[2] * dn + (dS[3] - dS[1]);
}

__global__ void __launch_bounds__(kThreads) rotate_fwd_kernel(PRRotateArgs a) {
  const int64_t total = (int64_t)a.N * a.P;
  for (int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x; t < total; t += (int64_t)gridDim.x * kThreads) {
    const int n = (int)(t / a.P);
    const float* R = a.R + (a.R_batched ? n * 9 : 0);
    const float x = a.points[t * 3], y = a.points[t * 3 + 1], z = a.points[t * 3 + 2];
#pragma unroll
    for (int j = 0; j < 3; ++j) a.out[t * 3 + j] = (x * R[j] + y * R[3 + j]) + z * R[6 + j];
  }
}

// One workgroup per R (per batch if R_batched, else one for all): d R = sum_p p^T g,
// reduced in a fixed order (per lane, then a wave butterfly, then the waves in order);
// d points = g @ R^T alongside.
__global__ void __launch_bounds__(kThreads) rotate_bwd_kernel(PRRotateArgs a) {
  __shared__ float red[kThreads / 64][9];
  const int tid = threadIdx.x;
  const int r = blockIdx.x;
  const int n0 = a.R_batched ? r : 0, n1 = a.R_batched ? r + 1 : a.N;
  const float* R = a.R + (a.R_batched ? r * 9 : 0);
  float acc[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t lo = (int64_t)n0 * a.P, hi = (int64_t)n1 * a.P;
  for (int64_t t = lo + tid; t < hi; t += kThreads) {
    const float x = a.points[t * 3], y = a.points[t * 3 + 1], z = a.points[t * 3 + 2];
    const float g0 = a.grad_out[t * 3], g1 = a.grad_out[t * 3 + 1], g2 = a.grad_out[t * 3 + 2];
    if (a.grad_R) {
      acc[0] += x * g0; acc[1] += x * g1; acc[2] += x * g2;
      acc[3] += y * g0; acc[4] += y * g1; acc[5] += y * g2;
      acc[6] += z * g0; acc[7] += z * g1; acc[8] += z * g2;
    }
    if (a.grad_points) {
#pragma unroll
      for (int i = 0; i < 3; ++i) a.grad_points[t * 3 + i] = (g0 * R[i * 3] + g1 * R[i * 3 + 1]) + g2 * R[i * 3 + 2];
    }
  }
  if (!a.grad_R) return;
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) acc[i] += __shfl_xor(acc[i], m);
  if ((tid & 63) == 0)
#pragma unroll
    for (int i = 0; i < 9; ++i) red[tid >> 6][i] = acc[i];
  __syncthreads();
  if (tid < 9) {
    float v = red[0][tid];
    for (int w = 1; w < kThreads / 64; ++w) v += red[w][tid];
    a.grad_R[r * 9 + tid] = v;
  }
}

// One optimize_pose iteration's bookkeeping (pr_pose_step, PRPoseStepArgs): the loss and
// gradient-norm records, the best-loss pose, eval.py's grad-norm guard, the accumulation of the
// smoothing gradients and (post) their EMA and reset, the iteration counter.  A captured step otherwise spends
// ~20 one-element torch kernels on it (index_copy, where, norm, randn, mul, add, fill, copy).
__global__ void pose_step_kernel(PRPoseStepArgs a) {
  if (threadIdx.x != 0) return;
  const int64_t t = *a.it;
  if (t < 0 || t >= a.niter) return;  // past the records (the host sizes them): nothing written
  const float loss = *a.loss;
  a.losses[t] = loss;
  if (loss < *a.best_loss) {  // eval.py:372-374 (the pose that produced this loss, before the step)
    *a.best_loss = loss;
    for (int i = 0; i < a.n; ++i) a.best[i] = a.log_rot[i];
  }
  float ss = 0.f;
  for (int i = 0; i < a.n; ++i) ss += a.grad[i] * a.grad[i];
  const float gn = sqrtf(ss);
  a.gnorms[t] = gn;
  if (gn > 1000.f) {  // eval.py:375-379: grad = 1e-5 * normal (Philox draws keyed by the seed, t)
    const uint64_t key = (a.seed ? a.seed[0] : 0ull) ^ 0x67756172645f706full;
    for (int i = 0; i < a.n; i += 4) {
      const U4 u = philox4x32_10(U4{(uint32_t)t, (uint32_t)(t >> 32), (uint32_t)i, 0x706f7365u}, (uint32_t)key,
                                 (uint32_t)(key >> 32));
      float e[4];
      gauss4(u, e);
      for (int j = 0; j < 4 && i + j < a.n; ++j) a.grad[i + j] = 1e-5f * e[j];
    }
  }
  for (int i = 0; i < 3; ++i) {  // eval.py:382-385: the leaves' .grad accumulates until the EMA reads it
    if (!a.acc) break;
    float g = a.acc[i];
    if (a.leaf_grad[i]) g += *a.leaf_grad[i];
    if (a.post) {
      a.v[i] = 0.9f * a.v[i] + 0.1f * g;
      g = 0.f;
    }
    a.acc[i] = g;
  }
  if (a.adam) {  // torch.optim.Adam's fused step: its adam_math (double hyper-parameters, float state)
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
    const float step = *a.step + 1.f;
    *a.step = step;
    const double bc1 = 1.0 - pow(b1, (double)step), bc2 = 1.0 - pow(b2, (double)step);
    const double step_size = (double)*a.lr / bc1, bc2_sqrt = sqrt(bc2);
    for (int i = 0; i < a.n; ++i) {
      const float g = a.grad[i];
      const float m = (float)(b1 * a.exp_avg[i] + (1 - b1) * g);
      const float s = (float)(b2 * a.exp_avg_sq[i] + (1 - b2) * g * g);
      a.exp_avg[i] = m;
      a.exp_avg_sq[i] = s;
      const double denom = sqrtf(s) / bc2_sqrt + eps;
      a.log_rot[i] = (float)(a.log_rot[i] - step_size * m / denom);
    }
  }
  *a.it = t + 1;
}

// eval.py's RGB loss: per-workgroup partial sums in a fixed order, then one workgroup sums the
// partials in block order (deterministic); the backward is one elementwise pass
constexpr int kMseBlocks = 512;
PR_DEV int64_t mse_tidx(const PRRgbMseArgs& a, int64_t p) { return a.target_batched ? p : p % a.HW; }

__global__ void __launch_bounds__(kThreads) rgb_mse_partial_kernel(PRRgbMseArgs a) {
  __shared__ float red[kThreads / 64];
  float acc = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < a.P; p += (int64_t)gridDim.x * kThreads) {
    const float* im = a.image + p * a.C;
    const float* t = a.target + mse_tidx(a, p) * 3;
    const float d0 = im[0] - t[0], d1 = im[1] - t[1], d2 = im[2] - t[2];
    acc += (d0 * d0 + d1 * d1) + d2 * d2;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
    a.partials[blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(kThreads) rgb_mse_finalize_kernel(PRRgbMseArgs a, int nblk) {
  __shared__ float red[kThreads / 64];
  float acc = 0.f;
  for (int b = threadIdx.x; b < nblk; b += kThreads) acc += a.partials[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
    *a.loss = s / (float)(a.P * 3);
  }
}

__global__ void __launch_bounds__(kThreads) rgb_mse_bwd_kernel(PRRgbMseArgs a) {
  const float g = *a.grad_loss / (float)(a.P * 3);
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < a.P; p += (int64_t)gridDim.x * kThreads) {
    const float* im = a.image + p * a.C;
    const float* t = a.target + mse_tidx(a, p) * 3;
    float* o = a.grad_image + p * a.C;
    o[0] = g * (2.f * (im[0] - t[0]));
    o[1] = g * (2.f * (im[1] - t[1]));
    o[2] = g * (2.f * (im[2] - t[2]));
    for (int c = 3; c < a.C; ++c) o[c] = 0.f;
  }
}

int mse_blocks(int64_t P) { return (int)std::max<int64_t>(1, std::min<int64_t>((P + kThreads - 1) / kThreads, kMseBlocks)); }

int mse_check(const PRRgbMseArgs* a) {
  if (!a || a->P <= 0 || a->C < 3 || !a->image || !a->target || (!a->target_batched && (a->HW <= 0 || a->P % a->HW)))
    return set_error(PR_ERR_ARG, "rgb_mse: bad args");
  return PR_OK;
}

}  // namespace
}  // namespace pr

using namespace pr;

extern "C" size_t pr_rgb_mse_workspace(int64_t P) { return P > 0 ? (size_t)mse_blocks(P) : 1; }

extern "C" int pr_rgb_mse_fwd(const PRRgbMseArgs* a, void* stream) {
  if (int e = mse_check(a)) return e;
  if (!a->loss || !a->partials) return set_error(PR_ERR_ARG, "rgb_mse_fwd: loss / workspace missing");
  const int nb = mse_blocks(a->P);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  rgb_mse_partial_kernel<<<nb, kThreads, 0, st>>>(*a);
  if (int e = check_launch("rgb_mse_partial")) return e;
  rgb_mse_finalize_kernel<<<1, kThreads, 0, st>>>(*a, nb);
  return check_launch("rgb_mse_finalize");
}

extern "C" int pr_rgb_mse_bwd(const PRRgbMseArgs* a, void* stream) {
  if (int e = mse_check(a)) return e;
  if (!a->grad_loss || !a->grad_image) return set_error(PR_ERR_ARG, "rgb_mse_bwd: grads missing");
  rgb_mse_bwd_kernel<<<(int)std::min<int64_t>((a->P + kThreads - 1) / kThreads, 4096), kThreads, 0,
                       reinterpret_cast<hipStream_t>(stream)>>>(*a);
  return check_launch("rgb_mse_bwd");
}

extern "C" int pr_pose_step(const PRPoseStepArgs* a, void* stream) {
  if (!a || !a->loss || !a->log_rot || !a->grad || !a->it || !a->losses || !a->gnorms || !a->best_loss || !a->best ||
      a->n <= 0 || a->n > 64 || a->niter <= 0 || (a->post && (!a->v || !a->acc)) ||
      (a->adam && (!a->exp_avg || !a->exp_avg_sq || !a->step || !a->lr)))
    return set_error(PR_ERR_ARG, "pose_step: bad args");
  pose_step_kernel<<<1, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(*a);
  return check_launch("pose_step");
}

extern "C" int pr_so3_exp_fwd(const PRSO3Args* a, void* stream) {
  if (!a || a->N < 0 || (a->N > 0 && (!a->log_rot || !a->R))) return set_error(PR_ERR_ARG, "so3_exp_fwd: bad args");
  if (a->N == 0) return PR_OK;
  so3_exp_fwd_kernel<<<(a->N + 63) / 64, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(*a);
  return check_launch("so3_exp_fwd");
}

extern "C" int pr_so3_exp_bwd(const PRSO3Args* a, void* stream) {
  if (!a || a->N < 0 || (a->N > 0 && (!a->log_rot || !a->grad_R || !a->grad_log_rot)))
    return set_error(PR_ERR_ARG, "so3_exp_bwd: bad args");
  if (a->N == 0) return PR_OK;
  so3_exp_bwd_kernel<<<(a->N + 63) / 64, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(*a);
  return check_launch("so3_exp_bwd");
}

extern "C" int pr_rotate_fwd(const PRRotateArgs* a, void* stream) {
  if (!a || a->N < 0 || a->P < 0 || !a->R || ((int64_t)a->N * a->P > 0 && (!a->points || !a->out)))
    return set_error(PR_ERR_ARG, "rotate_fwd: bad args");
  const int64_t total = (int64_t)a->N * a->P;
  if (total == 0) return PR_OK;
  const int nb = (int)std::min<int64_t>((total + kThreads - 1) / kThreads, 4096);
  rotate_fwd_kernel<<<nb, kThreads, 0, reinterpret_cast<hipStream_t>(stream)>>>(*a);
  return check_launch("rotate_fwd");
}

extern "C" int pr_rotate_bwd(const PRRotateArgs* a, void* stream) {
  if (!a || a->N <= 0 || a->P < 0 || !a->R || !a->points || !a->grad_out) return set_error(PR_ERR_ARG, "rotate_bwd: bad args");
  if (!a->grad_R && !a->grad_points) return PR_OK;
  rotate_bwd_kernel<<<a->R_batched ? a->N : 1, kThreads, 0, reinterpret_cast<hipStream_t>(stream)>>>(*a);
  return check_launch("rotate_bwd");
}
