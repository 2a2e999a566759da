// Area-weighted vertex normals of a packed mesh (PyTorch3D Meshes.verts_normals_packed, the
// normals RandomPhongShader's phong_shading interpolates: eval.py's renderer, cfg 5), forward
// and backward.  Per face, each corner c adds cross(v_next - v_c, v_prev - v_c) to its vertex
// (PyTorch3D's three index_adds, same operand order), then every vertex row is normalised with
// F.normalize's max(||n||, 1e-6).  One launch per stage replaces ~20 small torch kernels
// (gathers, subtractions, crosses, index_adds, the norm) per direction.
#include "pr_common.h"

namespace pr {
namespace {

struct F3 {
  float x, y, z;
};
PR_DEV F3 sub(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PR_DEV F3 cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
PR_DEV F3 load3(const float* p, int64_t i) { return F3{p[i * 3], p[i * 3 + 1], p[i * 3 + 2]}; }
PR_DEV void add3(float* p, int64_t i, F3 v) {
  atomicAdd(p + i * 3, v.x);
  atomicAdd(p + i * 3 + 1, v.y);
  atomicAdd(p + i * 3 + 2, v.z);
}

// corner c of a face: (next, prev) corner indices as PyTorch3D's three crosses use them
//   corner 1: cross(v2 - v1, v0 - v1); corner 2: cross(v0 - v2, v1 - v2); corner 0: cross(v1 - v0, v2 - v0)
__global__ void face_cross_kernel(PRNormalsArgs a) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < a.F; f += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = a.faces[f * 3], i1 = a.faces[f * 3 + 1], i2 = a.faces[f * 3 + 2];
    const F3 v0 = load3(a.verts, i0), v1 = load3(a.verts, i1), v2 = load3(a.verts, i2);
    add3(a.normals, i1, cross(sub(v2, v1), sub(v0, v1)));
    add3(a.normals, i2, cross(sub(v0, v2), sub(v1, v2)));
    add3(a.normals, i0, cross(sub(v1, v0), sub(v2, v0)));
  }
}

PR_DEV float norm3(F3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }

// in place: n <- n / max(||n||, eps); the unnormalised sums are kept in `raw` for the backward
__global__ void normalize_kernel(PRNormalsArgs a) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.V; v += (int64_t)gridDim.x * blockDim.x) {
    const F3 n = load3(a.normals, v);
    if (a.raw) {
      a.raw[v * 3] = n.x; a.raw[v * 3 + 1] = n.y; a.raw[v * 3 + 2] = n.z;
    }
    const float d = fmaxf(norm3(n), 1e-6f);
    a.normals[v * 3] = n.x / d; a.normals[v * 3 + 1] = n.y / d; a.normals[v * 3 + 2] = n.z / d;
  }
}

// d raw from d normals: (g - y (y.g)) / ||x|| where ||x|| > eps, g / eps otherwise
__global__ void normalize_bwd_kernel(PRNormalsArgs a) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.V; v += (int64_t)gridDim.x * blockDim.x) {
    const F3 x = load3(a.raw, v), g = load3(a.grad_normals, v);
    const float nx = norm3(x);
    F3 r;
    if (nx > 1e-6f) {
      const F3 y{x.x / nx, x.y / nx, x.z / nx};
      const float yg = y.x * g.x + y.y * g.y + y.z * g.z;
      r = F3{(g.x - y.x * yg) / nx, (g.y - y.y * yg) / nx, (g.z - y.z * yg) / nx};
    } else {
      r = F3{g.x / 1e-6f, g.y / 1e-6f, g.z / 1e-6f};
    }
    a.grad_raw[v * 3] = r.x; a.grad_raw[v * 3 + 1] = r.y; a.grad_raw[v * 3 + 2] = r.z;
  }
}

// n = p x q with p = v_a - v_c, q = v_b - v_c:  dp = q x g, dq = g x p
PR_DEV void corner_bwd(float* gv, int64_t ic, int64_t ia, int64_t ib, F3 vc, F3 va, F3 vb, F3 g) {
  const F3 p = sub(va, vc), q = sub(vb, vc);
  const F3 dp = cross(q, g), dq = cross(g, p);
  add3(gv, ia, dp);
  add3(gv, ib, dq);
  add3(gv, ic, F3{-dp.x - dq.x, -dp.y - dq.y, -dp.z - dq.z});
}

__global__ void face_cross_bwd_kernel(PRNormalsArgs a) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < a.F; f += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = a.faces[f * 3], i1 = a.faces[f * 3 + 1], i2 = a.faces[f * 3 + 2];
    const F3 v0 = load3(a.verts, i0), v1 = load3(a.verts, i1), v2 = load3(a.verts, i2);
    corner_bwd(a.grad_verts, i1, i2, i0, v1, v2, v0, load3(a.grad_raw, i1));
    corner_bwd(a.grad_verts, i2, i0, i1, v2, v0, v1, load3(a.grad_raw, i2));
    corner_bwd(a.grad_verts, i0, i1, i2, v0, v1, v2, load3(a.grad_raw, i0));
  }
}

// ---- CSR form (vert_corner_start / vert_corners): one thread per vertex, its corners in
// PyTorch3D's index_add order (corner-1 entries by face, then corner 2, then corner 0), so the
// sums are sequential in that order; no atomics, no memset, deterministic.
PR_DEV F3 corner_cross(const PRNormalsArgs& a, int64_t t) {
  const int64_t f = t / 3;
  const int c = (int)(t - f * 3);
  const F3 v0 = load3(a.verts, a.faces[f * 3]), v1 = load3(a.verts, a.faces[f * 3 + 1]),
           v2 = load3(a.verts, a.faces[f * 3 + 2]);
  return c == 1 ? cross(sub(v2, v1), sub(v0, v1)) : (c == 2 ? cross(sub(v0, v2), sub(v1, v2)) : cross(sub(v1, v0), sub(v2, v0)));
}

__global__ void normals_gather_kernel(PRNormalsArgs a) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.V; v += (int64_t)gridDim.x * blockDim.x) {
    F3 n{0.f, 0.f, 0.f};
    for (int64_t j = a.vert_corner_start[v]; j < a.vert_corner_start[v + 1]; ++j) {
      const F3 c = corner_cross(a, a.vert_corners[j]);
      n.x += c.x; n.y += c.y; n.z += c.z;
    }
    if (a.raw) { a.raw[v * 3] = n.x; a.raw[v * 3 + 1] = n.y; a.raw[v * 3 + 2] = n.z; }
    const float d = fmaxf(norm3(n), 1e-6f);
    a.normals[v * 3] = n.x / d; a.normals[v * 3 + 1] = n.y / d; a.normals[v * 3 + 2] = n.z / d;
  }
}

// d verts of vertex v: for every face it is a corner of, the three corner crosses' partials
// with respect to v (dp = q x g, dq = g x p, and -dp - dq for the corner vertex itself)
__global__ void normals_bwd_gather_kernel(PRNormalsArgs a) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.V; v += (int64_t)gridDim.x * blockDim.x) {
    F3 acc{0.f, 0.f, 0.f};
    for (int64_t j = a.vert_corner_start[v]; j < a.vert_corner_start[v + 1]; ++j) {
      const int64_t t = a.vert_corners[j], f = t / 3;
      const int sv = (int)(t - f * 3);  // v's slot in face f
      const int64_t id[3] = {a.faces[f * 3], a.faces[f * 3 + 1], a.faces[f * 3 + 2]};
      const F3 vx[3] = {load3(a.verts, id[0]), load3(a.verts, id[1]), load3(a.verts, id[2])};
      // corners in face_cross_bwd_kernel's order: (c, a, b) = (1, 2, 0), (2, 0, 1), (0, 1, 2)
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int c = (r + 1) % 3, sa = (r + 2) % 3, sb = r;
        const F3 g = load3(a.grad_raw, id[c]);
        const F3 p = sub(vx[sa], vx[c]), q = sub(vx[sb], vx[c]);
        const F3 dp = cross(q, g), dq = cross(g, p);
        if (sv == sa) { acc.x += dp.x; acc.y += dp.y; acc.z += dp.z; }
        else if (sv == sb) { acc.x += dq.x; acc.y += dq.y; acc.z += dq.z; }
        else { acc.x += -dp.x - dq.x; acc.y += -dp.y - dq.y; acc.z += -dp.z - dq.z; }
      }
    }
    a.grad_verts[v * 3] = acc.x; a.grad_verts[v * 3 + 1] = acc.y; a.grad_verts[v * 3 + 2] = acc.z;
  }
}

int normals_check(const PRNormalsArgs* a) {
  if (!a || a->V < 0 || a->F < 0 || (a->F > 0 && (!a->verts || !a->faces)))
    return set_error(PR_ERR_ARG, "vert_normals: bad args");
  return PR_OK;
}

int blocks_for(int64_t n) { return (int)std::min<int64_t>((n + kThreads - 1) / kThreads, 4096); }

}  // namespace
}  // namespace pr

using namespace pr;

extern "C" int pr_vert_normals_fwd(const PRNormalsArgs* args, void* stream) {
  if (int e = normals_check(args)) return e;
  if (!args->normals) return set_error(PR_ERR_ARG, "vert_normals_fwd: normals missing");
  const PRNormalsArgs& a = *args;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.V == 0) return PR_OK;
  if (a.vert_corner_start && a.vert_corners) {
    normals_gather_kernel<<<blocks_for(a.V), kThreads, 0, st>>>(a);
    return check_launch("normals_gather");
  }
  if (hipMemsetAsync(a.normals, 0, (size_t)a.V * 3 * sizeof(float), st) != hipSuccess)
    return set_error(PR_ERR_HIP, "vert_normals_fwd: memset failed");
  if (a.F > 0) {
    face_cross_kernel<<<blocks_for(a.F), kThreads, 0, st>>>(a);
    if (int e = check_launch("face_cross")) return e;
  }
  normalize_kernel<<<blocks_for(a.V), kThreads, 0, st>>>(a);
  return check_launch("normalize");
}

extern "C" int pr_vert_normals_bwd(const PRNormalsArgs* args, void* stream) {
  if (int e = normals_check(args)) return e;
  const PRNormalsArgs& a = *args;
  if (!a.raw || !a.grad_normals || !a.grad_raw || !a.grad_verts)
    return set_error(PR_ERR_ARG, "vert_normals_bwd: buffers missing");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.V == 0) return PR_OK;
  const bool csr = a.vert_corner_start && a.vert_corners;
  if (!csr && hipMemsetAsync(a.grad_verts, 0, (size_t)a.V * 3 * sizeof(float), st) != hipSuccess)
    return set_error(PR_ERR_HIP, "vert_normals_bwd: memset failed");
  normalize_bwd_kernel<<<blocks_for(a.V), kThreads, 0, st>>>(a);
  if (int e = check_launch("normalize_bwd")) return e;
  if (csr) {
    normals_bwd_gather_kernel<<<blocks_for(a.V), kThreads, 0, st>>>(a);
    return check_launch("normals_bwd_gather");
  }
  if (a.F > 0) {
    face_cross_bwd_kernel<<<blocks_for(a.F), kThreads, 0, st>>>(a);
    if (int e = check_launch("face_cross_bwd")) return e;
  }
  return PR_OK;
}
