// Phong shading of fragment slots (PyTorch3D 0.4.0 phong_shading + the texel lookup of
// Meshes.sample_textures): the colour producer of RandomPhongShader (random_rasterizer.py:99-110,
// experiments/eval.py:170).  One thread per (pixel, slot); the valid-prefix counts let the
// backward skip padded slots without reading them.
//
// Forward: one pass, writes the (N,H,W,K,3) colours (39 MB at 256^2, K=50) in place of the
// ~60 elementwise torch kernels of the reference composition, each a (N,H,W,K,3) round trip.
// Backward: per-slot chain rule in registers; the per-vertex / per-batch gradients (verts,
// normals, vertex colours, light, camera) are reduced in LDS per workgroup and flushed with
// one global atomic per touched entry (meshes have few vertices -- the cube has 8 -- so
// per-slot global atomics would serialise on a handful of addresses).
#include "pr_common.h"

namespace pr {
namespace {

constexpr float kNormEps = 1e-6f;  // F.normalize(eps=1e-6)
constexpr int kLdsFloats = 8192;   // 32 KB reduction table per workgroup

struct V3 {
  float x, y, z;
};
PR_DEV V3 v3(const float* p) { return V3{p[0], p[1], p[2]}; }
PR_DEV V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PR_DEV V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PR_DEV V3 operator*(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
PR_DEV V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
PR_DEV float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
PR_DEV float sum3(V3 a) { return (a.x + a.y) + a.z; }

// x / max(|x|, eps) and its backward
PR_DEV float nrm(V3 x) { return fmaxf(sqrtf(dot(x, x)), kNormEps); }
PR_DEV V3 normalize(V3 x) {
  const float r = nrm(x);
  return V3{x.x / r, x.y / r, x.z / r};
}
PR_DEV V3 normalize_bwd(V3 x, V3 g) {
  const float r = sqrtf(dot(x, x));
  if (!(r > kNormEps)) return (1.f / kNormEps) * g;
  const V3 y = V3{x.x / r, x.y / r, x.z / r};
  return (1.f / r) * (g - dot(y, g) * y);
}

// (w0 r0 + w1 r1) + w2 r2 over a per-vertex table (interpolate_face_attributes order)
PR_DEV V3 interp3(const float* tab, const int64_t* fv, const float* b) {
  const float* r0 = tab + fv[0] * 3;
  const float* r1 = tab + fv[1] * 3;
  const float* r2 = tab + fv[2] * 3;
  return V3{(b[0] * r0[0] + b[1] * r1[0]) + b[2] * r2[0], (b[0] * r0[1] + b[1] * r1[1]) + b[2] * r2[1],
            (b[0] * r0[2] + b[1] * r1[2]) + b[2] * r2[2]};
}

// torch grid_sample, bilinear, align_corners=True, padding "border", on the vertically
// flipped map (v = 0 is the bottom row): source coordinate in the flipped map and the
// clip gradient (0 where the coordinate was clamped, as clip_coordinates_set_grad)
struct Bilin {
  int x0, y0;      // north-west corner in the flipped map
  float ix, iy;    // source coordinates
  float gx, gy;    // d ix / d u, d iy / d v (0 when clamped)
};
PR_DEV float src_coord(float uv, int size, float& grad) {
  const float g = uv * 2.f - 1.f;  // TexturesUV: uv * 2 - 1
  float c = ((g + 1.f) / 2.f) * (float)(size - 1);
  grad = (float)(size - 1);
  if (c <= 0.f) { c = 0.f; grad = 0.f; }
  else if (c >= (float)(size - 1)) { c = (float)(size - 1); grad = 0.f; }
  return c;
}
PR_DEV Bilin bilin(float u, float v, int Hm, int Wm) {
  Bilin b;
  b.ix = src_coord(u, Wm, b.gx);
  b.iy = src_coord(v, Hm, b.gy);
  b.x0 = (int)floorf(b.ix);
  b.y0 = (int)floorf(b.iy);
  return b;
}
// texel (flipped row r -> map row Hm-1-r) with torch's corner order nw, ne, sw, se
PR_DEV V3 bilin_sample(const float* map, int Hm, int Wm, const Bilin& b) {
  const float x1 = (float)(b.x0 + 1), y1 = (float)(b.y0 + 1), x0 = (float)b.x0, y0 = (float)b.y0;
  const float w[4] = {(x1 - b.ix) * (y1 - b.iy), (b.ix - x0) * (y1 - b.iy), (x1 - b.ix) * (b.iy - y0),
                      (b.ix - x0) * (b.iy - y0)};
  const int cx[4] = {b.x0, b.x0 + 1, b.x0, b.x0 + 1}, cy[4] = {b.y0, b.y0, b.y0 + 1, b.y0 + 1};
  V3 o{0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (cx[c] >= 0 && cx[c] < Wm && cy[c] >= 0 && cy[c] < Hm) {
      const float* t = map + ((int64_t)(Hm - 1 - cy[c]) * Wm + cx[c]) * 3;
      o = o + w[c] * v3(t);
    }
  }
  return o;
}

struct Slot {
  int64_t f;
  int n;
  float b[3];
};

PR_DEV Slot load_slot(const PRShadeArgs& a, int64_t s, int64_t HW) {
  Slot sl;
  const int64_t p = s / a.K;
  const int k = (int)(s - p * a.K);
  sl.n = (int)(p / HW);
  const bool valid = a.pix_count ? k < a.pix_count[p] : true;
  sl.f = valid ? a.pix_to_face[s] : -1;
  if (sl.f >= 0) {
    sl.b[0] = a.bary[s * 3]; sl.b[1] = a.bary[s * 3 + 1]; sl.b[2] = a.bary[s * 3 + 2];
  } else {
    sl.b[0] = sl.b[1] = sl.b[2] = 0.f;
  }
  return sl;
}

// everything the colour depends on, recomputed identically by the backward
struct Shade {
  V3 P, Nn, uvw;     // interpolated position, normal, (u, v, -)
  V3 tex;            // texel
  V3 dir, dh, nh;    // light direction (raw, normalized), normal (normalized)
  float cosang;
  V3 vraw, view, refl;
  float dotvr, alpha, mask;
  Bilin bl;
};

PR_DEV Shade shade(const PRShadeArgs& a, const Slot& sl, int64_t s, const int64_t* fv) {
  Shade z;
  const V3 zero{0.f, 0.f, 0.f};
  z.P = sl.f >= 0 ? interp3(a.verts, fv, sl.b) : zero;
  z.Nn = sl.f >= 0 ? interp3(a.normals, fv, sl.b) : zero;
  z.uvw = zero;
  if (a.texture == PR_TEX_GIVEN) {
    z.tex = v3(a.texels + s * 3);
  } else if (a.texture == PR_TEX_VERTEX) {
    z.tex = sl.f >= 0 ? interp3(a.vert_colors, fv, sl.b) : zero;
  } else {
    if (sl.f >= 0) {
      const float* q = a.face_uvs + sl.f * 6;
      z.uvw.x = (sl.b[0] * q[0] + sl.b[1] * q[2]) + sl.b[2] * q[4];
      z.uvw.y = (sl.b[0] * q[1] + sl.b[1] * q[3]) + sl.b[2] * q[5];
    }
    z.bl = bilin(z.uvw.x, z.uvw.y, a.Hm, a.Wm);
    z.tex = bilin_sample(a.maps + (int64_t)sl.n * a.Hm * a.Wm * 3, a.Hm, a.Wm, z.bl);
  }
  const V3 L = v3(a.light + sl.n * 3);
  z.dir = a.directional ? L : L - z.P;
  z.dh = normalize(z.dir);
  z.nh = normalize(z.Nn);
  z.cosang = dot(z.nh, z.dh);
  z.vraw = v3(a.camera + sl.n * 3) - z.P;
  z.view = normalize(z.vraw);
  z.refl = V3{-z.dh.x + 2.f * (z.cosang * z.nh.x), -z.dh.y + 2.f * (z.cosang * z.nh.y),
              -z.dh.z + 2.f * (z.cosang * z.nh.z)};
  z.mask = z.cosang > 0.f ? 1.f : 0.f;
  z.dotvr = dot(z.view, z.refl);
  z.alpha = fmaxf(z.dotvr, 0.f) * z.mask;
  return z;
}

__global__ void __launch_bounds__(kThreads) shade_fwd_kernel(PRShadeArgs a, int64_t PK, int64_t HW) {
  for (int64_t s = (int64_t)blockIdx.x * kThreads + threadIdx.x; s < PK; s += (int64_t)gridDim.x * kThreads) {
    const Slot sl = load_slot(a, s, HW);
    const int64_t fz[3] = {0, 0, 0};
    const int64_t* fv = sl.f >= 0 ? a.faces + sl.f * 3 : fz;
    const Shade z = shade(a, sl, s, fv);
    const int n = sl.n;
    const float angle = fmaxf(z.cosang, 0.f);
    const V3 dl = angle * v3(a.diffuse_color + n * 3);
    const float pw = powf(z.alpha, a.shininess[n]);
    const V3 sp = pw * v3(a.specular_color + n * 3);
    const V3 lit = v3(a.ambient + n * 3) + v3(a.mat_diffuse + n * 3) * dl;
    const V3 c = lit * z.tex + v3(a.mat_specular + n * 3) * sp;
    float* o = a.colors + s * 3;
    o[0] = c.x; o[1] = c.y; o[2] = c.z;
  }
}

// LDS reduction table: [verts V*3][normals V*3][vert colors V*3][light N*3][camera N*3]
struct Tab {
  int vOff, nOff, cOff, lOff, camOff, size;
  bool useV, useB;  // per-vertex / per-batch entries reduced in LDS (else global atomics)
};

PR_DEV void acc(float* lds, bool use_lds, int off, float* global, int64_t gi, V3 g) {
  if (use_lds) {
    atomicAdd(&lds[off + 0], g.x); atomicAdd(&lds[off + 1], g.y); atomicAdd(&lds[off + 2], g.z);
  } else if (global) {
    atomicAdd(&global[gi * 3 + 0], g.x); atomicAdd(&global[gi * 3 + 1], g.y); atomicAdd(&global[gi * 3 + 2], g.z);
  }
}

// PR_DETERMINISTIC: instead of scattering, every slot writes its contributions as entries of
// three ordered scatter-adds (pr_detsum.hip): per-vertex (slot corner i: verts | normals |
// vertex colours, 9 components), per-batch (light | camera, 6) and per-texel (bilinear corner,
// 3); padded slots write dropped keys.
struct ShadeDet {
  DetSum v, b, m;  // n == 0: not requested
};

PR_DEV void put3(float* p, V3 g) { p[0] = g.x; p[1] = g.y; p[2] = g.z; }

// (slots [s0, PK): the deterministic mode runs the frame in batches; the fast path s0 = 0)
template <bool DET>
__global__ void __launch_bounds__(kThreads) shade_bwd_kernel(PRShadeArgs a, int64_t s0, int64_t PK, int64_t HW,
                                                             Tab tab, ShadeDet det) {
  extern __shared__ float lds[];
  if (!DET) {
    for (int i = threadIdx.x; i < tab.size; i += kThreads) lds[i] = 0.f;
    __syncthreads();
  }
  for (int64_t s = s0 + (int64_t)blockIdx.x * kThreads + threadIdx.x; s < PK; s += (int64_t)gridDim.x * kThreads) {
    const int64_t ds = s - s0;  // entry row of this batch (PR_DETERMINISTIC)
    (void)ds;
    const Slot sl = load_slot(a, s, HW);
    const int n = sl.n;
    const V3 gc = v3(a.grad_colors + s * 3);
    if (sl.f < 0) {
      // padded slot: only the texel term can carry a gradient (p = n = 0: no light, no specular)
      if (a.grad_bary) { a.grad_bary[s * 3] = 0.f; a.grad_bary[s * 3 + 1] = 0.f; a.grad_bary[s * 3 + 2] = 0.f; }
      if (a.texture == PR_TEX_GIVEN && a.grad_texels) {
        const V3 g = v3(a.ambient + n * 3) * gc;
        float* o = a.grad_texels + s * 3;
        o[0] = g.x; o[1] = g.y; o[2] = g.z;
      }
      if (DET) {
        if (det.v.n)
          for (int i = 0; i < 3; ++i) det.v.keys[ds * 3 + i] = (uint32_t)det.v.M;
        if (det.b.n) det.b.keys[ds] = (uint32_t)det.b.M;
        if (det.m.n)
          for (int c = 0; c < 4; ++c) det.m.keys[ds * 4 + c] = (uint32_t)det.m.M;
      }
      continue;
    }
    const int64_t* fv = a.faces + sl.f * 3;
    const Shade z = shade(a, sl, s, fv);
    const float angle = fmaxf(z.cosang, 0.f);
    const V3 dcol = v3(a.diffuse_color + n * 3), scol = v3(a.specular_color + n * 3);
    const V3 mdif = v3(a.mat_diffuse + n * 3), mspec = v3(a.mat_specular + n * 3);
    const V3 lit = v3(a.ambient + n * 3) + mdif * (angle * dcol);
    // colour = lit * tex + mspec * (pow(alpha, sh) * scol)
    const V3 g_tex = lit * gc;
    const float g_angle = dot(dcol, mdif * z.tex * gc);
    const float g_pow = dot(scol, mspec * gc);
    const float sh = a.shininess[n];
    const float g_alpha = z.alpha > 0.f ? g_pow * sh * powf(z.alpha, sh - 1.f) : 0.f;
    const float g_dotvr = z.dotvr > 0.f ? g_alpha * z.mask : 0.f;
    const V3 g_view = g_dotvr * z.refl, g_refl = g_dotvr * z.view;
    // refl = -dh + 2 c nh
    V3 g_dh = V3{0.f, 0.f, 0.f} - g_refl;
    float g_cos = 2.f * dot(g_refl, z.nh) + (z.cosang > 0.f ? g_angle : 0.f);
    V3 g_nh = (2.f * z.cosang) * g_refl;
    // c = nh . dh
    g_nh = g_nh + g_cos * z.dh;
    g_dh = g_dh + g_cos * z.nh;
    const V3 g_vraw = normalize_bwd(z.vraw, g_view);
    const V3 g_dir = normalize_bwd(z.dir, g_dh);
    const V3 g_Nn = normalize_bwd(z.Nn, g_nh);
    V3 g_P = V3{0.f, 0.f, 0.f} - g_vraw;
    if (!a.directional) g_P = g_P - g_dir;
    // interpolations: d bary and per-vertex scatters
    float gb[3];
    const float* b = sl.b;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int64_t vi = fv[i];
      gb[i] = dot(g_P, v3(a.verts + vi * 3)) + dot(g_Nn, v3(a.normals + vi * 3));
      if (DET) {
        if (det.v.n) {
          det.v.keys[ds * 3 + i] = (uint32_t)vi;
          float* e = det.v.vals + (ds * 3 + i) * 9;
          put3(e, b[i] * g_P);
          put3(e + 3, b[i] * g_Nn);
          put3(e + 6, V3{0.f, 0.f, 0.f});
        }
        continue;
      }
      if (a.grad_verts) acc(lds, tab.useV, tab.vOff + (int)vi * 3, a.grad_verts, vi, b[i] * g_P);
      if (a.grad_normals) acc(lds, tab.useV, tab.nOff + (int)vi * 3, a.grad_normals, vi, b[i] * g_Nn);
    }
    if (a.texture == PR_TEX_GIVEN) {
      if (a.grad_texels) {
        float* o = a.grad_texels + s * 3;
        o[0] = g_tex.x; o[1] = g_tex.y; o[2] = g_tex.z;
      }
    } else if (a.texture == PR_TEX_VERTEX) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int64_t vi = fv[i];
        gb[i] += dot(g_tex, v3(a.vert_colors + vi * 3));
        if (DET) {
          if (det.v.n) put3(det.v.vals + (ds * 3 + i) * 9 + 6, b[i] * g_tex);
          continue;
        }
        if (a.grad_vert_colors) acc(lds, tab.useV, tab.cOff + (int)vi * 3, a.grad_vert_colors, vi, b[i] * g_tex);
      }
    } else {
      // bilinear backward: d texel / d (ix, iy) from the four corners, then d (u, v)
      const Bilin& bl = z.bl;
      const float* map = a.maps + (int64_t)n * a.Hm * a.Wm * 3;
      const float x0 = (float)bl.x0, y0 = (float)bl.y0, x1 = x0 + 1.f, y1 = y0 + 1.f;
      const int cx[4] = {bl.x0, bl.x0 + 1, bl.x0, bl.x0 + 1}, cy[4] = {bl.y0, bl.y0, bl.y0 + 1, bl.y0 + 1};
      const float dwx[4] = {-(y1 - bl.iy), (y1 - bl.iy), -(bl.iy - y0), (bl.iy - y0)};
      const float dwy[4] = {-(x1 - bl.ix), -(bl.ix - x0), (x1 - bl.ix), (bl.ix - x0)};
      const float w[4] = {(x1 - bl.ix) * (y1 - bl.iy), (bl.ix - x0) * (y1 - bl.iy), (x1 - bl.ix) * (bl.iy - y0),
                          (bl.ix - x0) * (bl.iy - y0)};
      float gix = 0.f, giy = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bool in = cx[c] >= 0 && cx[c] < a.Wm && cy[c] >= 0 && cy[c] < a.Hm;
        if (DET && det.m.n) {
          det.m.keys[ds * 4 + c] = in ? (uint32_t)(((int64_t)n * a.Hm + (a.Hm - 1 - cy[c])) * a.Wm + cx[c])
                                     : (uint32_t)det.m.M;
          if (in) put3(det.m.vals + (ds * 4 + c) * 3, w[c] * g_tex);
        }
        if (in) {
          const int64_t ti = ((int64_t)(a.Hm - 1 - cy[c]) * a.Wm + cx[c]) * 3;
          const float gv = dot(v3(map + ti), g_tex);
          gix += dwx[c] * gv;
          giy += dwy[c] * gv;
          if (!DET && a.grad_maps) {
            float* gm = a.grad_maps + (int64_t)n * a.Hm * a.Wm * 3 + ti;
            atomicAdd(&gm[0], w[c] * g_tex.x); atomicAdd(&gm[1], w[c] * g_tex.y); atomicAdd(&gm[2], w[c] * g_tex.z);
          }
        }
      }
      const float gu = gix * bl.gx, gvv = giy * bl.gy;
      const float* q = a.face_uvs + sl.f * 6;
#pragma unroll
      for (int i = 0; i < 3; ++i) gb[i] += gu * q[2 * i] + gvv * q[2 * i + 1];
    }
    if (a.grad_bary) { a.grad_bary[s * 3] = gb[0]; a.grad_bary[s * 3 + 1] = gb[1]; a.grad_bary[s * 3 + 2] = gb[2]; }
    if (DET) {
      if (det.b.n) {
        det.b.keys[ds] = (uint32_t)n;
        put3(det.b.vals + ds * 6, g_dir);
        put3(det.b.vals + ds * 6 + 3, g_vraw);
      }
      continue;
    }
    if (a.grad_light) acc(lds, tab.useB, tab.lOff + n * 3, a.grad_light, n, g_dir);
    if (a.grad_camera) acc(lds, tab.useB, tab.camOff + n * 3, a.grad_camera, n, g_vraw);
  }
  if (DET) return;
  __syncthreads();
  // flush the workgroup's partial sums: one global atomic per touched entry
  for (int i = threadIdx.x; i < tab.size; i += kThreads) {
    const float v = lds[i];
    if (v == 0.f) continue;
    float* dst = nullptr;
    int j = i;
    if (tab.useV && i >= tab.vOff && i < tab.vOff + (int)a.V * 3) { dst = a.grad_verts; j = i - tab.vOff; }
    else if (tab.useV && i >= tab.nOff && i < tab.nOff + (int)a.V * 3) { dst = a.grad_normals; j = i - tab.nOff; }
    else if (tab.useV && i >= tab.cOff && i < tab.cOff + (int)a.V * 3) { dst = a.grad_vert_colors; j = i - tab.cOff; }
    else if (tab.useB && i >= tab.lOff && i < tab.lOff + a.N * 3) { dst = a.grad_light; j = i - tab.lOff; }
    else if (tab.useB && i >= tab.camOff && i < tab.camOff + a.N * 3) { dst = a.grad_camera; j = i - tab.camOff; }
    if (dst) atomicAdd(&dst[j], v);
  }
}

int shade_check(const PRShadeArgs& a) {
  if (a.N <= 0 || a.H <= 0 || a.W <= 0 || a.K <= 0) return set_error(PR_ERR_ARG, "shade: bad shape");
  if (!a.pix_to_face || !a.bary || !a.faces || !a.verts || !a.normals)
    return set_error(PR_ERR_ARG, "shade: fragment / mesh buffer missing");
  if (!a.light || !a.ambient || !a.diffuse_color || !a.specular_color || !a.mat_diffuse || !a.mat_specular ||
      !a.shininess || !a.camera)
    return set_error(PR_ERR_ARG, "shade: lighting buffer missing");
  if (a.texture == PR_TEX_GIVEN ? !a.texels
      : a.texture == PR_TEX_VERTEX ? !a.vert_colors
      : a.texture == PR_TEX_UV ? (!a.face_uvs || !a.maps || a.Hm <= 0 || a.Wm <= 0)
      : true)
    return set_error(PR_ERR_ARG, "shade: texture source missing or unknown");
  if (a.V < 0 || a.F < 0 || a.V >= (int64_t(1) << 31)) return set_error(PR_ERR_ARG, "shade: bad mesh size");
  return PR_OK;
}

int shade_blocks(int64_t PK) { return (int)std::min<int64_t>((PK + kThreads - 1) / kThreads, 16384); }

// ---- deterministic mode layout: [vertex scatter][batch scatter][texel scatter][V x 9][N x 6]
constexpr int64_t kDetChunk = 1024;  // entries per sequential chunk (cube vertices hold ~10^5)

struct DetPlan {
  int64_t nv, nb, nm, Mv, Mb, Mm;
  size_t wv, wb, wm, out9, out6;
};

size_t al(size_t b) { return (b + 255) / 256 * 256; }

// sized for one batch of det_batch() slots (the frame runs in batches: shade_bwd_deterministic)
DetPlan det_plan(const PRShadeArgs& a) {
  DetPlan p{};
  const int64_t PK = std::min<int64_t>((int64_t)a.N * a.H * a.W * a.K, det_batch());
  const bool vtx = a.grad_verts || a.grad_normals || (a.texture == PR_TEX_VERTEX && a.grad_vert_colors);
  p.nv = vtx && a.V > 0 ? PK * 3 : 0;
  p.Mv = a.V;
  p.nb = a.grad_light || a.grad_camera ? PK : 0;
  p.Mb = a.N;
  p.nm = a.texture == PR_TEX_UV && a.grad_maps ? PK * 4 : 0;
  p.Mm = (int64_t)a.N * a.Hm * a.Wm;
  p.wv = al(detsum_workspace(p.nv, p.Mv, 9));
  p.wb = al(detsum_workspace(p.nb, p.Mb, 6));
  p.wm = al(detsum_workspace(p.nm, p.Mm, 3));
  p.out9 = p.nv ? al((size_t)a.V * 9 * 4) : 0;
  p.out6 = p.nb ? al((size_t)a.N * 6 * 4) : 0;
  return p;
}

__global__ void split_kernel(const float* src, int64_t rows, int C, float* d0, float* d1, float* d2) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * C; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / C;
    const int c = (int)(i - r * C), part = c / 3;
    float* d = part == 0 ? d0 : (part == 1 ? d1 : d2);
    if (d) d[r * 3 + c % 3] = src[i];
  }
}

int shade_bwd_deterministic(const PRShadeArgs& a, hipStream_t st) {
  const DetPlan p = det_plan(a);
  const size_t need = p.wv + p.wb + p.wm + p.out9 + p.out6;
  if (!a.workspace || a.workspace_bytes < need) return set_error(PR_ERR_WORKSPACE, "shade_bwd: workspace too small");
  char* w = reinterpret_cast<char*>(a.workspace);
  float* out9 = reinterpret_cast<float*>(w + p.wv + p.wb + p.wm);
  float* out6 = reinterpret_cast<float*>(w + p.wv + p.wb + p.wm + p.out9);
  const int64_t total = (int64_t)a.N * a.H * a.W * a.K, batch = det_batch();
  Tab tab{};
  // batches of slots [s0, s0 + nb): each batch's ordered sums are added to the previous batches'
  // (deterministic: the batch size is fixed; one batch below det_batch() slots)
  for (int64_t s0 = 0; s0 < total; s0 += batch) {
    const int64_t nb = std::min(batch, total - s0);
    ShadeDet det;
    if (int e = detsum_layout(w, p.wv, p.nv ? nb * 3 : 0, p.Mv, 9, det.v)) return e;
    if (int e = detsum_layout(w + p.wv, p.wb, p.nb ? nb : 0, p.Mb, 6, det.b)) return e;
    if (int e = detsum_layout(w + p.wv + p.wb, p.wm, p.nm ? nb * 4 : 0, p.Mm, 3, det.m)) return e;
    shade_bwd_kernel<true><<<shade_blocks(nb), kThreads, 0, st>>>(a, s0, s0 + nb, (int64_t)a.H * a.W, tab, det);
    if (int e = check_launch("shade_bwd_det")) return e;
    const DetSum* ds[3] = {&det.v, &det.b, &det.m};
    float* outs[3] = {out9, out6, a.grad_maps};
    for (int i = 0; i < 3; ++i) {
      if (ds[i]->n == 0) continue;
      if (int e = detsum_sort(*ds[i], st)) return e;
      if (int e = detsum_gather(*ds[i], st)) return e;
      if (int e = detsum_reduce(*ds[i], outs[i], kDetChunk, s0 > 0, st)) return e;
    }
  }
  if (p.nv) {
    split_kernel<<<shade_blocks(a.V * 9), kThreads, 0, st>>>(out9, a.V, 9, a.grad_verts, a.grad_normals,
                                                             a.texture == PR_TEX_VERTEX ? a.grad_vert_colors : nullptr);
    if (int e = check_launch("shade_split_v")) return e;
  }
  if (p.nb) {
    split_kernel<<<1, kThreads, 0, st>>>(out6, a.N, 6, a.grad_light, a.grad_camera, nullptr);
    if (int e = check_launch("shade_split_b")) return e;
  }
  return PR_OK;
}

}  // namespace
}  // namespace pr

using namespace pr;

extern "C" int pr_shade_fwd(const PRShadeArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "shade_fwd: null args");
  const PRShadeArgs& a = *args;
  if (int e = shade_check(a)) return e;
  if (!a.colors) return set_error(PR_ERR_ARG, "shade_fwd: colors missing");
  const int64_t PK = (int64_t)a.N * a.H * a.W * a.K;
  shade_fwd_kernel<<<shade_blocks(PK), kThreads, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      a, PK, (int64_t)a.H * a.W);
  return check_launch("shade_fwd");
}

extern "C" size_t pr_shade_bwd_workspace_size(const PRShadeArgs* args) {
  if (!args || !(args->flags & PR_DETERMINISTIC)) return 0;
  const DetPlan p = det_plan(*args);
  return p.wv + p.wb + p.wm + p.out9 + p.out6;
}

extern "C" int pr_shade_bwd(const PRShadeArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "shade_bwd: null args");
  const PRShadeArgs& a = *args;
  if (int e = shade_check(a)) return e;
  if (!a.grad_colors) return set_error(PR_ERR_ARG, "shade_bwd: grad_colors missing");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.flags & PR_DETERMINISTIC) return shade_bwd_deterministic(a, st);
  struct Z { float* p; size_t n; } zs[] = {
      {a.grad_verts, (size_t)a.V * 3}, {a.grad_normals, (size_t)a.V * 3},
      {a.texture == PR_TEX_VERTEX ? a.grad_vert_colors : nullptr, (size_t)a.V * 3},
      {a.texture == PR_TEX_UV ? a.grad_maps : nullptr, (size_t)a.N * a.Hm * a.Wm * 3},
      {a.grad_light, (size_t)a.N * 3}, {a.grad_camera, (size_t)a.N * 3}};
  for (const Z& z : zs)
    if (z.p && z.n && hipMemsetAsync(z.p, 0, z.n * sizeof(float), st) != hipSuccess)
      return set_error(PR_ERR_HIP, "shade_bwd: memset failed");
  Tab tab;
  const int v3n = (int)std::min<int64_t>(a.V * 3, kLdsFloats);
  tab.useV = a.V * 9 + (int64_t)a.N * 6 <= kLdsFloats;
  tab.useB = (int64_t)a.N * 6 <= kLdsFloats / 4;
  tab.vOff = 0;
  tab.nOff = tab.useV ? v3n : 0;
  tab.cOff = tab.useV ? 2 * v3n : 0;
  tab.lOff = tab.useV ? 3 * v3n : 0;
  tab.camOff = tab.lOff + (tab.useB ? a.N * 3 : 0);
  tab.size = tab.camOff + (tab.useB ? a.N * 3 : 0);
  if (tab.size == 0) tab.size = 1;
  const int64_t PK = (int64_t)a.N * a.H * a.W * a.K;
  // fewer, fatter workgroups when the LDS table is large (its zero + flush is per workgroup)
  const int nb = std::min(shade_blocks(PK), tab.size > 1024 ? 1024 : 16384);
  shade_bwd_kernel<false><<<nb, kThreads, (size_t)tab.size * sizeof(float), st>>>(a, 0, PK, (int64_t)a.H * a.W, tab,
                                                                                  ShadeDet{});
  return check_launch("shade_bwd");
}
