// Phong shading of one fragment slot, device side: PyTorch3D 0.4.0 phong_shading with the texel
// lookup of Meshes.sample_textures (TexturesUV bilinear / TexturesVertex / given texels), the colour
// producer of RandomPhongShader (random_rasterizer.py:99-110, experiments/eval.py:170).  Shared by the
// shading kernels (pr_shade.hip) and the blend's fused Phong colour mode (pr_blend.hip, PR_BLEND_PHONG):
// one source, so both compute every slot colour with the same operations (bit-identical results).
#pragma once
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



PR_DEV Slot pad_slot(int n) { return Slot{-1, n, {0.f, 0.f, 0.f}}; }

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

// fv: the face's vertices (read only when sl.f >= 0); s < 0 skips the per-slot texel of
// PR_TEX_GIVEN (the per-image padded terms)
PR_DEV Shade shade(const PRShadeArgs& a, const Slot& sl, int64_t s, const int64_t* fv) {
  Shade z;
  const V3 zero{0.f, 0.f, 0.f};
  z.P = sl.f >= 0 ? interp3(a.verts, fv, sl.b) : zero;
  z.Nn = sl.f >= 0 ? interp3(a.normals, fv, sl.b) : zero;
  z.uvw = zero;
  if (a.texture == PR_TEX_GIVEN) {
    z.tex = s >= 0 ? v3(a.texels + s * 3) : zero;
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

// colour = lit * tex + spec
struct Terms {
  V3 lit, spec, tex;
};

PR_DEV Terms terms_of(const PRShadeArgs& a, int n, const Shade& z) {
  const float angle = fmaxf(z.cosang, 0.f);
  const V3 dl = angle * v3(a.diffuse_color + n * 3);
  const float pw = powf(z.alpha, a.shininess[n]);
  const V3 sp = pw * v3(a.specular_color + n * 3);
  return Terms{v3(a.ambient + n * 3) + v3(a.mat_diffuse + n * 3) * dl, v3(a.mat_specular + n * 3) * sp, z.tex};
}

PR_DEV Terms slot_terms(const PRShadeArgs& a, const Slot& sl, int64_t s, const int64_t* fv) {
  const Shade z = shade(a, sl, s, fv);
  return terms_of(a, sl.n, z);
}

PR_DEV V3 colour(V3 lit, V3 tex, V3 spec) { return lit * tex + spec; }

// ---- per-slot backward of the colour: every gradient piece of one live slot, before any scatter
// (pr_shade.hip's slot_bwd scatters them into its LDS table or ordered sums; the blend's fused
// Phong mode, pr_blend.hip, into global accumulators).  gc = d colour of the slot.
struct PhongGrad {
  V3 g_P, g_Nn, g_tex;  // d position, d normal (both interpolated), d texel
  V3 g_dir, g_vraw;     // d light (location or direction), d camera centre
  float gb[3];          // d bary: interpolations (+ the UV lookup)
  float w[4];           // UV: bilinear corner weights (torch's nw, ne, sw, se)
  int64_t ti[4];        // UV: corner texel offsets (floats) in the image's map, -1 outside
};

// (z: the slot's forward state, shade(a, sl, s, fv))
PR_DEV PhongGrad phong_bwd_z(const PRShadeArgs& a, const Slot& sl, const Shade& z, const int64_t* fv, V3 gc) {
  PhongGrad q;
  const int n = sl.n;
  const float angle = fmaxf(z.cosang, 0.f);
  const V3 dcol = v3(a.diffuse_color + n * 3), scol = v3(a.specular_color + n * 3);
  const V3 mdif = v3(a.mat_diffuse + n * 3), mspec = v3(a.mat_specular + n * 3);
  const V3 lit = v3(a.ambient + n * 3) + mdif * (angle * dcol);
  // colour = lit * tex + mspec * (pow(alpha, sh) * scol)
  q.g_tex = lit * gc;
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
  q.g_vraw = normalize_bwd(z.vraw, g_view);
  q.g_dir = normalize_bwd(z.dir, g_dh);
  q.g_Nn = normalize_bwd(z.Nn, g_nh);
  q.g_P = V3{0.f, 0.f, 0.f} - q.g_vraw;
  if (!a.directional) q.g_P = q.g_P - q.g_dir;
  // interpolations: d bary
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int64_t vi = fv[i];
    q.gb[i] = dot(q.g_P, v3(a.verts + vi * 3)) + dot(q.g_Nn, v3(a.normals + vi * 3));
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) { q.w[c] = 0.f; q.ti[c] = -1; }
  if (a.texture == PR_TEX_VERTEX) {
#pragma unroll
    for (int i = 0; i < 3; ++i) q.gb[i] += dot(q.g_tex, v3(a.vert_colors + fv[i] * 3));
  } else if (a.texture == PR_TEX_UV) {
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
      q.w[c] = w[c];
      if (cx[c] >= 0 && cx[c] < a.Wm && cy[c] >= 0 && cy[c] < a.Hm) {
        const int64_t ti = ((int64_t)(a.Hm - 1 - cy[c]) * a.Wm + cx[c]) * 3;
        q.ti[c] = ti;
        const float gv = dot(v3(map + ti), q.g_tex);
        gix += dwx[c] * gv;
        giy += dwy[c] * gv;
      }
    }
    const float gu = gix * bl.gx, gvv = giy * bl.gy;
    const float* uvq = a.face_uvs + sl.f * 6;
#pragma unroll
    for (int i = 0; i < 3; ++i) q.gb[i] += gu * uvq[2 * i] + gvv * uvq[2 * i + 1];
  }
  return q;
}

PR_DEV PhongGrad phong_bwd(const PRShadeArgs& a, const Slot& sl, int64_t s, const int64_t* fv, V3 gc) {
  const Shade z = shade(a, sl, s, fv);
  return phong_bwd_z(a, sl, z, fv, gc);
}

}  // namespace
}  // namespace pr
