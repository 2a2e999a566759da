// K-nearest-face mesh rasterizer (forward + backward) and face-attribute
// interpolation, with the semantics of PyTorch3D 0.4.0's rasterize_meshes
// (the [p3d] dependency of the reference, requirements.txt:7, called through
// MeshRasterizer at experiments/eval.py:165-168).  Semantics restated in
// SURVEY.md §8 a10/a11 and oracle/rast_oracle.c.
//
// Forward (MI355X layout): one wave per tile (4x4 pixels by default), lane = (pixel,
// face slice).  The tile's faces are culled (fp16 boxes, ballot compaction), sorted by
// depth near the tile centre and staged through LDS in chunks; the slices of a pixel test
// interleaved sorted positions with a two-stage (certain-reject, then exact) face test and
// share one K-queue per pixel in LDS, sorted by (z, face id) -- PyTorch3D's ordering.  The
// output pass writes p2f/zbuf, the winners' barycentrics / distances and the per-pixel
// valid-prefix counts.  MeshRasterizer's projection can run in the same face pass
// (pr_project_rast_fwd).  Scheduling: tiles are dispatched centre-out (Chebyshev rings)
// so a centred object's heavy tiles start first, and waves with long face lists raise
// their priority (the kernel's span is its heaviest tiles).
//
// Backward: per tile, the valid-prefix slots are compacted, each face gets a tile-local index,
// the per-slot gradients go to LDS without atomics and are summed per face by a
// face x pixel transpose; one global atomic per (face, component) per tile.
#include <cstdlib>
#include <type_traits>

#include <hip/hip_fp16.h>

#include "pr_common.h"

namespace pr {
namespace {

constexpr float kEps = 1e-8f;  // PyTorch3D kEpsilon
constexpr int kTile = 4;       // narrowest forward tile width (4x4 tiles at 4 slices)

struct V2 {
  float x, y;
};

// a / b: IEEE division (FAST = false: every forward value and every decision that
// must agree with the forward) or reciprocal-multiply (FAST: backward arithmetic,
// ~1 ulp, compared with a tolerance)
template <bool FAST = false>
PR_DEV float dv(float a, float b) {
  if constexpr (FAST) return a * __builtin_amdgcn_rcpf(b);
  else return a / b;
}

PR_DEV float edge_fn(V2 p, V2 a, V2 b) { return (p.x - a.x) * (b.y - a.y) - (p.y - a.y) * (b.x - a.x); }

PR_DEV void bary_fwd(V2 p, V2 v0, V2 v1, V2 v2, float w[3]) {
  const float area = edge_fn(v2, v0, v1) + kEps;
  w[0] = edge_fn(p, v1, v2) / area;
  w[1] = edge_fn(p, v2, v0) / area;
  w[2] = edge_fn(p, v0, v1) / area;
}

template <bool FAST = false>
PR_DEV void persp_fwd(const float b[3], float z0, float z1, float z2, float o[3]) {
  const float t0 = b[0] * z1 * z2, t1 = z0 * b[1] * z2, t2 = z0 * z1 * b[2];
  float d = t0 + t1 + t2;
  d = d > kEps ? d : kEps;
  o[0] = dv<FAST>(t0, d); o[1] = dv<FAST>(t1, d); o[2] = dv<FAST>(t2, d);
}

template <bool FAST = false>
PR_DEV void clip_fwd(const float b[3], float o[3]) {
  const float w0 = b[0] > 0.f ? b[0] : 0.f, w1 = b[1] > 0.f ? b[1] : 0.f, w2 = b[2] > 0.f ? b[2] : 0.f;
  float s = w0 + w1 + w2;
  s = s > 1e-5f ? s : 1e-5f;
  o[0] = dv<FAST>(w0, s); o[1] = dv<FAST>(w1, s); o[2] = dv<FAST>(w2, s);
}

// squared distance from p to segment ab
PR_DEV float seg_dist2(V2 p, V2 a, V2 b) {
  const float bax = b.x - a.x, bay = b.y - a.y;
  const float l2 = bax * bax + bay * bay;
  if (l2 <= kEps) {
    const float dx = p.x - b.x, dy = p.y - b.y;
    return dx * dx + dy * dy;
  }
  float t = (bax * (p.x - a.x) + bay * (p.y - a.y)) / l2;
  t = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
  const float qx = a.x + t * bax, qy = a.y + t * bay;
  const float dx = p.x - qx, dy = p.y - qy;
  return dx * dx + dy * dy;
}

PR_DEV float tri_dist2(V2 p, V2 v0, V2 v1, V2 v2) {
  const float e01 = seg_dist2(p, v0, v1), e02 = seg_dist2(p, v0, v2), e12 = seg_dist2(p, v1, v2);
  float m = e01 < e02 ? e01 : e02;
  return m < e12 ? m : e12;
}

PR_DEV float ndc(int i, int S1, int S2) {
  float range = 2.0f;
  if (S1 > S2) range = ((float)S1 * range) / (float)S2;
  const float off = range / 2.0f;
  return -off + (range * (float)i + off) / (float)S1;
}

// Per-face record for the forward traversal (96 B).  Besides the vertices it holds
// the edge deltas and the (area + eps) that bary_fwd / seg_dist2 would compute:
// the same IEEE operations on the same operands, so every per-pixel value below is
// bit-identical to the straightforward formulas (and to oracle/rast_oracle.c).
// Invalid faces get an empty bbox (+inf / -inf) so every cull rejects them.
struct FaceRec {
  float4 a;  // v0.x v0.y v0.z v1.x
  float4 b;  // v1.y v1.z v2.x v2.y
  float4 c;  // v2.z xmin xmax ymin   (bbox grown by sqrt(blur))
  float4 d;  // ymax area+eps l2_01 l2_12
  float4 e;  // D01.x D01.y D12.x D12.y   (D01 = v1 - v0, D12 = v2 - v1)
  float4 f;  // D20.x D20.y l2_20 z_min   (D20 = v0 - v2)
};

// the face record and cull box of one face from its projected corners
// Cull boxes in fp16, rounded outward (never smaller than the exact box): 8 B per face of
// L2 traffic per tile instead of 16.  The cull only selects a superset; the per-pixel test
// re-checks the exact box from the face record, so results do not change.
PR_DEV uint32_t half_bits(__half h) { return (uint32_t)__half_as_ushort(h); }
PR_DEV uint2 pack_box(float xmin, float xmax, float ymin, float ymax) {
  return make_uint2(half_bits(__float2half_rd(xmin)) | (half_bits(__float2half_ru(xmax)) << 16),
                    half_bits(__float2half_rd(ymin)) | (half_bits(__float2half_ru(ymax)) << 16));
}
PR_DEV float4 unpack_box(uint2 b) {
  return make_float4(__half2float(__ushort_as_half((unsigned short)(b.x & 0xffffu))),
                     __half2float(__ushort_as_half((unsigned short)(b.x >> 16))),
                     __half2float(__ushort_as_half((unsigned short)(b.y & 0xffffu))),
                     __half2float(__ushort_as_half((unsigned short)(b.y >> 16))));
}

PR_DEV void write_face_rec(const float v[9], float blur, int cull_backfaces, FaceRec* out, uint2* bbox) {
  const float x0 = v[0], y0 = v[1], z0 = v[2], x1 = v[3], y1 = v[4], z1 = v[5], x2 = v[6], y2 = v[7], z2 = v[8];
  const float r = sqrtf(blur);
  float xmin = fminf(x0, fminf(x1, x2)) - r, xmax = fmaxf(x0, fmaxf(x1, x2)) + r;
  float ymin = fminf(y0, fminf(y1, y2)) - r, ymax = fmaxf(y0, fmaxf(y1, y2)) + r;
  const float zmax = fmaxf(z0, fmaxf(z1, z2));
  const float area = edge_fn(V2{x0, y0}, V2{x1, y1}, V2{x2, y2});
  const bool back = area < 0.f;
  const bool zero_area = area <= kEps && area >= -kEps;
  const bool valid = !(zmax < 0.f || (cull_backfaces && back) || zero_area);
  if (!valid) { xmin = ymin = __builtin_inff(); xmax = ymax = -__builtin_inff(); }
  const float d01x = x1 - x0, d01y = y1 - y0, d12x = x2 - x1, d12y = y2 - y1, d20x = x0 - x2, d20y = y0 - y2;
  FaceRec rec;
  rec.a = make_float4(x0, y0, z0, x1);
  rec.b = make_float4(y1, z1, x2, y2);
  rec.c = make_float4(z2, xmin, xmax, ymin);
  rec.d = make_float4(ymax, edge_fn(V2{x2, y2}, V2{x0, y0}, V2{x1, y1}) + kEps, d01x * d01x + d01y * d01y,
                      d12x * d12x + d12y * d12y);
  rec.e = make_float4(d01x, d01y, d12x, d12y);
  rec.f = make_float4(d20x, d20y, d20x * d20x + d20y * d20y, fminf(z0, fminf(z1, z2)));
  *out = rec;
  *bbox = pack_box(xmin, xmax, ymin, ymax);
}

// ---- coarse bins (PyTorch3D's bin_size / max_faces_per_bin, rasterize_meshes.py): bins of
//      bs x bs pixels (bs a multiple of every tile shape), per mesh.  The face pass appends
//      each face to the bins its blur-grown box overlaps (an atomic per (face, bin)); a tile
//      culls only its bin's list, or the whole mesh if the bin overflowed its capacity.
struct BinGrid {
  int bs, nx, ny, cap;  // bin side (pixels), bins per row / column, list capacity per bin
  int* count;           // (N, ny, nx) list lengths (may exceed cap: overflow); null = no bins
  int* list;            // (N, ny, nx, cap) face ids (any order)
  int H, W;
};

// the bin's rectangle in NDC (its extreme pixel centres; a tile's rectangle lies inside)
PR_DEV void bin_rect(const BinGrid& g, int bx, int by, float& xmin, float& xmax, float& ymin, float& ymax) {
  const int c0 = bx * g.bs, c1 = min(c0 + g.bs - 1, g.W - 1), r0 = by * g.bs, r1 = min(r0 + g.bs - 1, g.H - 1);
  xmax = ndc(g.W - 1 - c0, g.W, g.H); xmin = ndc(g.W - 1 - c1, g.W, g.H);
  ymax = ndc(g.H - 1 - r0, g.H, g.W); ymin = ndc(g.H - 1 - r1, g.H, g.W);
}

// pixel index range [lo, hi] (one pixel of margin) whose NDC centres can lie in [vmin, vmax]
// along an axis of S1 pixels (ndc's inverse, clamped), as columns/rows counted from the far edge
PR_DEV void pix_range(float vmin, float vmax, int S1, int S2, int& lo, int& hi) {
  float range = 2.0f;
  if (S1 > S2) range = ((float)S1 * range) / (float)S2;
  const float off = range / 2.0f;
  const float ilo = fminf(fmaxf(((vmin + off) * (float)S1 - off) / range, -2.f), (float)S1 + 1.f);
  const float ihi = fminf(fmaxf(((vmax + off) * (float)S1 - off) / range, -2.f), (float)S1 + 1.f);
  // ndc index i maps to pixel S1 - 1 - i
  lo = max(0, (int)floorf((float)(S1 - 1) - ihi) - 1);
  hi = min(S1 - 1, (int)ceilf((float)(S1 - 1) - ilo) + 1);
}

PR_DEV void bin_face(const BinGrid& g, int n, int64_t f, uint2 packed) {
  const float4 bb = unpack_box(packed);  // the tiles' cull box: bins select a superset
  if (!(bb.x <= bb.y && bb.z <= bb.w)) return;  // culled face (empty box) or NaN
  int c0, c1, r0, r1;
  pix_range(bb.x, bb.y, g.W, g.H, c0, c1);
  pix_range(bb.z, bb.w, g.H, g.W, r0, r1);
  if (c0 > c1 || r0 > r1) return;
  const int bx0 = c0 / g.bs, nbx = c1 / g.bs - bx0 + 1, by0 = r0 / g.bs, nby = r1 / g.bs - by0 + 1;
  auto hits = [&](int bx, int by) {
    float xmin, xmax, ymin, ymax;
    bin_rect(g, bx, by, xmin, xmax, ymin, ymax);
    return !(bb.x > xmax || bb.y < xmin || bb.z > ymax || bb.w < ymin);
  };
  if (nbx * nby <= 16) {
    // every append's atomic in flight at once (one round trip per face, not one per bin)
    int b[16], c[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int bx = bx0 + k % nbx, by = by0 + k / nbx;
      b[k] = k < nbx * nby && hits(bx, by) ? (n * g.ny + by) * g.nx + bx : -1;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = b[k] >= 0 ? atomicAdd(g.count + b[k], 1) : g.cap;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (c[k] < g.cap) g.list[(int64_t)b[k] * g.cap + c[k]] = (int)f;
    return;
  }
  for (int by = by0; by < by0 + nby; ++by) {
    for (int bx = bx0; bx < bx0 + nbx; ++bx) {
      if (!hits(bx, by)) continue;
      const int bi = (n * g.ny + by) * g.nx + bx;
      const int c = atomicAdd(g.count + bi, 1);
      if (c < g.cap) g.list[(int64_t)bi * g.cap + c] = (int)f;
    }
  }
}

// mesh of packed face f (meshes are packed in order: mesh_first_face ascending)
PR_DEV int mesh_of_sorted(const int64_t* first, int N, int64_t f) {
  int lo = 0, hi = N - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (first[mid] <= f) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ void face_prep_kernel(const float* fv, int64_t F, float blur_v, const float* blur_dev, int cull_backfaces,
                                 FaceRec* out, uint2* bbox, BinGrid bins, const int64_t* mesh_first, int N) {
  const float blur = blur_dev ? *blur_dev : blur_v;
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < F; f += (int64_t)gridDim.x * blockDim.x) {
    float v[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) v[i] = fv[f * 9 + i];
    write_face_rec(v, blur, cull_backfaces, out + f, bbox + f);
    if (bins.count) bin_face(bins, mesh_of_sorted(mesh_first, N, f), f, bbox[f]);
  }
}

// q = i / d, r = i - q d for 0 <= i < 2^20 and 0 < d < 2^20 (float reciprocal + one correction)
PR_DEV int divmod_small(int i, int d, float inv_d, int& r) {
  int q = (int)((float)i * inv_d);
  r = i - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
  return q;
}

PR_DEV bool key_less(float za, int fa, float zb, int fb) { return za < zb || (za == zb && fa < fb); }

// seg_dist2 with the segment delta (b - a) and its squared length precomputed;
// branch-free (the degenerate-segment case is a select) so that several faces'
// tests form one straight-line block the scheduler can interleave
PR_DEV float seg_dist2_d(V2 p, V2 a, float bax, float bay, float l2, V2 b) {
  const float bx = p.x - b.x, by = p.y - b.y;
  const float db = bx * bx + by * by;
  float t = (bax * (p.x - a.x) + bay * (p.y - a.y)) / l2;
  t = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
  const float qx = a.x + t * bax, qy = a.y + t * bay;
  const float dx = p.x - qx, dy = p.y - qy;
  const float ds = dx * dx + dy * dy;
  return l2 <= kEps ? db : ds;
}

// Per-pixel evaluation of one face from its record: (clipped) barycentrics, their
// depth, the inside flag and the squared distance to the nearest edge, with exactly
// the operations of bary_fwd / persp_fwd / clip_fwd / tri_dist2 (bit-identical).
// Branch-free so that several faces' division chains interleave (ILP is the latency
// hiding at one wave per SIMD).  Perspective correction / clipping are compile-time.
template <bool PERSP, bool CLIP>
PR_DEV void face_eval(const FaceRec& r, V2 p, float bc[3], float& pz, bool& inside, float& d) {
  const V2 v0{r.a.x, r.a.y}, v1{r.a.w, r.b.x}, v2{r.b.z, r.b.w};
  const float z0 = r.a.z, z1 = r.b.y, z2 = r.c.x;
  const float area = r.d.y;
  // edge functions E(p,v1,v2), E(p,v2,v0), E(p,v0,v1) with the precomputed deltas
  const float e0 = (p.x - v1.x) * r.e.w - (p.y - v1.y) * r.e.z;
  const float e1 = (p.x - v2.x) * r.f.y - (p.y - v2.y) * r.f.x;
  const float e2 = (p.x - v0.x) * r.e.y - (p.y - v0.y) * r.e.x;
  float b[3] = {e0 / area, e1 / area, e2 / area};
  if constexpr (PERSP) {
    const float t0 = b[0] * z1 * z2, t1 = z0 * b[1] * z2, t2 = z0 * z1 * b[2];
    float s = t0 + t1 + t2;
    s = s > kEps ? s : kEps;
    b[0] = t0 / s; b[1] = t1 / s; b[2] = t2 / s;
  }
  if constexpr (CLIP) {
    clip_fwd(b, bc);
  } else {
    bc[0] = b[0]; bc[1] = b[1]; bc[2] = b[2];
  }
  pz = bc[0] * z0 + bc[1] * z1 + bc[2] * z2;
  inside = b[0] > 0.f && b[1] > 0.f && b[2] > 0.f;
  const float d01 = seg_dist2_d(p, v0, r.e.x, r.e.y, r.d.z, v1);
  const float d02 = seg_dist2_d(p, v0, -r.f.x, -r.f.y, r.f.z, v2);
  const float d12 = seg_dist2_d(p, v1, r.e.z, r.e.w, r.d.w, v2);
  d = d01 < d02 ? d01 : d02;
  d = d < d12 ? d : d12;
}

// PyTorch3D's per-face decisions: in bbox -> bary -> perspective -> clip -> pz >= 0 ->
// inside or dist < blur
template <bool PERSP, bool CLIP>
PR_DEV bool face_test(const FaceRec& r, V2 p, float blur, float& pz) {
  const bool inbox = !(p.x < r.c.y || p.x > r.c.z || p.y < r.c.w || p.y > r.d.x);
  float bc[3], d;
  bool inside;
  face_eval<PERSP, CLIP>(r, p, bc, pz, inside, d);
  return inbox && !(pz < 0.f) && (inside || d < blur);
}

// ---- two-stage test (no perspective correction): a cheap stage that only ever REJECTS
// with certainty, then the exact face_test for the survivors.
//  * inside: b_i = e_i / area > 0  <=>  e_i != 0 and sign(e_i) == sign(area) (area != 0 for
//    every uncull'd face).  So "not inside by signs" implies "not inside" exactly.
//  * edge distance with t = dot * rcp(l2) instead of dot / l2: the two squared distances differ
//    by at most the face's margin m = 4 sqrt(blur) delta + 2 delta^2 + blur 2^-20, where
//    delta = 2^-19 U bounds the difference of the computed dx (and dy) and U is the largest
//    coordinate magnitude of the face's corners and the tile's pixels (t differs by <= 2^-22;
//    t * (b - a), a + t (b - a) and p - q round at <= 2^-24 of magnitudes <= 2U; where the exact
//    distance is below blur, |dx| and |dy| are below sqrt(blur)).  dist_margin computes m per
//    staged face: proportional to blur for the usual NDC-sized faces, unbounded for faces with
//    huge corners (partly behind the camera), which then always take the exact test.  (A fixed
//    band of 1e-3 blur, rounds 1-4, was too narrow for such faces: tests/test_gpu_rast.py
//    test_rasterizer_forward_division_fallbacks_bitwise.)
// A lane is rejected only if it is outside its box, or outside the face by signs and
// farther than blur + m.  Everything else runs the exact test, so every decision and every
// value equals face_test's.
PR_DEV float dist_margin(float4 ra, float4 rb, float ptile, float sqrt_blur, float blur) {
  const float m = fmaxf(fmaxf(fmaxf(fabsf(ra.x), fabsf(ra.y)), fmaxf(fabsf(ra.w), fabsf(rb.x))),
                        fmaxf(fmaxf(fabsf(rb.z), fabsf(rb.w)), ptile));
  const float delta = m * 0x1p-19f;
  return 4.f * sqrt_blur * delta + 2.f * delta * delta + blur * 0x1p-20f;
}

PR_DEV float seg_dist2_fast(V2 p, V2 a, float bax, float bay, float l2, V2 b) {
  const float bx = p.x - b.x, by = p.y - b.y;
  const float db = bx * bx + by * by;
  float t = (bax * (p.x - a.x) + bay * (p.y - a.y)) * __builtin_amdgcn_rcpf(l2);
  t = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
  const float qx = a.x + t * bax, qy = a.y + t * bay;
  const float dx = p.x - qx, dy = p.y - qy;
  const float ds = dx * dx + dy * dy;
  return l2 <= kEps ? db : ds;
}

PR_DEV bool face_maybe(const FaceRec& r, V2 p, float blur, float margin, float& dfast) {
  const bool inbox = !(p.x < r.c.y || p.x > r.c.z || p.y < r.c.w || p.y > r.d.x);
  const V2 v0{r.a.x, r.a.y}, v1{r.a.w, r.b.x}, v2{r.b.z, r.b.w};
  const float e0 = (p.x - v1.x) * r.e.w - (p.y - v1.y) * r.e.z;
  const float e1 = (p.x - v2.x) * r.f.y - (p.y - v2.y) * r.f.x;
  const float e2 = (p.x - v0.x) * r.e.y - (p.y - v0.y) * r.e.x;
  const bool pos = r.d.y > 0.f;
  const bool ins = e0 != 0.f && e1 != 0.f && e2 != 0.f && (e0 > 0.f) == pos && (e1 > 0.f) == pos &&
                   (e2 > 0.f) == pos;
  const float d01 = seg_dist2_fast(p, v0, r.e.x, r.e.y, r.d.z, v1);
  const float d02 = seg_dist2_fast(p, v0, -r.f.x, -r.f.y, r.f.z, v2);
  const float d12 = seg_dist2_fast(p, v1, r.e.z, r.e.w, r.d.w, v2);
  float d = d01 < d02 ? d01 : d02;
  d = d < d12 ? d : d12;
  dfast = d;
  return inbox && (ins || !(d > blur + margin));
}

// The exact test for a lane that face_maybe kept (no perspective correction): barycentrics,
// clipping, pz and the inside flag with face_test's operations; the exact edge distance
// only where the fast one is within the face's margin of blur (a branch that is rarely
// taken by any lane of the wave: below blur - m the exact distance is below blur too).
template <bool CLIP>
PR_DEV bool face_test_kept(const FaceRec& r, V2 p, float blur, float margin, float dfast, float& pz) {
  const V2 v0{r.a.x, r.a.y}, v1{r.a.w, r.b.x}, v2{r.b.z, r.b.w};
  const float z0 = r.a.z, z1 = r.b.y, z2 = r.c.x;
  const float area = r.d.y;
  const float e0 = (p.x - v1.x) * r.e.w - (p.y - v1.y) * r.e.z;
  const float e1 = (p.x - v2.x) * r.f.y - (p.y - v2.y) * r.f.x;
  const float e2 = (p.x - v0.x) * r.e.y - (p.y - v0.y) * r.e.x;
  const float b[3] = {e0 / area, e1 / area, e2 / area};
  float bc[3];
  if constexpr (CLIP) {
    clip_fwd(b, bc);
  } else {
    bc[0] = b[0]; bc[1] = b[1]; bc[2] = b[2];
  }
  pz = bc[0] * z0 + bc[1] * z1 + bc[2] * z2;
  const bool inside = b[0] > 0.f && b[1] > 0.f && b[2] > 0.f;
  bool near = dfast < blur - margin;
  if (!inside && !near && !(dfast > blur + margin)) {  // in the band: exact distance
    const float d01 = seg_dist2_d(p, v0, r.e.x, r.e.y, r.d.z, v1);
    const float d02 = seg_dist2_d(p, v0, -r.f.x, -r.f.y, r.f.z, v2);
    const float d12 = seg_dist2_d(p, v1, r.e.z, r.e.w, r.d.w, v2);
    float d = d01 < d02 ? d01 : d02;
    d = d < d12 ? d : d12;
    near = d < blur;
  }
  return !(pz < 0.f) && (inside || near);
}

PR_DEV bool in_bbox(const FaceRec& r, V2 p) {
  return !(p.x < r.c.y || p.x > r.c.z || p.y < r.c.w || p.y > r.d.x);
}

#ifdef PR_RAST_PROFILE
constexpr unsigned kProfTiles = 1 << 16;
__device__ long long g_rast_prof[kProfTiles * 16];  // per tile: x y z list t0 t1 hwid stamps[6] SL
#define PR_STAMP(i) (stamp[i] += (long long)__builtin_amdgcn_s_memtime() - t_, t_ = __builtin_amdgcn_s_memtime())
#else
#define PR_STAMP(i) ((void)0)
#endif

// per-slice-count forward configuration: per-round tile face list capacity (faces beyond
// it go to later rounds), faces tested together per lane (independent chains), LDS
// staging chunk.  Smaller tiles have shorter lists and want more resident waves
// (LDS, VGPRs) rather than per-wave ILP.
template <int SL> struct RastCfg {
  static constexpr int CAP = SL == 1 ? 512 : (SL == 2 ? 256 : 128);
#ifndef PR_RAST_G4  // sweeps: 3 / 4 faces per lane measured equal or slower
#define PR_RAST_G4 2
#endif
  static constexpr int G = SL == 1 ? 4 : (SL >= 4 ? PR_RAST_G4 : 2);
#ifndef PR_RAST_CH4  // sweeps (r2): 16 vs 32 equal at cfg 2 (80.6 vs 81.0 us), 11 % faster at cfg 4
#define PR_RAST_CH4 16  // (5.26 vs 5.94 ms: less LDS per wave, more waves resident at K = 150)
#endif
  static constexpr int CH = SL >= 4 ? PR_RAST_CH4 : 64;
  static_assert(CAP <= 8 * 64, "suffix-min pass holds CAP / 64 <= 8 entries per lane");
};
// Queue row padding in entries.  The output pass reads a pixel's consecutive slots from one
// lane to the next: at the unpadded 16-entry (128 B) row stride those reads pile onto two of
// the 64 banks (~30-way conflicts; they were essentially all of rast_fwd's 1.6 M LDS bank
// conflicts per launch at cfg 2), one entry of padding spreads them.  The 8-slice layout (deep
// queues, K > 128) stays unpadded: LDS per wave matters more there (4-13 % slower padded at cfg 4).
#ifndef PR_RAST_QPAD  // sweeps: a fixed padding for every slice count
template <int SL> constexpr int rast_qpad() { return SL == 4 ? 1 : 0; }
#else
template <int SL> constexpr int rast_qpad() { return PR_RAST_QPAD; }
#endif
#ifndef PR_RAST_MERGE  // 0: candidates landing inside a queue are inserted slice by slice (r1 path)
#define PR_RAST_MERGE 1
#endif
#ifndef PR_RAST_FRAGC  // 0: the output pass evaluates faces lane by lane over all slots (r2 path)
#define PR_RAST_FRAGC 1
#endif
#ifndef PR_RAST_CULLU  // sweeps: 8 measured equal, 4 slower (+10 us)
#define PR_RAST_CULLU 16
#endif
constexpr int kCullU = PR_RAST_CULLU;  // 64-face cull chunks whose boxes are in flight together

// Bitonic sort (ascending key) of n2 (power of two) LDS entries by NT threads.
template <int NT>
PR_DEV void bitonic_sort(float* key, int* val, int n2, int tid) {
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < n2; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const float a = key[i], b = key[ixj];
          if ((a > b) == up) {
            key[i] = b; key[ixj] = a;
            const int t = val[i]; val[i] = val[ixj]; val[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Bitonic sort of E*64 (key, val) pairs held in one wave's registers, element
// i = e*64 + lane.  Strides < 64 exchange through __shfl_xor, larger strides swap
// registers of the same lane; no LDS and no barriers.  Equal keys keep their own
// element on both sides, so the network stays a permutation.
template <int E>
PR_DEV void wave_bitonic_sort(float (&key)[E], int (&val)[E], int lane) {
#pragma unroll
  for (int k = 2; k <= E * 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int je = j >> 6;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int pe = e ^ je;
          if (pe > e) {
            const bool up = ((e * 64 + lane) & k) == 0;
            const float a = key[e], b = key[pe];
            if ((a > b) == up) {
              key[e] = b; key[pe] = a;
              const int t = val[e]; val[e] = val[pe]; val[pe] = t;
            }
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float ok = __shfl_xor(key[e], j);
          const int ov = __shfl_xor(val[e], j);
          const int i = e * 64 + lane;
          const bool up = (i & k) == 0, lower = (lane & j) == 0;
          // lower index keeps min when ascending, max when descending; upper the opposite
          const bool take = lower == up ? (ok < key[e]) : (ok > key[e]);
          if (take) { key[e] = ok; val[e] = ov; }
        }
      }
    }
  }
}

// sort lkey/lidx[0, n2) (n2 a power of two, <= 512) by wave 0 of the workgroup
template <int E>
PR_DEV void wave_sort_lds(float* lkey, int* lidx, int lane) {
  float kk[E];
  int vv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { kk[e] = lkey[e * 64 + lane]; vv[e] = lidx[e * 64 + lane]; }
  wave_bitonic_sort<E>(kk, vv, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) { lkey[e * 64 + lane] = kk[e]; lidx[e * 64 + lane] = vv[e]; }
}

PR_DEV bool ekey_less(float2 x, float2 y) { return key_less(x.x, __float_as_int(x.y), y.x, __float_as_int(y.y)); }

// one wave's LDS region of rast_fwd_kernel (16-byte multiple: the next wave's chunk records)
template <int SL>
PR_HD size_t rast_fwd_wave_bytes(int K) {
  using C = RastCfg<SL>;
  const size_t b = C::CH * sizeof(FaceRec) + (size_t)K * (64 / SL + rast_qpad<SL>()) * 8 + 64 * 4 + C::CH * 12;
  return (b + 15) / 16 * 16;
}

template <int SL>
size_t rast_fwd_lds_sl(int K, int NW) {
  return NW * rast_fwd_wave_bytes<SL>(K) + (size_t)RastCfg<SL>::CAP * 12 + 16;
}

size_t rast_fwd_lds(int K, int SL, int NW = 1) {
  return SL == 8 ? rast_fwd_lds_sl<8>(K, 1)
                 : SL == 4 ? rast_fwd_lds_sl<4>(K, NW) : (SL == 2 ? rast_fwd_lds_sl<2>(K, 1) : rast_fwd_lds_sl<1>(K, 1));
}

// v from the lane of the same pixel that holds slice s (lane = pixel * SL + slice):
// one DPP quad permutation
template <int SL>
PR_DEV int from_slice(int v, int s) {
  if constexpr (SL == 1) {
    return v;
  } else if constexpr (SL == 2) {
    switch (s) {
      case 0: return __builtin_amdgcn_update_dpp(0, v, 0xA0, 0xf, 0xf, false);  // quad_perm [0,0,2,2]
      default: return __builtin_amdgcn_update_dpp(0, v, 0xF5, 0xf, 0xf, false); // quad_perm [1,1,3,3]
    }
  } else if constexpr (SL == 8) {  // beyond a DPP quad: a lane permute
    return __shfl(v, (int)(__lane_id() & ~7u) | s);
  } else {
    switch (s) {
      case 0: return __builtin_amdgcn_update_dpp(0, v, 0x00, 0xf, 0xf, false);  // quad_perm [0,0,0,0]
      case 1: return __builtin_amdgcn_update_dpp(0, v, 0x55, 0xf, 0xf, false);
      case 2: return __builtin_amdgcn_update_dpp(0, v, 0xAA, 0xf, 0xf, false);
      default: return __builtin_amdgcn_update_dpp(0, v, 0xFF, 0xf, 0xf, false);
    }
  }
}

// v from the lane r places further along the pixel's SL lanes (cyclically): DPP quad
// rotations, so every lane sees its pixel's other slices
template <int SL>
PR_DEV int quad_rot(int v, int r) {
  if constexpr (SL == 2) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  } else if constexpr (SL == 8) {
    const unsigned l = __lane_id();
    return __shfl(v, (int)((l & ~7u) | ((l + (unsigned)r) & 7u)));
  } else {
    switch (r) {
      case 1: return __builtin_amdgcn_update_dpp(0, v, 0x39, 0xf, 0xf, false);  // quad_perm [1,2,3,0]
      case 2: return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
      default: return __builtin_amdgcn_update_dpp(0, v, 0x93, 0xf, 0xf, false); // quad_perm [3,0,1,2]
    }
  }
}

// Forward: per-pixel K nearest (z, face) keys -> pix_to_face, zbuf (+ barycentrics and
// signed distances with FRAG).  One wave per tile of TP = 64 / SL pixels (8x8, 8x4 or
// 4x4); lane = pixel * SL + slice.  The SL lanes of a pixel (one DPP quad) split the
// tile's face list -- slice h tests sorted positions h, h+SL, ... -- and share ONE
// K-queue per pixel in LDS: after each test group the slices insert their candidates
// in turn, the pixel's queue state (size, last key) travelling between them by DPP.
// Slicing cuts the heaviest tiles' serial face loop (the kernel's critical path) by SL
// while the per-pixel queue keeps LDS at K*TP*8 B, so several tiles share a SIMD.
// Per round: cull the mesh's faces against the tile (boxes of 16 chunks in flight,
// ballot compaction), sort the survivors by their depth near the tile centre, then
// walk the sorted list in CH-face chunks staged in LDS, each lane testing kGroup faces
// at once (independent chains).  The queue is an LDS column sorted by (z, face id),
// PyTorch3D's order, and ends as the K smallest keys of all candidates: it depends
// neither on SL nor on the traversal order.
//
// Tile order (ring = 1, square grids of even side): block b takes the b-th tile of the
// Chebyshev rings around the image centre, so the tiles of a centred object -- the heavy
// ones -- are dispatched first and the cheap empty border tiles fill the tail (row-major
// order started the bottom quarter's heavy tiles only when the first tiles retired).
PR_DEV void ring_tile(int b, int m, int& tx, int& ty) {
  int r = (int)(__builtin_sqrtf((float)b) * 0.5f);
  while (4 * (r + 1) * (r + 1) <= b) ++r;
  while (4 * r * r > b) --r;
  const int k = b - 4 * r * r, s = 2 * r + 2, c0 = m / 2 - r - 1;  // ring r: side s, corner (c0, c0)
  if (k < s) { tx = c0 + k; ty = c0; }
  else if (k < 2 * s - 2) { tx = c0 + s - 1; ty = c0 + 1 + (k - s); }
  else if (k < 3 * s - 2) { tx = c0 + s - 1 - (k - (2 * s - 2)); ty = c0 + s - 1; }
  else { tx = c0; ty = c0 + s - 2 - (k - (3 * s - 2)); }
}

#ifndef PR_RAST_WPE  // sweeps: 4 waves/SIMD (with PR_RAST_CH4=16: 128 VGPRs, 2 spills) measured equal
#define PR_RAST_WPE 1
#endif
#ifndef PR_RAST_DUO_WPE  // two-wave tiles: waves per SIMD the register budget must allow
#define PR_RAST_DUO_WPE 1
#endif
// NW = 2 (PR_RAST_DUO, SL = 4): two waves per tile.  Wave 0 culls and sorts the tile's face
// list; the waves then walk alternate chunks of it, each into its own per-pixel K-queue, so a
// heavy tile's test loop -- its critical path -- is split in two; the output pass reads the
// k-th smallest key of the two queues by a merge-path search and is split over both waves.
// The queues end as the K smallest keys of their halves, so the merged K smallest are the
// one-wave kernel's: the same fragments bit for bit.
template <int SL, bool PERSP, bool CLIP, bool FRAG, int NW>
__global__ void __launch_bounds__(64 * NW, NW == 2 ? PR_RAST_DUO_WPE : PR_RAST_WPE)
    rast_fwd_kernel(PRRastArgs a, const FaceRec* __restrict__ faces, const uint2* __restrict__ fbox, int ring,
                    BinGrid bins) {
  constexpr int TW = SL >= 4 ? 4 : 8, TH = 64 / SL / TW, TP = TW * TH;
  constexpr int kCap = RastCfg<SL>::CAP, kGroup = RastCfg<SL>::G, CH = RastCfg<SL>::CH;
  constexpr int QS = TP + rast_qpad<SL>();  // queue row stride (entries): padding spreads a pixel's rows over banks
  constexpr int NT = 64 * NW;               // threads per tile
  extern __shared__ float smem[];
  const int K = a.K;
  const int tid = threadIdx.x, lane = tid & 63, wv = NW == 2 ? tid >> 6 : 0;
  const int pix = lane / SL, slice = lane % SL;
  // per-wave regions [staged chunk | queues | queue sizes | chunk ids | suffix mins | margins],
  // then the tile's shared face list (rast_fwd_lds_sl)
  const size_t wbytes = rast_fwd_wave_bytes<SL>(K);
  char* wbase = reinterpret_cast<char*>(smem) + wv * wbytes;
  FaceRec* lrec = reinterpret_cast<FaceRec*>(wbase);                // [CH] staged chunk
  float2* q = reinterpret_cast<float2*>(lrec + CH);                 // [K][QS] per-pixel queues
  int* qsz = reinterpret_cast<int*>(q + (size_t)K * QS);            // [64] queue sizes (per pixel)
  int* lcf = qsz + 64;                                              // [CH] staged chunk face ids
  float* lcs = reinterpret_cast<float*>(lcf + CH);                  // [CH] staged chunk suffix mins
  float* lmg = lcs + CH;                                            // [CH] staged faces' distance margins
  int* lfid = reinterpret_cast<int*>(reinterpret_cast<char*>(smem) + NW * wbytes);  // [kCap] tile face list
  float* lkey = reinterpret_cast<float*>(lfid + kCap);              // [kCap] sort key, then
  float* lsuf = lkey;                                               //   suffix min of z_min
  int* lidx = reinterpret_cast<int*>(lkey + kCap);                  // [kCap] sorted -> cull order
  int64_t* lctl = reinterpret_cast<int64_t*>(lidx + kCap);          // [2] round: next cull position, list size
  const int n = blockIdx.z;
  const int H = a.H, W = a.W;
  int tile_x = blockIdx.x, tile_y = blockIdx.y;
  if (ring & 1) {
    const int b = blockIdx.y * gridDim.x + blockIdx.x;
    if (gridDim.y == gridDim.x) {
      ring_tile(b, gridDim.x, tile_x, tile_y);
    } else {  // gridDim.y == 2 gridDim.x: rings over 1x2 super-tiles
      ring_tile(b >> 1, gridDim.x, tile_x, tile_y);
      tile_y = 2 * tile_y + (b & 1);
    }
  }
  const int row0 = tile_y * TH, col0 = tile_x * TW;
  const int row = row0 + pix / TW, col = col0 + pix % TW;
  const bool inimg = row < H && col < W;
  const V2 p{ndc(W - 1 - min(col, W - 1), W, H), ndc(H - 1 - min(row, H - 1), H, W)};
  // tile rectangle in NDC (pixel centres); +X points left, +Y up
  const int c1 = min(col0 + TW - 1, W - 1), r1 = min(row0 + TH - 1, H - 1);
  const float txmax = ndc(W - 1 - col0, W, H), txmin = ndc(W - 1 - c1, W, H);
  const float tymax = ndc(H - 1 - row0, H, W), tymin = ndc(H - 1 - r1, H, W);
  const float tcx = 0.5f * (txmin + txmax), tcy = 0.5f * (tymin + tymax);
  const float ptile = fmaxf(fmaxf(fabsf(txmin), fabsf(txmax)), fmaxf(fabsf(tymin), fabsf(tymax)));
  const int64_t fb = a.mesh_first_face[n];
  // the faces to cull: the tile's bin list, or the whole mesh (no bins, or the bin overflowed)
  const int* ids = nullptr;
  int64_t fe = a.mesh_num_faces[n];
  if (bins.count) {
    const int b = (n * bins.ny + row0 / bins.bs) * bins.nx + col0 / bins.bs;
    const int c = bins.count[b];
    if (c <= bins.cap) { ids = bins.list + (int64_t)b * bins.cap; fe = c; }
  }
  constexpr bool clip = CLIP;
  const float blur = a.blur_radius_dev ? *a.blur_radius_dev : a.blur_radius, sqrt_blur = sqrtf(blur);
  // the pixel's queue state, replicated in its SL lanes
  int qs = 0;
  float qlast_z = __builtin_inff();
  int qlast_f = 0x7fffffff;
  int64_t base = 0;  // position in the cull list (face fb + base, or ids[base])
#ifdef PR_RAST_PROFILE
  long long stamp[6] = {0, 0, 0, 0, 0, 0}, t_ = __builtin_amdgcn_s_memtime();
  const long long rt0 = __builtin_amdgcn_s_memrealtime();
  int nlist = 0, n_app = 0, n_ins = 0, w_ins = 0;
#endif
  while (base < fe) {
    // ---- gather this round's culled faces (expanded bbox overlaps the tile): kCullU
    //      chunks' boxes in flight at once, appended in face order without atomics; a
    //      chunk that would overflow the round's list starts the next round (wave 0)
    int nl = 0;
    while (wv == 0 && base < fe && nl <= kCap - 64) {
      uint2 pb[kCullU];  // packed fp16 boxes: half the registers of unpacked ones
      int fi[kCullU];
#pragma unroll
      for (int u = 0; u < kCullU; ++u) {
        const int64_t i = base + u * 64 + lane;
        const int64_t ic = i < fe ? i : fe - 1;
        fi[u] = ids ? ids[ic] : (int)(fb + ic);
      }
#pragma unroll
      for (int u = 0; u < kCullU; ++u) pb[u] = fbox[fi[u]];
      int64_t next = base + 64 * kCullU;
      bool stop = false;  // wave-uniform; no break, so bb[] stays in registers
#pragma unroll
      for (int u = 0; u < kCullU; ++u) {
        const int64_t i = base + u * 64 + lane;
        const float4 bb = unpack_box(pb[u]);
        const bool keep = i < fe && !(bb.x > txmax || bb.y < txmin || bb.z > tymax || bb.w < tymin);
        const uint64_t bal = __ballot(keep);
        const int cnt = __popcll(bal);
        if (!stop && nl + cnt > kCap) { stop = true; next = base + u * 64; }
        if (!stop) {
          if (keep) lfid[nl + __popcll(bal & ((1ull << lane) - 1ull))] = fi[u];
          nl += cnt;
        }
      }
      base = next < fe ? next : fe;
    }
    if constexpr (NW > 1) {  // the round's list size and next cull position to the other wave
      if (tid == 0) { lctl[0] = base; lctl[1] = nl; }
      __syncthreads();
      base = lctl[0];
      nl = (int)lctl[1];
    }
    __syncthreads();
    PR_STAMP(0);
#ifdef PR_RAST_PROFILE
    nlist += nl;
#endif
    if (nl == 0) continue;
    if (ring & 2) {  // critical-path priority: the tiles with the longest face lists bound the kernel
      const int t = ring >> 8;  // levels at t, t + 16, t + 32 faces
      if (nl >= t + 32) __builtin_amdgcn_s_setprio(3);
      else if (nl >= t + 16) __builtin_amdgcn_s_setprio(2);
      else if (nl >= t) __builtin_amdgcn_s_setprio(1);
    }
    bool done = !inimg;  // the early exit below is only valid inside one sorted round
    // ---- sort key: the face plane's depth at the tile centre, clamped to the face's
    //      z range (an ordering heuristic only: it makes the per-pixel inserts mostly
    //      appends).  Exactness does not depend on it; the early exit uses z_min.
    int n2 = 64;
    while (n2 < nl) n2 <<= 1;
    for (int i = tid; i < n2; i += NT) {
      float key = __builtin_inff();
      if (i < nl) {
        const FaceRec& r = faces[lfid[i]];
        const float4 ra = r.a, rb = r.b, re = r.e, rf = r.f;
        const float z2 = r.c.x, area = r.d.y;
        const float e0 = (tcx - ra.w) * re.w - (tcy - rb.x) * re.z;
        const float e1 = (tcx - rb.z) * rf.y - (tcy - rb.w) * rf.x;
        const float e2 = (tcx - ra.x) * re.y - (tcy - ra.y) * re.x;
        const float ia = 1.f / area;
        const float zc = (e0 * ia) * ra.z + (e1 * ia) * rb.y + (e2 * ia) * z2;
        const float zmx = fmaxf(ra.z, fmaxf(rb.y, z2));
        key = fminf(fmaxf(zc, rf.w), zmx);
        if (key != key) key = rf.w;
        key = fminf(key, 3.0e38f);  // real faces sort before the +inf padding
        if (key != key) key = 0.f;
      }
      lkey[i] = key;
      lidx[i] = i < nl ? i : 0x7fffffff;
    }
    __syncthreads();
    PR_STAMP(1);
    if (wv == 0) {
      if (n2 == 64) wave_sort_lds<1>(lkey, lidx, lane);
      else if (kCap >= 128 && n2 == 128) wave_sort_lds<2>(lkey, lidx, lane);
      else if (kCap >= 256 && n2 == 256) wave_sort_lds<4>(lkey, lidx, lane);
      else if constexpr (kCap >= 512) wave_sort_lds<8>(lkey, lidx, lane);
    }
    __syncthreads();
    PR_STAMP(2);
    // suffix minimum of z_min along the sorted order (faces after position i cannot
    // produce pz below lsuf[i] when barycentrics are clipped)
    {
      const int per = (nl + 63) / 64;  // contiguous run of sorted positions per lane (wave 0)
      const int i0 = lane * per, i1 = wv == 0 ? min(nl, i0 + per) : i0;
      float zl[8];  // z_min of this lane's run (per <= kCap / 64)
#pragma unroll
      for (int u = 0; u < 8; ++u) zl[u] = i0 + u < i1 ? faces[lfid[lidx[i0 + u]]].f.w : __builtin_inff();
      float m = __builtin_inff();
#pragma unroll
      for (int u = 0; u < 8; ++u) m = fminf(m, zl[u]);
      // exclusive suffix-min across lanes (lanes above this one)
      float ex = m;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float t = __shfl_down(ex, o);
        if (lane + o < 64) ex = fminf(ex, t);
      }
      float run = __shfl_down(ex, 1);
      if (lane == 63) run = __builtin_inff();
      __syncthreads();  // lsuf aliases lkey: every lane is past its sorted reads
#pragma unroll
      for (int u = 7; u >= 0; --u) {
        run = fminf(run, zl[u]);
        if (i0 + u < i1) lsuf[i0 + u] = run;
      }
    }
    __syncthreads();
    PR_STAMP(3);
    // ---- traversal in chunks of CH sorted positions; the chunk's records are gathered
    //      one chunk ahead (registers), so the global latency of chunk c+1 overlaps the
    //      tests of chunk c
    float4 nra, nrb, nrc, nrd, nre, nrf;  // next chunk's record (explicit registers: no scratch)
    int nfid = 0;
    float nsuf = 0.f;
    if (lane < CH) {
      const int sp = min(wv * CH + lane, nl - 1);
      nfid = lfid[lidx[sp]];
      nsuf = lsuf[sp];
      const FaceRec* fp = faces + nfid;
      nra = fp->a; nrb = fp->b; nrc = fp->c; nrd = fp->d; nre = fp->e; nrf = fp->f;
    }
    for (int c0 = wv * CH; c0 < nl && __ballot(!done) != 0; c0 += NW * CH) {
      const int cnt = min(CH, nl - c0);
      __builtin_amdgcn_wave_barrier();
      if (lane < cnt) {
        FaceRec& d = lrec[lane];
        d.a = nra; d.b = nrb; d.c = nrc; d.d = nrd; d.e = nre; d.f = nrf;
        lcf[lane] = nfid;
        lcs[lane] = nsuf;
        if constexpr (!PERSP) lmg[lane] = dist_margin(nra, nrb, ptile, sqrt_blur, blur);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (c0 + NW * CH < nl && lane < CH) {
        const int sp = c0 + NW * CH + min(lane, nl - c0 - NW * CH - 1);
        nfid = lfid[lidx[sp]];
        nsuf = lsuf[sp];
        const FaceRec* fp = faces + nfid;
        nra = fp->a; nrb = fp->b; nrc = fp->c; nrd = fp->d; nre = fp->e; nrf = fp->f;
      }
      const int steps = (cnt + SL - 1) / SL;  // positions per slice in this chunk (upper bound)
      for (int t = 0; t < steps; t += kGroup) {
        bool cand[kGroup], ok[kGroup];
        float pzv[kGroup];
        int idx[kGroup];
        FaceRec rr[kGroup];
        bool any = false;
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
          idx[j] = (t + j) * SL + slice;
          ok[j] = idx[j] < cnt;
          rr[j] = lrec[min(idx[j], cnt - 1)];  // one LDS wait per group
        }
        bool maybe[kGroup];
        float dfast[kGroup], mg[kGroup];
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
          // the cheap certain-reject stage (non-perspective; the box test otherwise)
          dfast[j] = 0.f;
          mg[j] = PERSP ? 0.f : lmg[min(idx[j], cnt - 1)];
          if constexpr (PERSP) maybe[j] = ok[j] && in_bbox(rr[j], p);
          else maybe[j] = ok[j] && face_maybe(rr[j], p, blur, mg[j], dfast[j]);
          any |= __ballot(maybe[j]) != 0;
        }
        if (!any) continue;
#ifdef PR_RAST_PROFILE
        const int ins_before = n_ins;
#endif
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
          if constexpr (PERSP) cand[j] = face_test<PERSP, CLIP>(rr[j], p, blur, pzv[j]) && maybe[j];
          else cand[j] = face_test_kept<CLIP>(rr[j], p, blur, mg[j], dfast[j], pzv[j]) && maybe[j];
        }
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
          // clipped barycentrics make pz a convex combination of the vertex depths, so
          // pz >= z_min for this and every later face of the slice (up to rounding:
          // 1e-6 margin)
          const float zk = lcs[min(idx[j], cnt - 1)];
          const int fid = lcf[min(idx[j], cnt - 1)];
          if constexpr (SL > 1) {
            // ---- batch path: when every candidate of the wave is an append (the common
            //      case, faces arrive in depth order), a pixel's SL candidates enter its
            //      queue together, each at qs + its rank among them; else the candidates
            //      merge into the queues (PR_RAST_MERGE; the r1 path inserted slice by slice
            //      below).  Same queue either way (the K smallest keys, sorted).
            if (ok[j] && clip && qs == K && zk > qlast_z + fabsf(qlast_z) * 1e-6f) done = true;
            const float pz = pzv[j];
            const bool enter = ok[j] && !done && cand[j] && (qs < K || key_less(pz, fid, qlast_z, qlast_f));
            const bool app = enter && (qs == 0 || key_less(qlast_z, qlast_f, pz, fid));
            const bool slow = __ballot(enter && !app) != 0;
#if PR_RAST_MERGE
            if (__ballot(enter) == 0) continue;
            {
#else
            if (!slow) {
              if (__ballot(enter) == 0) continue;
#endif
              bool oe[SL - 1];
              float oz[SL - 1];
              int of[SL - 1];
              int rank = 0, nq = enter ? 1 : 0;
#pragma unroll
              for (int r = 1; r < SL; ++r) {
                oe[r - 1] = quad_rot<SL>((int)enter, r) != 0;
                oz[r - 1] = __int_as_float(quad_rot<SL>(__float_as_int(pz), r));
                of[r - 1] = quad_rot<SL>(fid, r);
                nq += oe[r - 1] ? 1 : 0;
                rank += (enter && oe[r - 1] && key_less(oz[r - 1], of[r - 1], pz, fid)) ? 1 : 0;
              }
#if PR_RAST_MERGE
              if (slow) {
                // ---- merge path: some candidate of the wave lands inside its pixel's queue.
                //      Each candidate's final position is (queue keys below it) + (its rank
                //      among the pixel's entering candidates); the queue entries at or above
                //      the lowest landing point move up by the number of candidates below
                //      them, the pixel's SL lanes sharing the moves (top down: every write
                //      lands at or above the reads still to come).  Entries pushed to K or
                //      beyond drop off.  Same queue as inserting one candidate at a time.
                int below = qs;
                if (enter && !app) {  // key below the queue's last: binary search in [0, qs - 1]
                  int lo = 0, hi = qs - 1;
                  while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    const float2 e = q[mid * QS + pix];
                    if (key_less(e.x, __float_as_int(e.y), pz, fid)) lo = mid + 1;
                    else hi = mid;
                  }
                  below = lo;
                }
                int pmin = enter ? below : qs;
#pragma unroll
                for (int r = 1; r < SL; ++r) pmin = min(pmin, quad_rot<SL>(pmin, r));
                for (int i = qs - 1 - slice; i >= pmin; i -= 2 * SL) {
                  const bool two = i - SL >= pmin;
                  const float2 e0 = q[i * QS + pix];
                  const float2 e1 = q[(two ? i - SL : i) * QS + pix];
                  int s0 = enter && key_less(pz, fid, e0.x, __float_as_int(e0.y)) ? 1 : 0;
                  int s1 = enter && key_less(pz, fid, e1.x, __float_as_int(e1.y)) ? 1 : 0;
#pragma unroll
                  for (int r = 0; r < SL - 1; ++r) {
                    s0 += oe[r] && key_less(oz[r], of[r], e0.x, __float_as_int(e0.y)) ? 1 : 0;
                    s1 += oe[r] && key_less(oz[r], of[r], e1.x, __float_as_int(e1.y)) ? 1 : 0;
                  }
                  if (i + s0 < K) q[(i + s0) * QS + pix] = e0;
                  if (two && i - SL + s1 < K) q[(i - SL + s1) * QS + pix] = e1;
                }
                const int pos = below + rank;
                if (enter && pos < K) q[pos * QS + pix] = make_float2(pz, __int_as_float(fid));
                qs = min(qs + nq, K);
                if (qs > 0) {
                  const float2 last = q[(qs - 1) * QS + pix];
                  qlast_z = last.x;
                  qlast_f = __float_as_int(last.y);
                }
#ifdef PR_RAST_PROFILE
                n_ins += enter && !app ? 1 : 0;
                n_app += enter && app ? 1 : 0;
#endif
                continue;
              }
#endif
              const int nkept = min(nq, K - qs);  // the largest ones drop off a full queue
              if (enter && rank < nkept) q[(qs + rank) * QS + pix] = make_float2(pz, __int_as_float(fid));
              if (nkept > 0) {  // new last key: the entered one of rank nkept - 1
                const bool last = enter && rank == nkept - 1;
                float lz = pz;
                int lf = fid;
#pragma unroll
                for (int r = 1; r < SL; ++r) {
                  if (quad_rot<SL>((int)last, r) != 0) { lz = oz[r - 1]; lf = of[r - 1]; }
                }
                qlast_z = lz;
                qlast_f = lf;
                qs += nkept;
              }
#ifdef PR_RAST_PROFILE
              n_app += enter && rank < nkept ? 1 : 0;
#endif
              continue;
            }
          }
#pragma unroll
          for (int sl = 0; sl < SL; ++sl) {
            const bool mine = slice == sl && ok[j];
            if (mine && clip && qs == K && zk > qlast_z + fabsf(qlast_z) * 1e-6f) done = true;
            const float pz = pzv[j];
            // (qlast_z, qlast_f) = the queue's last (largest) key
            const bool enter = mine && !done && cand[j] && (qs < K || key_less(pz, fid, qlast_z, qlast_f));
            if (__ballot(enter) == 0) continue;  // no queue of the wave changes: no state exchange
            {
              if (enter) {
                if (qs == 0 || key_less(qlast_z, qlast_f, pz, fid)) {
                  // append (the common case: faces arrive roughly in depth order)
                  q[qs * QS + pix] = make_float2(pz, __int_as_float(fid));
                  ++qs;
                  qlast_z = pz;
                  qlast_f = fid;
#ifdef PR_RAST_PROFILE
                  ++n_app;
#endif
                } else {
#ifdef PR_RAST_PROFILE
                  ++n_ins;
#endif
                  int pos = qs < K ? qs : K - 1;
                  if (qs < K) ++qs;
                  // shift the entries greater than the key up by one, reading up to four
                  // of them per LDS round trip
                  while (pos > 0) {
                    float2 e[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) e[i] = q[max(pos - 1 - i, 0) * QS + pix];
                    int sh = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                      if (sh == i && pos - 1 - i >= 0 && key_less(pz, fid, e[i].x, __float_as_int(e[i].y))) {
                        q[(pos - i) * QS + pix] = e[i];
                        sh = i + 1;
                      }
                    }
                    pos -= sh;
                    if (sh < 4) break;
                  }
                  q[pos * QS + pix] = make_float2(pz, __int_as_float(fid));
                  const float2 last = q[(qs - 1) * QS + pix];
                  qlast_z = last.x;
                  qlast_f = __float_as_int(last.y);
                }
              }
            }
            if constexpr (SL > 1) {  // slice sl's queue state to the pixel's other lanes
              qs = from_slice<SL>(qs, sl);
              qlast_z = __int_as_float(from_slice<SL>(__float_as_int(qlast_z), sl));
              qlast_f = from_slice<SL>(qlast_f, sl);
            }
          }
        }
#ifdef PR_RAST_PROFILE
        w_ins += __ballot(n_ins != ins_before) != 0;
#endif
        if (__ballot(!done) == 0) break;
      }
    }
    __syncthreads();
    PR_STAMP(4);
  }
  if (slice == 0) qsz[pix] = inimg ? qs : 0;
  if constexpr (NW == 1) {
    if (slice == 0 && inimg && a.pix_count) a.pix_count[((int64_t)n * H + row) * W + col] = qs;
  }
  __syncthreads();
  // NW = 2: the tile's two queues (each sorted, disjoint faces) and their merged sizes
  const float2* qa = reinterpret_cast<const float2*>(reinterpret_cast<const char*>(lrec) - wv * wbytes + CH * sizeof(FaceRec));
  const float2* qb = reinterpret_cast<const float2*>(reinterpret_cast<const char*>(qa) + wbytes);
  const int* qsa = reinterpret_cast<const int*>(qa + (size_t)K * QS);
  const int* qsb = reinterpret_cast<const int*>(qb + (size_t)K * QS);
  if constexpr (NW == 2) {
    if (wv == 0 && slice == 0 && inimg && a.pix_count)
      a.pix_count[((int64_t)n * H + row) * W + col] = min(K, qsa[pix] + qsb[pix]);
  }
  // the merged queue's size at tile pixel t, and its k-th smallest key (merge path: i of A's
  // entries are among the k smallest when A[i-1] < B[k-i] and B[k-i-1] < A[i])
  auto msize = [&](int t) { return NW == 2 ? min(K, qsa[t] + qsb[t]) : qsz[t]; };
  auto kth = [&](int t, int k) -> float2 {
    if constexpr (NW == 1) {
      return q[k * QS + t];
    } else {
      const int na = qsa[t], nb = qsb[t];
      int lo = max(0, k - nb), hi = min(k, na);
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ekey_less(qa[mid * QS + t], qb[(k - 1 - mid) * QS + t])) lo = mid + 1;
        else hi = mid;
      }
      const int j = k - lo;
      if (lo >= na) return qb[j * QS + t];
      if (j >= nb) return qa[lo * QS + t];
      const float2 x = qa[lo * QS + t], y = qb[j * QS + t];
      return ekey_less(x, y) ? x : y;
    }
  };
  // ---- coalesced output: each tile row's pixels own a contiguous ncols*K slot range;
  //      the wave walks the tile's rows as one flat index (4 slots per lane in flight)
  {
    const int ncols = min(TW, W - col0), nrows = min(TH, H - row0);
    const int per_row = ncols * K, total = nrows * per_row;
    const float inv_row = 1.f / (float)per_row, inv_k = 1.f / (float)K;
#ifndef PR_RAST_OUTU  // slots per lane in flight in the output pass (sweep knob)
#define PR_RAST_OUTU 4
#endif
    constexpr int U = PR_RAST_OUTU;
    // compacted fragment pass (tiles of <= 16 pixels): the slot walk writes p2f / zbuf and the
    // padded slots' -1s only; the valid slots' barycentrics / distances are then computed one
    // valid slot per lane (a pixel's valid slots are its queue prefix), so no face evaluation
    // runs for a lane group that holds padding -- on a heavy tile half or more of its slots
    constexpr bool kCompact = FRAG && TP <= 16 && PR_RAST_FRAGC;
    // PR_RAST_VALID_ONLY (counts written): the padding is not written at all; the compacted pass
    // below writes the valid slots' p2f / zbuf with their barycentrics and distances
    const bool valid_only = kCompact && a.pix_count && (a.flags & PR_RAST_VALID_ONLY);
    for (int base = 0; base < (valid_only ? 0 : total); base += NT * U) {
      float2 e[U];
      int sz[U], kk[U], cc[U], rr[U];
      int64_t o[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(base + u * NT + tid, total - 1);
        int rem;
        rr[u] = divmod_small(i, per_row, inv_row, rem);
        cc[u] = divmod_small(rem, K, inv_k, kk[u]);
        const int tl = rr[u] * TW + cc[u];
        o[u] = (((int64_t)n * H + row0 + rr[u]) * W + col0) * K + rem;
        sz[u] = msize(tl);
        if constexpr (NW == 1) e[u] = q[kk[u] * QS + tl];  // read with the size (stale beyond it, unused)
        else e[u] = kk[u] < sz[u] ? kth(tl, kk[u]) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (base + u * NT + tid >= total) break;
        const bool valid = kk[u] < sz[u];
        const int fid = __float_as_int(e[u].y);
        a.pix_to_face[o[u]] = valid ? (int64_t)fid : (int64_t)-1;
        a.zbuf[o[u]] = valid ? e[u].x : -1.f;
        if constexpr (kCompact) {
          if (!valid) {
            a.dists[o[u]] = -1.f;
            a.bary[o[u] * 3 + 0] = -1.f;
            a.bary[o[u] * 3 + 1] = -1.f;
            a.bary[o[u] * 3 + 2] = -1.f;
          }
        } else if constexpr (FRAG) {
          float bc[3] = {-1.f, -1.f, -1.f}, dist = -1.f;
          if (valid) {
            const V2 pp{ndc(W - 1 - (col0 + cc[u]), W, H), ndc(H - 1 - (row0 + rr[u]), H, W)};
            const FaceRec r = faces[fid];
            float pz, d;
            bool inside;
            face_eval<PERSP, CLIP>(r, pp, bc, pz, inside, d);
            dist = inside ? -d : d;
          }
          a.dists[o[u]] = dist;
          a.bary[o[u] * 3 + 0] = bc[0];
          a.bary[o[u] * 3 + 1] = bc[1];
          a.bary[o[u] * 3 + 2] = bc[2];
        }
      }
    }
    if constexpr (kCompact) {
      // valid slot v belongs to the pixel t with ex[t] <= v < ex[t] + qsz[t] (ex: exclusive
      // prefix of the queue sizes over the tile's pixels, wave-uniform), at queue position v - ex[t]
      const int mysz = lane < TP ? msize(lane) : 0;
      int incl = mysz;
#pragma unroll
      for (int o = 1; o < TP; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
      }
      const int excl = incl - mysz;
      int ex[TP];
#pragma unroll
      for (int t = 0; t < TP; ++t) ex[t] = __builtin_amdgcn_readlane(excl, t);
      const int nvalid = __builtin_amdgcn_readlane(incl, TP - 1);
      for (int vb = 0; vb < nvalid; vb += NT * U) {
        float2 e[U];
        int tl[U], kk[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int v = min(vb + u * NT + tid, nvalid - 1);
          int t = 0, e0 = 0;
#pragma unroll
          for (int s = 1; s < TP; ++s) {
            const bool ge = v >= ex[s];
            t = ge ? s : t;
            e0 = ge ? ex[s] : e0;
          }
          tl[u] = t;
          kk[u] = v - e0;
          e[u] = kth(t, kk[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (vb + u * NT + tid >= nvalid) break;
          const int fid = __float_as_int(e[u].y);
          const int rr = tl[u] / TW, cc = tl[u] % TW;
          const int64_t o = (((int64_t)n * H + row0 + rr) * W + col0 + cc) * K + kk[u];
          const V2 pp{ndc(W - 1 - (col0 + cc), W, H), ndc(H - 1 - (row0 + rr), H, W)};
          const FaceRec r = faces[fid];
          float bc[3], pz, d;
          bool inside;
          face_eval<PERSP, CLIP>(r, pp, bc, pz, inside, d);
          if (valid_only) {
            a.pix_to_face[o] = (int64_t)fid;
            a.zbuf[o] = e[u].x;
          }
          a.dists[o] = inside ? -d : d;
          a.bary[o * 3 + 0] = bc[0];
          a.bary[o * 3 + 1] = bc[1];
          a.bary[o * 3 + 2] = bc[2];
        }
      }
    }
  }
#ifdef PR_RAST_PROFILE
  __syncthreads();
  PR_STAMP(5);
  int n_app_tot = n_app, n_ins_tot = n_ins;
  for (int o = 32; o > 0; o >>= 1) { n_app_tot += __shfl_xor(n_app_tot, o); n_ins_tot += __shfl_xor(n_ins_tot, o); }
  if (tid == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const unsigned t = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (t < kProfTiles) {
      long long* rec = g_rast_prof + (size_t)t * 16;
      rec[0] = tile_x; rec[1] = tile_y; rec[2] = blockIdx.z; rec[3] = nlist;
      rec[4] = rt0; rec[5] = (long long)__builtin_amdgcn_s_memrealtime();
      rec[6] = (long long)hw | ((long long)(xcc & 0xf) << 32);
      for (int i = 0; i < 6; ++i) rec[7 + i] = stamp[i];
      rec[13] = SL;
      rec[14] = n_app_tot;
      rec[15] = ((long long)n_ins_tot << 32) | (unsigned)w_ins;
    }
  }
#endif
}

template <int SL, bool PERSP, bool CLIP>
void launch_rast_fwd_sl(const PRRastArgs& a, const FaceRec* fr, const uint2* fb, bool frag, size_t lds,
                        const BinGrid& bins, hipStream_t st, int nw) {
  constexpr int TW = SL >= 4 ? 4 : 8, TH = 64 / SL / TW;
  dim3 grid((a.W + TW - 1) / TW, (a.H + TH - 1) / TH, a.N);
  // centre-out tile order on square grids of even side (PR_RAST_ORDER bit 0; 0: row-major)
  static const bool ring_env = (getenv("PR_RAST_ORDER") ? atoi(getenv("PR_RAST_ORDER")) : 3) & 1;
  // wave priority raised for long face lists (PR_RAST_PRIO=0: off)
  static const bool prio_env = getenv("PR_RAST_PRIO") ? atoi(getenv("PR_RAST_PRIO")) != 0 : true;
  static const int prio_t = getenv("PR_RAST_PRIO_T") ? atoi(getenv("PR_RAST_PRIO_T")) & 255 : 40;
  const bool sq = grid.x % 2 == 0 && (grid.y == grid.x || grid.y == 2 * grid.x);
  const int ring = (ring_env && sq ? 1 : 0) | (prio_env ? 2 : 0) | (prio_t << 8);
  ktimer_mark(0, "rast_fwd_kernel", st);
  if constexpr (SL == 4) {
    if (nw == 2) {
      if (frag) rast_fwd_kernel<SL, PERSP, CLIP, true, 2><<<grid, 128, lds, st>>>(a, fr, fb, ring, bins);
      else rast_fwd_kernel<SL, PERSP, CLIP, false, 2><<<grid, 128, lds, st>>>(a, fr, fb, ring, bins);
      ktimer_mark(1, "rast_fwd_kernel", st);
      return;
    }
  }
  if (frag) rast_fwd_kernel<SL, PERSP, CLIP, true, 1><<<grid, 64, lds, st>>>(a, fr, fb, ring, bins);
  else rast_fwd_kernel<SL, PERSP, CLIP, false, 1><<<grid, 64, lds, st>>>(a, fr, fb, ring, bins);
  ktimer_mark(1, "rast_fwd_kernel", st);
}

template <bool PERSP, bool CLIP>
void launch_rast_fwd_pc(const PRRastArgs& a, const FaceRec* fr, const uint2* fb, int sl, bool frag, size_t lds,
                        const BinGrid& bins, hipStream_t st, int nw) {
  if (sl == 8) launch_rast_fwd_sl<8, PERSP, CLIP>(a, fr, fb, frag, lds, bins, st, 1);
  else if (sl == 4) launch_rast_fwd_sl<4, PERSP, CLIP>(a, fr, fb, frag, lds, bins, st, nw);
  else if (sl == 2) launch_rast_fwd_sl<2, PERSP, CLIP>(a, fr, fb, frag, lds, bins, st, 1);
  else launch_rast_fwd_sl<1, PERSP, CLIP>(a, fr, fb, frag, lds, bins, st, 1);
}

void launch_rast_fwd(const PRRastArgs& a, const FaceRec* fr, const uint2* fb, int sl, bool frag, size_t lds,
                     const BinGrid& bins, hipStream_t st, int nw) {
  const bool persp = a.perspective_correct != 0, clip = a.clip_barycentric_coords != 0;
  if (persp && clip) launch_rast_fwd_pc<true, true>(a, fr, fb, sl, frag, lds, bins, st, nw);
  else if (persp) launch_rast_fwd_pc<true, false>(a, fr, fb, sl, frag, lds, bins, st, nw);
  else if (clip) launch_rast_fwd_pc<false, true>(a, fr, fb, sl, frag, lds, bins, st, nw);
  else launch_rast_fwd_pc<false, false>(a, fr, fb, sl, frag, lds, bins, st, nw);
}

// Forward, pass 2: barycentrics (perspective-corrected, clipped) and signed squared
// distances of every slot, one lane per slot.
template <bool WIDE>
__global__ void __launch_bounds__(kThreads) rast_frag_kernel(PRRastArgs a, int64_t total) {
  using idx_t = typename std::conditional<WIDE, int64_t, uint32_t>::type;
  const bool persp = a.perspective_correct != 0, clip = a.clip_barycentric_coords != 0;
  for (int64_t oo = (int64_t)blockIdx.x * kThreads + threadIdx.x; oo < total; oo += (int64_t)gridDim.x * kThreads) {
    const idx_t o = (idx_t)oo;
    const int64_t fid = a.pix_to_face[o];
    float bc[3] = {-1.f, -1.f, -1.f}, dist = -1.f;
    if (fid >= 0) {
      const idx_t pix = o / (idx_t)a.K;
      const int col = (int)(pix % (idx_t)a.W), row = (int)((pix / (idx_t)a.W) % (idx_t)a.H);
      const V2 pp{ndc(a.W - 1 - col, a.W, a.H), ndc(a.H - 1 - row, a.H, a.W)};
      const float* v = a.face_verts + fid * 9;
      const V2 v0{v[0], v[1]}, v1{v[3], v[4]}, v2{v[6], v[7]};
      float b0[3], b[3];
      bary_fwd(pp, v0, v1, v2, b0);
      if (persp) persp_fwd(b0, v[2], v[5], v[8], b); else { b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2]; }
      if (clip) clip_fwd(b, bc); else { bc[0] = b[0]; bc[1] = b[1]; bc[2] = b[2]; }
      const bool inside = b[0] > 0.f && b[1] > 0.f && b[2] > 0.f;
      const float d = tri_dist2(pp, v0, v1, v2);
      dist = inside ? -d : d;
    }
    a.dists[o] = dist;
    a.bary[o * 3 + 0] = bc[0];
    a.bary[o * 3 + 1] = bc[1];
    a.bary[o * 3 + 2] = bc[2];
  }
}

// ------------------------------------------------------------------ backward
// d/d(p, a, b) of the squared point-segment distance, t held fixed (PyTorch3D form)
PR_DEV void seg_dist2_bwd(V2 p, V2 a, V2 b, float g, V2& ga, V2& gb) {
  const float bax = b.x - a.x, bay = b.y - a.y;
  const float l2 = bax * bax + bay * bay;
  float t;
  if (l2 <= kEps) t = 1.f;
  else {
    t = dv<true>(bax * (p.x - a.x) + bay * (p.y - a.y), l2);
    t = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
  }
  const float qx = (1.f - t) * a.x + t * b.x, qy = (1.f - t) * a.y + t * b.y;
  const float dx = qx - p.x, dy = qy - p.y;
  ga.x = g * (1.f - t) * 2.f * dx; ga.y = g * (1.f - t) * 2.f * dy;
  gb.x = g * t * 2.f * dx;         gb.y = g * t * 2.f * dy;
}

PR_DEV void tri_dist2_bwd(V2 p, V2 v0, V2 v1, V2 v2, float g, V2 gv[3]) {
  const float e01 = seg_dist2(p, v0, v1), e02 = seg_dist2(p, v0, v2), e12 = seg_dist2(p, v1, v2);
  gv[0] = V2{0.f, 0.f}; gv[1] = V2{0.f, 0.f}; gv[2] = V2{0.f, 0.f};
  if (e01 <= e02 && e01 <= e12) seg_dist2_bwd(p, v0, v1, g, gv[0], gv[1]);
  else if (e02 <= e01 && e02 <= e12) seg_dist2_bwd(p, v0, v2, g, gv[0], gv[2]);
  else seg_dist2_bwd(p, v1, v2, g, gv[1], gv[2]);
}

// edge_fn(p, a, b) partials w.r.t. a and b
PR_DEV void edge_bwd(V2 p, V2 a, V2 b, float g, V2& ga, V2& gb) {
  ga.x += g * (p.y - b.y);
  ga.y += g * (b.x - p.x);
  gb.x += g * (a.y - p.y);
  gb.y += g * (p.x - a.x);
}

// b_i = e_i / area, e0 = E(p,v1,v2), e1 = E(p,v2,v0), e2 = E(p,v0,v1), area = E(v2,v0,v1) + eps
PR_DEV void bary_bwd(V2 p, V2 v0, V2 v1, V2 v2, const float gb[3], V2 gv[3]) {
  const float area = edge_fn(v2, v0, v1) + kEps;
  const float e0 = edge_fn(p, v1, v2), e1 = edge_fn(p, v2, v0), e2 = edge_fn(p, v0, v1);
  const float ia = __builtin_amdgcn_rcpf(area);
  const float de0 = gb[0] * ia, de1 = gb[1] * ia, de2 = gb[2] * ia;
  const float darea = -(gb[0] * e0 + gb[1] * e1 + gb[2] * e2) * (ia * ia);
  V2 g0{0.f, 0.f}, g1{0.f, 0.f}, g2{0.f, 0.f};
  edge_bwd(p, v1, v2, de0, g1, g2);
  edge_bwd(p, v2, v0, de1, g2, g0);
  edge_bwd(p, v0, v1, de2, g0, g1);
  // area = E(v2, v0, v1): also depends on its first argument v2
  {
    const V2 a = v0, b = v1, q = v2;
    g0.x += darea * (q.y - b.y);  g0.y += darea * (b.x - q.x);
    g1.x += darea * (a.y - q.y);  g1.y += darea * (q.x - a.x);
    g2.x += darea * (b.y - a.y);  g2.y += darea * (a.x - b.x);
  }
  gv[0] = g0; gv[1] = g1; gv[2] = g2;
}

// o_i = t_i / sum t, t0 = b0 z1 z2, t1 = z0 b1 z2, t2 = z0 z1 b2 (sum clamped at eps)
PR_DEV void persp_bwd(const float b[3], float z0, float z1, float z2, const float go[3], float gb[3], float gz[3]) {
  const float t0 = b[0] * z1 * z2, t1 = z0 * b[1] * z2, t2 = z0 * z1 * b[2];
  const float s = t0 + t1 + t2;
  float gt[3];
  if (s > kEps) {
    const float is = __builtin_amdgcn_rcpf(s);
    const float dot = (go[0] * t0 + go[1] * t1 + go[2] * t2) * (is * is);
    gt[0] = go[0] * is - dot; gt[1] = go[1] * is - dot; gt[2] = go[2] * is - dot;
  } else {
    gt[0] = go[0] * 1e8f; gt[1] = go[1] * 1e8f; gt[2] = go[2] * 1e8f;
  }
  gb[0] = gt[0] * z1 * z2; gb[1] = gt[1] * z0 * z2; gb[2] = gt[2] * z0 * z1;
  gz[0] = gt[1] * b[1] * z2 + gt[2] * z1 * b[2];
  gz[1] = gt[0] * b[0] * z2 + gt[2] * z0 * b[2];
  gz[2] = gt[0] * b[0] * z1 + gt[1] * z0 * b[1];
}

// o_i = max(b_i,0) / max(sum, 1e-5)
PR_DEV void clip_bwd(const float b[3], const float go[3], float gb[3]) {
  const float w0 = b[0] > 0.f ? b[0] : 0.f, w1 = b[1] > 0.f ? b[1] : 0.f, w2 = b[2] > 0.f ? b[2] : 0.f;
  const float s = w0 + w1 + w2;
  float gw[3];
  if (s > 1e-5f) {
    const float is = __builtin_amdgcn_rcpf(s);
    const float dot = (go[0] * w0 + go[1] * w1 + go[2] * w2) * (is * is);
    gw[0] = go[0] * is - dot; gw[1] = go[1] * is - dot; gw[2] = go[2] * is - dot;
  } else {
    gw[0] = go[0] * 1e5f; gw[1] = go[1] * 1e5f; gw[2] = go[2] * 1e5f;
  }
  gb[0] = b[0] > 0.f ? gw[0] : 0.f;
  gb[1] = b[1] > 0.f ? gw[1] : 0.f;
  gb[2] = b[2] > 0.f ? gw[2] : 0.f;
}

PR_DEV void slot_grad(const PRRastArgs& a, V2 p, const float* v, int64_t o, float g[9]) {
  const V2 v0{v[0], v[1]}, v1{v[3], v[4]}, v2{v[6], v[7]};
  const float z0 = v[2], z1 = v[5], z2 = v[8];
  const bool persp = a.perspective_correct != 0, clip = a.clip_barycentric_coords != 0;
  const float gzb = a.grad_zbuf ? a.grad_zbuf[o] : 0.f;
  const float gd = a.grad_dists ? a.grad_dists[o] : 0.f;
  float gbu[3] = {0.f, 0.f, 0.f};
  if (a.grad_bary) { gbu[0] = a.grad_bary[o * 3]; gbu[1] = a.grad_bary[o * 3 + 1]; gbu[2] = a.grad_bary[o * 3 + 2]; }
  float bw[3], bp[3], bc[3];
  bary_fwd(p, v0, v1, v2, bw);
  // bw is exact (its signs decide inside / clip masks as in the forward); the rest
  // only feeds gradient arithmetic
  if (persp) persp_fwd<true>(bw, z0, z1, z2, bp); else { bp[0] = bw[0]; bp[1] = bw[1]; bp[2] = bw[2]; }
  if (clip) clip_fwd<true>(bp, bc); else { bc[0] = bp[0]; bc[1] = bp[1]; bc[2] = bp[2]; }
  const bool inside = bp[0] > 0.f && bp[1] > 0.f && bp[2] > 0.f;
  V2 gdv[3];
  tri_dist2_bwd(p, v0, v1, v2, inside ? -gd : gd, gdv);
  // zbuf = sum_i bc_i z_i
  float gsum[3] = {gbu[0] + gzb * z0, gbu[1] + gzb * z1, gbu[2] + gzb * z2};
  float gpp[3] = {gsum[0], gsum[1], gsum[2]};
  if (clip) clip_bwd(bp, gsum, gpp);
  float gw[3] = {gpp[0], gpp[1], gpp[2]};
  float gz[3] = {0.f, 0.f, 0.f};
  if (persp) persp_bwd(bw, z0, z1, z2, gpp, gw, gz);
  V2 gbv[3];
  bary_bwd(p, v0, v1, v2, gw, gbv);
  g[0] = gbv[0].x + gdv[0].x; g[1] = gbv[0].y + gdv[0].y; g[2] = gzb * bc[0] + gz[0];
  g[3] = gbv[1].x + gdv[1].x; g[4] = gbv[1].y + gdv[1].y; g[5] = gzb * bc[1] + gz[1];
  g[6] = gbv[2].x + gdv[2].x; g[7] = gbv[2].y + gdv[2].y; g[8] = gzb * bc[2] + gz[2];
}

// ---- exact slot gradient: oracle/rast_oracle.c rast_bwd's operations in its order (PyTorch3D's
// CPU backward): IEEE divisions, one accumulator per vertex component with the distance terms
// first, then the barycentric terms edge by edge, then the area terms.  A slot's contribution is
// the oracle's bit for bit; summed per face in slot order (PR_DETERMINISTIC) the face gradients
// are the oracle's bits.
PR_DEV void acc_edge(V2 p, V2 a, V2 b, float g, float* ga, float* gb) {  // edge_fn(p, a, b) partials
  ga[0] += g * (p.y - b.y); ga[1] += g * (b.x - p.x);
  gb[0] += g * (a.y - p.y); gb[1] += g * (p.x - a.x);
}

PR_DEV void acc_seg(V2 p, V2 a, V2 b, float g, float* ga, float* gb) {  // squared segment distance
  const float bax = b.x - a.x, bay = b.y - a.y;
  const float l2 = bax * bax + bay * bay;
  float t = 1.f;
  if (!(l2 <= kEps)) {
    t = (bax * (p.x - a.x) + bay * (p.y - a.y)) / l2;
    t = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
  }
  const float qx = (1.f - t) * a.x + t * b.x, qy = (1.f - t) * a.y + t * b.y;
  const float dx = qx - p.x, dy = qy - p.y;
  ga[0] += g * (1.f - t) * 2.f * dx; ga[1] += g * (1.f - t) * 2.f * dy;
  gb[0] += g * t * 2.f * dx;         gb[1] += g * t * 2.f * dy;
}

PR_DEV void slot_grad_exact(const PRRastArgs& a, V2 p, const float* v, int64_t o, float out[9]) {
  const V2 v0{v[0], v[1]}, v1{v[3], v[4]}, v2{v[6], v[7]};
  const float z0 = v[2], z1 = v[5], z2 = v[8];
  const bool persp = a.perspective_correct != 0, clip = a.clip_barycentric_coords != 0;
  const float gzb = a.grad_zbuf ? a.grad_zbuf[o] : 0.f;
  const float gd = a.grad_dists ? a.grad_dists[o] : 0.f;
  float gbu[3] = {0.f, 0.f, 0.f};
  if (a.grad_bary) { gbu[0] = a.grad_bary[o * 3]; gbu[1] = a.grad_bary[o * 3 + 1]; gbu[2] = a.grad_bary[o * 3 + 2]; }
  float bw[3], bp[3], bc[3];
  bary_fwd(p, v0, v1, v2, bw);
  if (persp) persp_fwd(bw, z0, z1, z2, bp); else { bp[0] = bw[0]; bp[1] = bw[1]; bp[2] = bw[2]; }
  if (clip) clip_fwd(bp, bc); else { bc[0] = bp[0]; bc[1] = bp[1]; bc[2] = bp[2]; }
  const bool inside = bp[0] > 0.f && bp[1] > 0.f && bp[2] > 0.f;
  float gv[3][2] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
  {
    const float g = inside ? -gd : gd;
    const float e01 = seg_dist2(p, v0, v1), e02 = seg_dist2(p, v0, v2), e12 = seg_dist2(p, v1, v2);
    if (e01 <= e02 && e01 <= e12) acc_seg(p, v0, v1, g, gv[0], gv[1]);
    else if (e02 <= e01 && e02 <= e12) acc_seg(p, v0, v2, g, gv[0], gv[2]);
    else acc_seg(p, v1, v2, g, gv[1], gv[2]);
  }
  const float gsum[3] = {gbu[0] + gzb * z0, gbu[1] + gzb * z1, gbu[2] + gzb * z2};
  float gpp[3] = {gsum[0], gsum[1], gsum[2]};
  if (clip) {
    const float w0 = bp[0] > 0.f ? bp[0] : 0.f, w1 = bp[1] > 0.f ? bp[1] : 0.f, w2 = bp[2] > 0.f ? bp[2] : 0.f;
    const float s = w0 + w1 + w2;
    float gw[3];
    if (s > 1e-5f) {
      const float dot = (gsum[0] * w0 + gsum[1] * w1 + gsum[2] * w2) / (s * s);
      gw[0] = gsum[0] / s - dot; gw[1] = gsum[1] / s - dot; gw[2] = gsum[2] / s - dot;
    } else {
      gw[0] = gsum[0] / 1e-5f; gw[1] = gsum[1] / 1e-5f; gw[2] = gsum[2] / 1e-5f;
    }
    gpp[0] = bp[0] > 0.f ? gw[0] : 0.f; gpp[1] = bp[1] > 0.f ? gw[1] : 0.f; gpp[2] = bp[2] > 0.f ? gw[2] : 0.f;
  }
  float gw[3] = {gpp[0], gpp[1], gpp[2]}, gzp[3] = {0.f, 0.f, 0.f};
  if (persp) {
    const float t0 = bw[0] * z1 * z2, t1 = z0 * bw[1] * z2, t2 = z0 * z1 * bw[2];
    const float s = t0 + t1 + t2;
    float gt[3];
    if (s > kEps) {
      const float dot = (gpp[0] * t0 + gpp[1] * t1 + gpp[2] * t2) / (s * s);
      gt[0] = gpp[0] / s - dot; gt[1] = gpp[1] / s - dot; gt[2] = gpp[2] / s - dot;
    } else {
      gt[0] = gpp[0] / kEps; gt[1] = gpp[1] / kEps; gt[2] = gpp[2] / kEps;
    }
    gw[0] = gt[0] * z1 * z2; gw[1] = gt[1] * z0 * z2; gw[2] = gt[2] * z0 * z1;
    gzp[0] = gt[1] * bw[1] * z2 + gt[2] * z1 * bw[2];
    gzp[1] = gt[0] * bw[0] * z2 + gt[2] * z0 * bw[2];
    gzp[2] = gt[0] * bw[0] * z1 + gt[1] * z0 * bw[1];
  }
  // barycentric terms: b_i = e_i / area, area = E(v2, v0, v1) + eps
  const float area = edge_fn(v2, v0, v1) + kEps;
  const float e0 = edge_fn(p, v1, v2), e1 = edge_fn(p, v2, v0), e2 = edge_fn(p, v0, v1);
  const float darea = -(gw[0] * e0 + gw[1] * e1 + gw[2] * e2) / (area * area);
  acc_edge(p, v1, v2, gw[0] / area, gv[1], gv[2]);
  acc_edge(p, v2, v0, gw[1] / area, gv[2], gv[0]);
  acc_edge(p, v0, v1, gw[2] / area, gv[0], gv[1]);
  gv[2][0] += darea * (v1.y - v0.y);
  gv[2][1] += darea * (v0.x - v1.x);
  acc_edge(v2, v0, v1, darea, gv[0], gv[1]);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    out[i * 3 + 0] = gv[i][0];
    out[i * 3 + 1] = gv[i][1];
    out[i * 3 + 2] = gzb * bc[i] + gzp[i];
  }
}

template <bool EXACT>
PR_DEV void slot_grad_any(const PRRastArgs& a, V2 p, const float* v, int64_t o, float g[9]) {
  if constexpr (EXACT) slot_grad_exact(a, p, v, o, g);
  else slot_grad(a, p, v, o, g);
}

// ---- deterministic mode (PR_DETERMINISTIC): key every slot by its face (padded slots by F),
// stable-sort, exact slot gradients at their sorted positions, in-order face sums (pr_detsum.hip)
// (one batch of slots [s0, s0 + n): entry i is slot s0 + i)
__global__ void rast_bwd_keys_kernel(PRRastArgs a, uint32_t* keys, int64_t s0, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = s0 + i, pix = o / a.K;
    const bool valid = a.pix_count ? (int)(o - pix * a.K) < a.pix_count[pix] : true;
    const int64_t f = valid ? a.pix_to_face[o] : -1;
    keys[i] = f >= 0 ? (uint32_t)f : (uint32_t)a.F;
  }
}

__global__ void rast_bwd_sorted_grad_kernel(PRRastArgs a, const uint32_t* keys, const uint32_t* idx, float* vals,
                                            int64_t s0, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t f = keys[i];
    if ((int64_t)f >= a.F) continue;
    const int64_t o = s0 + idx[i];
    const int64_t pix = o / a.K;
    const int col = (int)(pix % a.W), row = (int)((pix / a.W) % a.H);
    const V2 p{ndc(a.W - 1 - col, a.W, a.H), ndc(a.H - 1 - row, a.H, a.W)};
    float g[9];
    slot_grad_exact(a, p, a.face_verts + (int64_t)f * 9, o, g);
#pragma unroll
    for (int c = 0; c < 9; ++c) vals[i * 9 + c] = g[c];
  }
}

constexpr int kHash = 512;      // LDS hash entries per workgroup (distinct faces of one tile)
constexpr int kBwdTile = 8;     // tile width; rows per tile (<= 8) chosen at launch
constexpr int kBwdThreads = 256;
#ifndef PR_BWD_ENT  // sweeps: -DPR_BWD_ENT=256 / 1024 measured 46.8 / 77 us vs 44 us at 512
#define PR_BWD_ENT 512
#endif
constexpr int kBwdEnt = PR_BWD_ENT;  // slots scanned (and at most valid) per round: 2 per thread
constexpr int kBwdFaces = 128;  // faces per tile reduced by the transpose; later ones use global atomics

// One 256-thread workgroup per 8 x tile_rows pixel tile (tile_rows <= 8), rounds of
// kBwdEnt slots.  No per-slot atomics on the gradient values (LDS float atomics cost
// ~4 cycles per lane on gfx950, and a slot has 9 components):
//  1. scan: the round's slots (tile rows are contiguous ncols*K slot ranges: coalesced
//     p2f reads) are compacted into an LDS list of the valid ones (wave ballot, one
//     LDS append per wave); each new face id gets a tile-local index through an LDS
//     hash (one CAS per slot, a second atomic per distinct face).
//  2. gradient: one lane per valid slot, densely: the 9 vertex-gradient components go
//     to gbuf[entry] (plain LDS stores) and the entry index to M[face][pixel] (a pixel
//     holds a face at most once, so every (face, pixel) cell has one writer).
//  3. transpose: the owner lane of each tile-local face walks its M row (the tile's
//     pixels) and sums its entries' gbuf rows in registers.
//  4. after the last round the owners' sums go to LDS and the flush adds each (face,
//     component) once to global memory, lane-contiguously (global float atomics run at
//     the memory side; 64 lanes on 64 scattered rows collapse that rate — MI355X guide,
//     Global float atomics).
// Faces past the first kBwdFaces of a tile, and hash overflow, add their slots straight
// to global memory (correct, slower; dense meshes under large tiles only).
template <int ROWS, bool EXACT>
__global__ void __launch_bounds__(kBwdThreads) rast_bwd_kernel(PRRastArgs a, int order) {
  constexpr int tile_rows = ROWS, TP = kBwdTile * ROWS;  // tile pixels
  __shared__ int hkey[kHash];
  __shared__ int hfl[kHash];                      // tile-local face index of a hash entry
  __shared__ int flist[kBwdFaces];                // face id of each tile-local index
  // [pixel / 4][face][pixel % 4] -> entry index of this round: the transpose's owner lanes (one
  // per face) read 4 pixels' entries as one 8-B word at consecutive addresses (the [face][pixel]
  // layout put the lanes 32 B apart: 8-way bank conflicts)
  __shared__ alignas(8) uint16_t M[kBwdFaces * TP];
  __shared__ float gbuf[9 * kBwdEnt];             // [component][entry]; reused for the sums
  __shared__ int2 clist[kBwdEnt];                 // (pixel << 16 | k, face id)
  __shared__ int ccount, nface;
  __shared__ float pxs[kBwdTile], pys[ROWS];
  __shared__ int pcnt[kBwdTile * ROWS];           // valid-prefix counts of the tile's pixels (or K)
  __shared__ int pstart[kBwdTile * ROWS + 1];     // exclusive prefix sum of pcnt
  const int tid = threadIdx.x, lane = tid & 63;
  const int K = a.K, H = a.H, W = a.W;
  const int n = blockIdx.z, col0 = blockIdx.x * kBwdTile;
  const int row0 = (order ? centre_out(blockIdx.y, gridDim.y) : (int)blockIdx.y) * tile_rows;
  const int ncols = min(kBwdTile, W - col0), nrows = min(tile_rows, H - row0);
  const int64_t tile_o = (((int64_t)n * H + row0) * W + col0) * K;  // slot offset of the tile's first row
  const int64_t row_stride = (int64_t)W * K;
  for (int i = tid; i < kHash; i += kBwdThreads) hkey[i] = -1;
  for (int i = tid; i < kBwdFaces * TP; i += kBwdThreads) M[i] = 0xffff;
  if (tid < kBwdTile) pxs[tid] = ndc(W - 1 - min(col0 + tid, W - 1), W, H);
  if (tid >= 64 && tid < 64 + ROWS) pys[tid - 64] = ndc(H - 1 - min(row0 + tid - 64, H - 1), H, W);
  if (tid == 0) nface = 0;
  if (tid < TP) {
    const int r = tid / kBwdTile, c = tid - r * kBwdTile;
    pcnt[tid] = (r < nrows && c < ncols) ? (a.pix_count ? a.pix_count[((int64_t)n * H + row0 + r) * W + col0 + c] : K) : 0;
  }
  __syncthreads();
  if (tid == 0) {
    int acc_s = 0;
    for (int q = 0; q < TP; ++q) { pstart[q] = acc_s; acc_s += pcnt[q]; }
    pstart[TP] = acc_s;
  }
  __syncthreads();
  // the rounds walk the tile's valid-prefix slots only (pixel q's slots 0..pcnt[q]-1 are
  // entries pstart[q].. of the walk): a tile with <= kBwdEnt valid slots is one round
  const int total = pstart[TP];
  float acc[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // owner lane tid < kBwdFaces
  for (int c0 = 0; c0 < total; c0 += kBwdEnt) {
    if (tid == 0) ccount = 0;
    __syncthreads();  // also: the previous round's transpose is done (M reset, gbuf free)
    // ---- 1. scan + compaction + face registration
    int64_t f[kBwdEnt / kBwdThreads];
    int pk[kBwdEnt / kBwdThreads];  // (pixel << 16) | k
#pragma unroll
    for (int u = 0; u < kBwdEnt / kBwdThreads; ++u) {
      const int i = c0 + u * kBwdThreads + tid;
      f[u] = -1;
      pk[u] = 0;
      if (i < total) {
        int q = 0;  // the pixel: last q with pstart[q] <= i (binary search over TP entries)
#pragma unroll
        for (int step = TP / 2; step > 0; step >>= 1)
          if (pstart[q + step] <= i) q += step;
        const int k = i - pstart[q], r = q / kBwdTile, c = q - r * kBwdTile;
        pk[u] = (q << 16) | k;
        f[u] = a.pix_to_face[tile_o + r * row_stride + c * K + k];
      }
    }
#pragma unroll
    for (int u = 0; u < kBwdEnt / kBwdThreads; ++u) {
      const bool keep = f[u] >= 0;
      const uint64_t bal = __ballot(keep);
      if (bal == 0) continue;
      int off = 0;
      if (lane == 0) off = atomicAdd(&ccount, __popcll(bal));
      off = __shfl(off, 0);
      if (!keep) continue;
      const int fi = (int)f[u];
      clist[off + __popcll(bal & ((1ull << lane) - 1ull))] = make_int2(pk[u], fi);
      uint32_t h = ((uint32_t)fi * 2654435761u) & (kHash - 1);
      for (int probe = 0; probe < 32; ++probe) {
        const int cur = atomicCAS(&hkey[h], -1, fi);
        if (cur == -1) {  // first slot of this face in the tile: assign its local index
          const int fl = atomicAdd(&nface, 1);
          hfl[h] = fl;
          if (fl < kBwdFaces) flist[fl] = fi;
          break;
        }
        if (cur == fi) break;
        h = (h + 1) & (kHash - 1);
      }
    }
    __syncthreads();
    // ---- 2. dense per-slot gradients
    const int nv = ccount;
    for (int j = tid; j < nv; j += kBwdThreads) {
      const int2 e = clist[j];
      const int pix = e.x >> 16, k = e.x & 0xffff, fi = e.y;
      const int r = pix >> 3, c = pix & 7;
      const int64_t o = tile_o + r * row_stride + c * K + k;
      const V2 p{pxs[c], pys[r]};
      float g[9];
      slot_grad_any<EXACT>(a, p, a.face_verts + (int64_t)fi * 9, o, g);
      uint32_t h = ((uint32_t)fi * 2654435761u) & (kHash - 1);
      int fl = kBwdFaces;  // not found (hash overflow): global path
      for (int probe = 0; probe < 32; ++probe) {
        const int cur = hkey[h];
        if (cur == fi) { fl = hfl[h]; break; }
        if (cur == -1) break;
        h = (h + 1) & (kHash - 1);
      }
      if (fl < kBwdFaces) {
#pragma unroll
        for (int cc = 0; cc < 9; ++cc) gbuf[cc * kBwdEnt + j] = g[cc];
        M[((pix >> 2) * kBwdFaces + fl) * 4 + (pix & 3)] = (uint16_t)j;
      } else {
#pragma unroll
        for (int cc = 0; cc < 9; ++cc) atomicAdd(&a.grad_face_verts[(int64_t)fi * 9 + cc], g[cc]);
      }
    }
    __syncthreads();
    // ---- 3. transpose: owner lanes sum their face's entries (and reset their M row)
    if (tid < min(nface, kBwdFaces)) {
      uint64_t* col = reinterpret_cast<uint64_t*>(M) + tid;
      for (int q = 0; q < nrows * kBwdTile; q += 4) {
        const uint64_t four = col[(q >> 2) * kBwdFaces];
        if (four == ~0ull) continue;
        col[(q >> 2) * kBwdFaces] = ~0ull;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t jj = (uint32_t)(four >> (16 * t)) & 0xffffu;
          if (jj == 0xffffu) continue;
#pragma unroll
          for (int cc = 0; cc < 9; ++cc) acc[cc] += gbuf[cc * kBwdEnt + jj];
        }
      }
    }
  }
  __syncthreads();
  // ---- 4. flush: sums to LDS, then lane-contiguous over (face, component)
  const int nf = min(nface, kBwdFaces);
  if (tid < nf) {
#pragma unroll
    for (int cc = 0; cc < 9; ++cc) gbuf[tid * 9 + cc] = acc[cc];
  }
  __syncthreads();
  for (int i = tid; i < nf * 9; i += kBwdThreads) {
    const int fl = i / 9, cc = i - fl * 9;
    atomicAdd(&a.grad_face_verts[(int64_t)flist[fl] * 9 + cc], gbuf[i]);
  }
}

// ------------------------------------------------------------ interpolation
// Row offset of corner i of face f in the attribute table: per-face-corner (F,3,D)
// or, with a.faces, per-vertex (V,D) gathered through the face indices.
PR_DEV int64_t attr_row(const PRInterpArgs& a, int64_t f, int i) {
  return a.faces ? a.faces[f * 3 + i] * a.D : (f * 3 + i) * a.D;
}

__global__ void interp_fwd_kernel(PRInterpArgs a) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < a.PK; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = a.pix_to_face[s];
    float* o = a.out + s * a.D;
    if (f < 0) {
      for (int d = 0; d < a.D; ++d) o[d] = 0.f;
      continue;
    }
    const float w0 = a.bary[s * 3], w1 = a.bary[s * 3 + 1], w2 = a.bary[s * 3 + 2];
    const float* r0 = a.face_attr + attr_row(a, f, 0);
    const float* r1 = a.face_attr + attr_row(a, f, 1);
    const float* r2 = a.face_attr + attr_row(a, f, 2);
    for (int d = 0; d < a.D; ++d) o[d] = (w0 * r0[d] + w1 * r1[d]) + w2 * r2[d];
  }
}

__global__ void interp_bwd_kernel(PRInterpArgs a) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < a.PK; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = a.pix_to_face[s];
    const float* go = a.grad_out + s * a.D;
    if (f < 0) {
      if (a.grad_bary) { a.grad_bary[s * 3] = 0.f; a.grad_bary[s * 3 + 1] = 0.f; a.grad_bary[s * 3 + 2] = 0.f; }
      continue;
    }
    const float w[3] = {a.bary[s * 3], a.bary[s * 3 + 1], a.bary[s * 3 + 2]};
    const int64_t rows[3] = {attr_row(a, f, 0), attr_row(a, f, 1), attr_row(a, f, 2)};
    float gb[3] = {0.f, 0.f, 0.f};
    for (int d = 0; d < a.D; ++d) {
      const float g = go[d];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        gb[i] += g * a.face_attr[rows[i] + d];
        if (a.grad_face_attr && g != 0.f) atomicAdd(&a.grad_face_attr[rows[i] + d], w[i] * g);
      }
    }
    if (a.grad_bary) { a.grad_bary[s * 3] = gb[0]; a.grad_bary[s * 3 + 1] = gb[1]; a.grad_bary[s * 3 + 2] = gb[2]; }
  }
}

// ---------------------------------------------------------------- projection
PR_DEV int mesh_of(const int64_t* first, const int64_t* nf, int N, int64_t f) {
  for (int n = 0; n < N; ++n)
    if (f >= first[n] && f < first[n] + nf[n]) return n;
  return 0;
}

// [x,y,z,1] @ M (row-vector, PyTorch3D Transform3d) followed by the w division
PR_DEV void xform(const float* M, float x, float y, float z, float o[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) o[c] = ((x * M[c] + y * M[4 + c]) + z * M[8 + c]) + M[12 + c];
}

__global__ void project_fwd_kernel(PRProjectArgs a) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < a.F * 3; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = t / 3;
    const int n = mesh_of(a.mesh_first_face, a.mesh_num_faces, a.N, f);
    const float* v = a.verts + a.faces[t] * 3;
    float o[4], c[4];
    xform(a.world_to_view + n * 16, v[0], v[1], v[2], o);
    const float vx = o[0] / o[3], vy = o[1] / o[3], vz = o[2] / o[3];
    xform(a.proj + n * 16, vx, vy, vz, c);
    a.face_verts[t * 3 + 0] = c[0] / c[3];
    a.face_verts[t * 3 + 1] = c[1] / c[3];
    a.face_verts[t * 3 + 2] = vz;
  }
}

// MeshRasterizer's projection and the rasterizer's face preparation in one pass (one
// thread per face, project_fwd_kernel's operations per corner), plus the zeroing of the
// backward's accumulators (grad_face_verts, grad_verts) so the backward needs no memset.
__global__ void project_prep_kernel(PRProjectArgs a, float blur_v, const float* blur_dev, int cull_backfaces,
                                    FaceRec* recs, uint2* bbox, float* zero_fv, float* zero_v, BinGrid bins) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const float blur = blur_dev ? *blur_dev : blur_v;
  if (a.seed_advance && blockIdx.x == 0 && threadIdx.x == 0) {  // the caller's deferred key advances
    const unsigned i = threadIdx.x;  // (lane-indexed: a vector store)
    uint64_t s = a.seed_advance[i];
    for (int k = 0; k < a.seed_advance_n; ++k) s = seed_next(s);
    a.seed_advance[i] = s;
  }
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < a.F; f += stride) {
    const int n = mesh_of(a.mesh_first_face, a.mesh_num_faces, a.N, f);
    float fv[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float* v = a.verts + a.faces[f * 3 + i] * 3;
      float o[4], c[4];
      xform(a.world_to_view + n * 16, v[0], v[1], v[2], o);
      const float vx = o[0] / o[3], vy = o[1] / o[3], vz = o[2] / o[3];
      xform(a.proj + n * 16, vx, vy, vz, c);
      fv[i * 3 + 0] = c[0] / c[3];
      fv[i * 3 + 1] = c[1] / c[3];
      fv[i * 3 + 2] = vz;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) a.face_verts[f * 9 + i] = fv[i];
    write_face_rec(fv, blur, cull_backfaces, recs + f, bbox + f);
    if (bins.count) bin_face(bins, n, f, bbox[f]);
  }
  if (zero_fv)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.F * 9; i += stride) zero_fv[i] = 0.f;
  if (zero_v)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.V * 3; i += stride) zero_v[i] = 0.f;
}

// d v_view -> d v_world through [v,1] @ M / w, and d NDC (x, y) + d view z -> d v_view
PR_DEV void project_vertex_bwd(const float* M, const float* P, const float* v, float gx, float gy, float gz,
                               float gout[3]) {
  float o[4], c[4];
  xform(M, v[0], v[1], v[2], o);
  const float vv[3] = {o[0] / o[3], o[1] / o[3], o[2] / o[3]};
  xform(P, vv[0], vv[1], vv[2], c);
  const float i3 = 1.f / c[3], i33 = i3 * i3;
  float gvv[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    gvv[k] = gx * (P[k * 4 + 0] * i3 - c[0] * P[k * 4 + 3] * i33) + gy * (P[k * 4 + 1] * i3 - c[1] * P[k * 4 + 3] * i33);
  gvv[2] += gz;
  const float j3 = 1.f / o[3], j33 = j3 * j3;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    float g = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) g += gvv[k] * (M[m * 4 + k] * j3 - o[k] * M[m * 4 + 3] * j33);
    gout[m] = g;
  }
}

// CSR form: each vertex sums its corners' d face_verts in corner order (the verts[faces]
// backward), then one Jacobian per vertex.  Deterministic, no atomics, every row written.
// The corners go in batches of kGatherB: the batch's corner ids, then their gradients, each
// level's loads in flight together (a vertex has ~6 corners: two load round trips instead of a
// dependent pair per corner); the sums keep the corner order.
constexpr int kGatherB = 8;
__global__ void project_bwd_gather_kernel(PRProjectArgs a) {
  for (int64_t vi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; vi < a.V; vi += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = a.vert_corner_start[vi], e = a.vert_corner_start[vi + 1];
    float g[3] = {0.f, 0.f, 0.f};
    if (s < e) {
      float gx = 0.f, gy = 0.f, gz = 0.f;
      int64_t t0 = 0;
      for (int64_t j0 = s; j0 < e; j0 += kGatherB) {
        int64_t t[kGatherB];
#pragma unroll
        for (int u = 0; u < kGatherB; ++u) t[u] = j0 + u < e ? a.vert_corners[j0 + u] : -1;
        if (j0 == s) t0 = t[0];
        float c[kGatherB][3];
#pragma unroll
        for (int u = 0; u < kGatherB; ++u) {
          if (t[u] >= 0) {
            c[u][0] = a.grad_face_verts[t[u] * 3];
            c[u][1] = a.grad_face_verts[t[u] * 3 + 1];
            c[u][2] = a.grad_face_verts[t[u] * 3 + 2];
          }
        }
#pragma unroll
        for (int u = 0; u < kGatherB; ++u) {
          if (t[u] >= 0) {
            gx += c[u][0];
            gy += c[u][1];
            gz += c[u][2];
          }
        }
      }
      const int n = mesh_of(a.mesh_first_face, a.mesh_num_faces, a.N, t0 / 3);
      project_vertex_bwd(a.world_to_view + n * 16, a.proj + n * 16, a.verts + vi * 3, gx, gy, gz, g);
    }
    a.grad_verts[vi * 3] = g[0];
    a.grad_verts[vi * 3 + 1] = g[1];
    a.grad_verts[vi * 3 + 2] = g[2];
  }
}

__global__ void project_bwd_kernel(PRProjectArgs a) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < a.F * 3; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = t / 3;
    const int n = mesh_of(a.mesh_first_face, a.mesh_num_faces, a.N, f);
    const int64_t vi = a.faces[t];
    const float* v = a.verts + vi * 3;
    const float* M = a.world_to_view + n * 16;
    const float* P = a.proj + n * 16;
    float o[4], c[4];
    xform(M, v[0], v[1], v[2], o);
    const float vv[3] = {o[0] / o[3], o[1] / o[3], o[2] / o[3]};
    xform(P, vv[0], vv[1], vv[2], c);
    const float gx = a.grad_face_verts[t * 3], gy = a.grad_face_verts[t * 3 + 1], gz = a.grad_face_verts[t * 3 + 2];
    const float i3 = 1.f / c[3], i33 = i3 * i3;
    float gvv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      gvv[k] = gx * (P[k * 4 + 0] * i3 - c[0] * P[k * 4 + 3] * i33) + gy * (P[k * 4 + 1] * i3 - c[1] * P[k * 4 + 3] * i33);
    }
    gvv[2] += gz;
    const float j3 = 1.f / o[3], j33 = j3 * j3;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float g = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) g += gvv[k] * (M[m * 4 + k] * j3 - o[k] * M[m * 4 + 3] * j33);
      atomicAdd(&a.grad_verts[vi * 3 + m], g);
    }
  }
}

int rast_check(const PRRastArgs& a) {
  if (a.N <= 0 || a.H <= 0 || a.W <= 0 || a.K <= 0) return set_error(PR_ERR_ARG, "rast: bad shape");
  if (a.F < 0 || a.F >= (int64_t(1) << 31)) return set_error(PR_ERR_ARG, "rast: face count out of range");
  if (!a.face_verts && a.F > 0) return set_error(PR_ERR_ARG, "rast: face_verts missing");
  if (!a.mesh_first_face || !a.mesh_num_faces) return set_error(PR_ERR_ARG, "rast: mesh index missing");
  if (a.K > 512) return set_error(PR_ERR_ARG, "rast: faces_per_pixel must be <= 512");
  if ((int64_t)a.H > 65535 || (int64_t)a.W > 65535 * kTile || a.N > 65535)
    return set_error(PR_ERR_ARG, "rast: image too large");
  return PR_OK;
}

}  // namespace
}  // namespace pr

using namespace pr;

#ifdef PR_RAST_PROFILE
// diagnostic build only: copy the per-tile profile records of the last launches to the host
extern "C" int pr_rast_prof_dump(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rast_prof), bytes < sizeof(g_rast_prof) ? bytes : sizeof(g_rast_prof),
                             0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

// the coarse bin grid of a forward call (no bins: count == nullptr); pointers into the
// workspace after the face records and cull boxes when ws is given
static BinGrid bin_grid(const PRRastArgs& a, void* ws) {
  BinGrid g{};
  g.H = a.H; g.W = a.W;
  if (a.bin_size <= 0 || a.N <= 0 || a.H <= 0 || a.W <= 0) return g;
  g.bs = (a.bin_size + 7) / 8 * 8;  // a multiple of every tile shape
  g.nx = (a.W + g.bs - 1) / g.bs;
  g.ny = (a.H + g.bs - 1) / g.bs;
  // PyTorch3D's default cap (rasterize_meshes.py: max(10000, F / 5)), never above F
  const int64_t F = a.F > 0 ? a.F : 1;
  const int64_t mfpb = a.max_faces_per_bin > 0 ? a.max_faces_per_bin : std::max<int64_t>(10000, F / 5);
  g.cap = (int)std::min<int64_t>(mfpb, F);
  if (ws) {
    char* p = reinterpret_cast<char*>(ws) + (size_t)F * (sizeof(FaceRec) + sizeof(uint2));
    g.count = reinterpret_cast<int*>(p);
    g.list = g.count + (size_t)a.N * g.ny * g.nx;
  }
  return g;
}

static size_t bin_bytes(const PRRastArgs& a) {
  const BinGrid g = bin_grid(a, nullptr);
  if (g.bs == 0) return 0;
  const size_t nb = (size_t)a.N * g.ny * g.nx;
  return nb * sizeof(int) * (1 + (size_t)g.cap);
}

extern "C" size_t pr_rast_fwd_workspace_size(const PRRastArgs* a) {
  if (!a) return 0;
  // records + fp16 cull boxes + bin counts and lists
  return (size_t)(a->F > 0 ? a->F : 1) * (sizeof(FaceRec) + sizeof(uint2)) + bin_bytes(*a);
}

// bins of this call, their counters zeroed on the stream (before the face pass appends)
static int bins_begin(const PRRastArgs& a, BinGrid& g, hipStream_t st) {
  g = bin_grid(a, a.workspace);
  if (!g.count) return PR_OK;
  if (hipMemsetAsync(g.count, 0, (size_t)a.N * g.ny * g.nx * sizeof(int), st) != hipSuccess)
    return set_error(PR_ERR_HIP, "rast_fwd: bin counter memset failed");
  return PR_OK;
}

static int rast_fwd_prepared(const PRRastArgs& a, const FaceRec* fr, const uint2* fbox, const BinGrid& bins,
                             hipStream_t st);

extern "C" int pr_rast_fwd(const PRRastArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "rast_fwd: null args");
  const PRRastArgs& a = *args;
  if (int e = rast_check(a)) return e;
  if (!a.pix_to_face || !a.zbuf || !a.bary || !a.dists) return set_error(PR_ERR_ARG, "rast_fwd: output missing");
  if (!a.workspace || a.workspace_bytes < pr_rast_fwd_workspace_size(args))
    return set_error(PR_ERR_WORKSPACE, "rast_fwd: workspace too small");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  FaceRec* fr = reinterpret_cast<FaceRec*>(a.workspace);
  uint2* fbox = reinterpret_cast<uint2*>(fr + (a.F > 0 ? a.F : 1));
  BinGrid bins;
  if (int e = bins_begin(a, bins, st)) return e;
  if (a.F > 0) {
    const int nb = (int)std::min<int64_t>((a.F + kThreads - 1) / kThreads, 1024);
    face_prep_kernel<<<nb, kThreads, 0, st>>>(a.face_verts, a.F, a.blur_radius, a.blur_radius_dev, a.cull_backfaces, fr,
                                              fbox, bins, a.mesh_first_face, a.N);
    if (int e = check_launch("rast_face_prep")) return e;
  }
  return rast_fwd_prepared(a, fr, fbox, bins, st);
}

static int rast_fwd_prepared(const PRRastArgs& a, const FaceRec* fr, const uint2* fbox, const BinGrid& bins,
                             hipStream_t st) {
  // face slices per pixel (tile 8x8 / 8x4 / 4x4): 4 measured fastest on the bench frame
  // with the two-stage face test (107 us vs 118-123 at 2 and 157 at 1); PR_RAST_SLICES=1|2|4
  // overrides (sweeps).  FRAG: barycentrics / distances written by the rasterizer itself
  // (no second pass over pix_to_face); PR_RAST_FRAG=0 selects the separate pass.
  // Deep queues (K > 128: more than 16 KB of 4x4-tile queue per wave) take 8 slices on 4x2 tiles,
  // half the queue LDS per wave, so more waves stay resident: cfg 4 (K = 150) 5.27 -> 5.01 ms;
  // at cfg 3 (K = 100) 4 slices stay faster (1.04 vs 1.14 ms).
  int sl = (int64_t)a.K * 16 * 8 > 16 * 1024 ? 8 : 4;
  if (const char* e = getenv("PR_RAST_SLICES")) {
    const int v = atoi(e);
    if (v == 1 || v == 2 || v == 4 || v == 8) sl = v;
  }
  bool frag = true;
  if (const char* e = getenv("PR_RAST_FRAG")) frag = atoi(e) != 0;
  // two waves per 4x4 tile (rast_fwd_kernel NW = 2; PR_RAST_DUO=1, read per call)
  const char* duo = getenv("PR_RAST_DUO");
  const int nw = sl == 4 && duo && duo[0] == '1' ? 2 : 1;
  size_t lds = rast_fwd_lds(a.K, sl, nw);
  if (const char* e = getenv("PR_RAST_LDS_MIN")) lds = std::max(lds, (size_t)atol(e));  // occupancy sweeps
  if (lds > 160 * 1024) return set_error(PR_ERR_ARG, "rast_fwd: faces_per_pixel too large for the LDS queue (max 300)");
  launch_rast_fwd(a, fr, fbox, sl, frag, lds, bins, st, nw);
  if (int e = check_launch("rast_fwd")) return e;
  if (frag) return PR_OK;
  const int64_t total = (int64_t)a.N * a.H * a.W * a.K;
  const int nb = (int)std::min<int64_t>((total + kThreads - 1) / kThreads, 1 << 20);
  if (total * 3 < (int64_t(1) << 32)) rast_frag_kernel<false><<<nb, kThreads, 0, st>>>(a, total);
  else rast_frag_kernel<true><<<nb, kThreads, 0, st>>>(a, total);
  return check_launch("rast_frag");
}

extern "C" size_t pr_rast_bwd_workspace_size(const PRRastArgs* a) {
  if (!a || !(a->flags & PR_DETERMINISTIC)) return 0;
  return detsum_workspace(std::min<int64_t>((int64_t)a->N * a->H * a->W * a->K, det_batch()), a->F, 9);
}

// PR_DETERMINISTIC: every face's slot gradients (exact arithmetic) summed in slot order, in
// batches of det_batch() slots whose sums continue each face's chain (bounded workspace: ~1.5 GB
// at most, whatever the frame; bitwise the single pass)
static int rast_bwd_deterministic(const PRRastArgs& a, hipStream_t st) {
  const int64_t total = (int64_t)a.N * a.H * a.W * a.K, batch = det_batch();
  if (a.F == 0) return PR_OK;
  for (int64_t s0 = 0; s0 < total; s0 += batch) {
    const int64_t n = std::min(batch, total - s0);
    DetSum d;
    if (int e = detsum_layout(a.workspace, a.workspace_bytes, n, a.F, 9, d)) return e;
    const int nb = (int)std::min<int64_t>((n + kThreads - 1) / kThreads, 16384);
    rast_bwd_keys_kernel<<<nb, kThreads, 0, st>>>(a, d.keys, s0, n);
    if (int e = check_launch("rast_bwd_keys")) return e;
    if (int e = detsum_sort(d, st)) return e;
    rast_bwd_sorted_grad_kernel<<<nb, kThreads, 0, st>>>(a, d.keys_sorted, d.idx_sorted, d.vals_sorted, s0, n);
    if (int e = check_launch("rast_bwd_sorted_grad")) return e;
    if (int e = detsum_reduce_chain(d, a.grad_face_verts, s0 == 0, st)) return e;
  }
  return PR_OK;
}

extern "C" int pr_rast_bwd(const PRRastArgs* args, void* stream) {
  if (!args) return set_error(PR_ERR_ARG, "rast_bwd: null args");
  const PRRastArgs& a = *args;
  if (int e = rast_check(a)) return e;
  if (!a.pix_to_face || !a.grad_face_verts) return set_error(PR_ERR_ARG, "rast_bwd: buffer missing");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.flags & PR_DETERMINISTIC) return rast_bwd_deterministic(a, st);
  if (a.F > 0 && !(a.flags & PR_GRAD_PREZEROED)) {
    if (hipMemsetAsync(a.grad_face_verts, 0, (size_t)a.F * 9 * sizeof(float), st) != hipSuccess)
      return set_error(PR_ERR_HIP, "rast_bwd: memset failed");
  }
  // rows per 8-wide workgroup tile: 2 measured fastest on the bench frame (more, smaller
  // workgroups hide the per-round latency chain), 4 on large batches (>= 2^18 pixels: cfg 3
  // 0.53 -> 0.45 ms, cfg 4 2.01 -> 1.71 ms); PR_RAST_BWD_ROWS=1|2|4|8 overrides (sweeps)
  const char* er = getenv("PR_RAST_BWD_ROWS");
  const int64_t npix = (int64_t)a.N * a.H * a.W;
  const int rows = er && (atoi(er) == 1 || atoi(er) == 2 || atoi(er) == 4 || atoi(er) == 8) ? atoi(er)
                                                                                            : (npix >= (1 << 18) ? 4 : 2);
  dim3 grid((a.W + kBwdTile - 1) / kBwdTile, (a.H + rows - 1) / rows, a.N);
  // tile rows dispatched centre-out (PR_RAST_ORDER bit 1; 0: row-major)
  static const int order = (getenv("PR_RAST_ORDER") ? atoi(getenv("PR_RAST_ORDER")) : 3) >> 1 & 1;
  // slot arithmetic: the oracle's exact operations (IEEE divisions, its accumulation order) by
  // default; PR_RAST_BWD_EXACT=0 selects reciprocal-multiply (sweeps)
  static const bool exact = !getenv("PR_RAST_BWD_EXACT") || atoi(getenv("PR_RAST_BWD_EXACT")) != 0;
#define PR_RAST_BWD_LAUNCH(R)                                               \
  do {                                                                      \
    if (exact) rast_bwd_kernel<R, true><<<grid, kBwdThreads, 0, st>>>(a, order);  \
    else rast_bwd_kernel<R, false><<<grid, kBwdThreads, 0, st>>>(a, order);       \
  } while (0)
  ktimer_mark(0, "rast_bwd_kernel", st);
  if (rows == 8) PR_RAST_BWD_LAUNCH(8);
  else if (rows == 4) PR_RAST_BWD_LAUNCH(4);
  else if (rows == 1) PR_RAST_BWD_LAUNCH(1);
  else PR_RAST_BWD_LAUNCH(2);
  ktimer_mark(1, "rast_bwd_kernel", st);
#undef PR_RAST_BWD_LAUNCH
  return check_launch("rast_bwd");
}

extern "C" int pr_interp_fwd(const PRInterpArgs* args, void* stream) {
  if (!args || !args->pix_to_face || !args->bary || !args->face_attr || !args->out || args->D <= 0)
    return set_error(PR_ERR_ARG, "interp_fwd: bad args");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (args->PK == 0) return PR_OK;
  const int nb = (int)std::min<int64_t>((args->PK + kThreads - 1) / kThreads, 8192);
  interp_fwd_kernel<<<nb, kThreads, 0, st>>>(*args);
  return check_launch("interp_fwd");
}

extern "C" int pr_interp_bwd(const PRInterpArgs* args, void* stream) {
  if (!args || !args->pix_to_face || !args->bary || !args->face_attr || !args->grad_out || args->D <= 0)
    return set_error(PR_ERR_ARG, "interp_bwd: bad args");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t rows = args->faces ? args->V : args->F * 3;
  if (args->grad_face_attr && rows > 0) {
    if (hipMemsetAsync(args->grad_face_attr, 0, (size_t)rows * args->D * sizeof(float), st) != hipSuccess)
      return set_error(PR_ERR_HIP, "interp_bwd: memset failed");
  }
  if (args->PK == 0) return PR_OK;
  const int nb = (int)std::min<int64_t>((args->PK + kThreads - 1) / kThreads, 8192);
  interp_bwd_kernel<<<nb, kThreads, 0, st>>>(*args);
  return check_launch("interp_bwd");
}

static int project_check(const PRProjectArgs* a) {
  if (!a || !a->verts || !a->faces || !a->mesh_first_face || !a->mesh_num_faces || !a->world_to_view || !a->proj ||
      a->N <= 0 || a->V < 0 || a->F < 0 || a->seed_advance_n < 0 || (a->seed_advance_n > 0 && !a->seed_advance))
    return set_error(PR_ERR_ARG, "project: bad args");
  return PR_OK;
}

extern "C" int pr_project_fwd(const PRProjectArgs* args, void* stream) {
  if (int e = project_check(args)) return e;
  if (!args->face_verts) return set_error(PR_ERR_ARG, "project_fwd: face_verts missing");
  if (args->F == 0) return PR_OK;
  const int nb = (int)std::min<int64_t>((args->F * 3 + kThreads - 1) / kThreads, 4096);
  project_fwd_kernel<<<nb, kThreads, 0, reinterpret_cast<hipStream_t>(stream)>>>(*args);
  return check_launch("project_fwd");
}

extern "C" int pr_project_bwd(const PRProjectArgs* args, void* stream) {
  if (int e = project_check(args)) return e;
  if (!args->grad_face_verts || !args->grad_verts) return set_error(PR_ERR_ARG, "project_bwd: buffers missing");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (args->vert_corner_start && args->vert_corners) {
    if (args->V == 0) return PR_OK;
    const int nb = (int)std::min<int64_t>((args->V + kThreads - 1) / kThreads, 4096);
    project_bwd_gather_kernel<<<nb, kThreads, 0, st>>>(*args);
    return check_launch("project_bwd_gather");
  }
  if (args->V > 0 && !(args->flags & PR_GRAD_PREZEROED) &&
      hipMemsetAsync(args->grad_verts, 0, (size_t)args->V * 3 * sizeof(float), st) != hipSuccess)
    return set_error(PR_ERR_HIP, "project_bwd: memset failed");
  if (args->F == 0) return PR_OK;
  const int nb = (int)std::min<int64_t>((args->F * 3 + kThreads - 1) / kThreads, 4096);
  project_bwd_kernel<<<nb, kThreads, 0, st>>>(*args);
  return check_launch("project_bwd");
}

extern "C" int pr_project_rast_fwd(const PRProjectArgs* pa, const PRRastArgs* ra, void* stream) {
  if (int e = project_check(pa)) return e;
  if (!ra) return set_error(PR_ERR_ARG, "project_rast_fwd: null rast args");
  const PRRastArgs& a = *ra;
  if (int e = rast_check(a)) return e;
  if (!pa->face_verts || pa->face_verts != a.face_verts || pa->F != a.F || pa->N != a.N)
    return set_error(PR_ERR_ARG, "project_rast_fwd: projection and rasterizer face buffers / counts differ");
  if (!a.pix_to_face || !a.zbuf || !a.bary || !a.dists) return set_error(PR_ERR_ARG, "rast_fwd: output missing");
  if (!a.workspace || a.workspace_bytes < pr_rast_fwd_workspace_size(ra))
    return set_error(PR_ERR_WORKSPACE, "rast_fwd: workspace too small");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  FaceRec* fr = reinterpret_cast<FaceRec*>(a.workspace);
  uint2* fbox = reinterpret_cast<uint2*>(fr + (a.F > 0 ? a.F : 1));
  BinGrid bins;
  if (int e = bins_begin(a, bins, st)) return e;
  const int64_t work = std::max<int64_t>(std::max<int64_t>(a.F, a.grad_face_verts ? a.F * 9 : 0),
                                         pa->grad_verts ? pa->V * 3 : 0);
  if (work > 0 || (pa->seed_advance && pa->seed_advance_n > 0)) {
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((work + kThreads - 1) / kThreads, 1024));
    project_prep_kernel<<<nb, kThreads, 0, st>>>(*pa, a.blur_radius, a.blur_radius_dev, a.cull_backfaces, fr, fbox,
                                                 a.grad_face_verts, pa->grad_verts, bins);
    if (int e = check_launch("project_prep")) return e;
  }
  return rast_fwd_prepared(a, fr, fbox, bins, st);
}
