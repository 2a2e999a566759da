/*
 * CPU oracle for the K-nearest-face mesh rasterizer  —  TEST INFRASTRUCTURE ONLY.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Plain-C restatement of PyTorch3D 0.4.0's naive CPU rasterizer
 * (rasterize_meshes_cpu.cpp: RasterizeMeshesNaiveCpu / RasterizeMeshesBackwardCpu)
 * and of interpolate_face_attributes, the [p3d] dependency the reference calls
 * through MeshRasterizer (experiments/eval.py:165-168; requirements.txt:7,
 * pytorch3d==0.4.0).  PyTorch3D is not vendored in /root/reference and is not
 * installed here, so this restates its published algorithm:
 *
 *   pixel (row, col) -> NDC: xi = W-1-col, yi = H-1-row (+X left, +Y up),
 *     x = -off + (range*xi + off)/W  (range 2, widened on the long side)
 *   per face of the pixel's mesh:  skip if zmax < 0, back-facing && cull,
 *     |area| <= 1e-8, or pixel outside bbox grown by sqrt(blur);
 *     bary = edge-function ratios (area + 1e-8), optional perspective
 *     correction, optional clip (clamp >= 0, renormalise by max(sum,1e-5));
 *     pz = bary_clip . z ; skip pz < 0;
 *     d = min squared point-segment distance; inside = all unclipped bary > 0;
 *     skip if !inside && d >= blur;   signed dist = inside ? -d : d
 *   keep the K smallest (pz, face id), ascending; pad p2f/zbuf/bary/dists with -1.
 *   Backward: d/d face verts of zbuf (via clipped bary and z), bary and dists;
 *     the point-segment distance treats the clamped projection t as constant.
 *
 * PARITY UNPINNED by the reference (no PyTorch3D sources, tests or fixtures are
 * available); pinned instead by the analytic known-answer tests and
 * finite-difference checks in tests/test_rast_oracle.py.
 *
 * Build: make -C oracle  (REAL=float -> librast_oracle_f32.so, REAL=double -> _f64)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifndef REAL
#define REAL float
#endif
typedef REAL real;

static const real kEps = (real)1e-8;

static real edge(real px, real py, real ax, real ay, real bx, real by) {
  return (px - ax) * (by - ay) - (py - ay) * (bx - ax);
}

static void bary2d(real px, real py, const real* v, real w[3]) {
  const real area = edge(v[6], v[7], v[0], v[1], v[3], v[4]) + kEps;
  w[0] = edge(px, py, v[3], v[4], v[6], v[7]) / area;
  w[1] = edge(px, py, v[6], v[7], v[0], v[1]) / area;
  w[2] = edge(px, py, v[0], v[1], v[3], v[4]) / area;
}

static void persp(const real b[3], real z0, real z1, real z2, real o[3]) {
  const real t0 = b[0] * z1 * z2, t1 = z0 * b[1] * z2, t2 = z0 * z1 * b[2];
  real d = t0 + t1 + t2;
  if (!(d > kEps)) d = kEps;
  o[0] = t0 / d; o[1] = t1 / d; o[2] = t2 / d;
}

static void clipb(const real b[3], real o[3]) {
  real w0 = b[0] > 0 ? b[0] : 0, w1 = b[1] > 0 ? b[1] : 0, w2 = b[2] > 0 ? b[2] : 0;
  real s = w0 + w1 + w2;
  if (!(s > (real)1e-5)) s = (real)1e-5;
  o[0] = w0 / s; o[1] = w1 / s; o[2] = w2 / s;
}

static real segd2(real px, real py, real ax, real ay, real bx, real by, real* tout) {
  const real bax = bx - ax, bay = by - ay;
  const real l2 = bax * bax + bay * bay;
  if (l2 <= kEps) {
    *tout = 1;
    return (px - bx) * (px - bx) + (py - by) * (py - by);
  }
  real t = (bax * (px - ax) + bay * (py - ay)) / l2;
  t = t < 0 ? 0 : (t > 1 ? 1 : t);
  *tout = t;
  const real qx = ax + t * bax, qy = ay + t * bay;
  return (px - qx) * (px - qx) + (py - qy) * (py - qy);
}

/* which edge is closest: 0 = (v0,v1), 1 = (v0,v2), 2 = (v1,v2) */
static real trid2(real px, real py, const real* v, int* which) {
  real t;
  const real e01 = segd2(px, py, v[0], v[1], v[3], v[4], &t);
  const real e02 = segd2(px, py, v[0], v[1], v[6], v[7], &t);
  const real e12 = segd2(px, py, v[3], v[4], v[6], v[7], &t);
  if (e01 <= e02 && e01 <= e12) { *which = 0; return e01; }
  if (e02 <= e01 && e02 <= e12) { *which = 1; return e02; }
  *which = 2;
  return e12;
}

static real ndc(int i, int S1, int S2) {
  real range = 2;
  if (S1 > S2) range = ((real)S1 * range) / (real)S2;
  const real off = range / 2;
  return -off + (range * (real)i + off) / (real)S1;
}

void rast_fwd(const real* fv, const int64_t* first, const int64_t* nfaces, int N, int H, int W, int K,
              real blur, int perspective_correct, int clip_bary, int cull_backfaces, int64_t* p2f,
              real* zbuf, real* bary, real* dists) {
  const real rb = (real)sqrt((double)blur);
#pragma omp parallel for collapse(2) schedule(dynamic, 1)
  for (int n = 0; n < N; ++n) {
    for (int row = 0; row < H; ++row) {
      real* qz = (real*)malloc(sizeof(real) * (size_t)(K + 1));
      int64_t* qf = (int64_t*)malloc(sizeof(int64_t) * (size_t)(K + 1));
      const real py = ndc(H - 1 - row, H, W);
      for (int col = 0; col < W; ++col) {
        const real px = ndc(W - 1 - col, W, H);
        int qs = 0;
        for (int64_t f = first[n]; f < first[n] + nfaces[n]; ++f) {
          const real* v = fv + f * 9;
          const real zmax = fmax(v[2], fmax(v[5], v[8]));
          const real area = edge(v[0], v[1], v[3], v[4], v[6], v[7]);
          if (zmax < 0 || (cull_backfaces && area < 0) || (area <= kEps && area >= -kEps)) continue;
          const real xmin = (real)fmin(v[0], fmin(v[3], v[6])) - rb, xmax = (real)fmax(v[0], fmax(v[3], v[6])) + rb;
          const real ymin = (real)fmin(v[1], fmin(v[4], v[7])) - rb, ymax = (real)fmax(v[1], fmax(v[4], v[7])) + rb;
          if (px > xmax || px < xmin || py > ymax || py < ymin) continue;
          real b0[3], b[3], bc[3];
          bary2d(px, py, v, b0);
          if (perspective_correct) persp(b0, v[2], v[5], v[8], b); else memcpy(b, b0, sizeof b);
          if (clip_bary) clipb(b, bc); else memcpy(bc, b, sizeof bc);
          const real pz = bc[0] * v[2] + bc[1] * v[5] + bc[2] * v[8];
          if (pz < 0) continue;
          int which;
          const real d = trid2(px, py, v, &which);
          const int inside = b[0] > 0 && b[1] > 0 && b[2] > 0;
          if (!inside && d >= blur) continue;
          /* insert into the ascending (z, face) list, truncated to K */
          if (qs == K && !(pz < qz[K - 1] || (pz == qz[K - 1] && f < qf[K - 1]))) continue;
          int pos = qs < K ? qs : K - 1;
          if (qs < K) ++qs;
          while (pos > 0 && (pz < qz[pos - 1] || (pz == qz[pos - 1] && f < qf[pos - 1]))) {
            qz[pos] = qz[pos - 1]; qf[pos] = qf[pos - 1]; --pos;
          }
          qz[pos] = pz; qf[pos] = f;
        }
        const int64_t pix = ((int64_t)n * H + row) * W + col;
        for (int k = 0; k < K; ++k) {
          const int64_t o = pix * K + k;
          if (k < qs) {
            const real* v = fv + qf[k] * 9;
            real b0[3], b[3], bc[3];
            bary2d(px, py, v, b0);
            if (perspective_correct) persp(b0, v[2], v[5], v[8], b); else memcpy(b, b0, sizeof b);
            if (clip_bary) clipb(b, bc); else memcpy(bc, b, sizeof bc);
            int which;
            const real d = trid2(px, py, v, &which);
            const int inside = b[0] > 0 && b[1] > 0 && b[2] > 0;
            p2f[o] = qf[k];
            zbuf[o] = qz[k];
            dists[o] = inside ? -d : d;
            bary[o * 3 + 0] = bc[0]; bary[o * 3 + 1] = bc[1]; bary[o * 3 + 2] = bc[2];
          } else {
            p2f[o] = -1;
            zbuf[o] = -1; dists[o] = -1;
            bary[o * 3 + 0] = -1; bary[o * 3 + 1] = -1; bary[o * 3 + 2] = -1;
          }
        }
      }
      free(qz);
      free(qf);
    }
  }
}

/* ------------------------------------------------------------------ backward */
static void segd2_bwd(real px, real py, real ax, real ay, real bx, real by, real g, real* ga, real* gb) {
  real t;
  segd2(px, py, ax, ay, bx, by, &t);
  const real qx = (1 - t) * ax + t * bx, qy = (1 - t) * ay + t * by;
  const real dx = qx - px, dy = qy - py;
  ga[0] += g * (1 - t) * 2 * dx; ga[1] += g * (1 - t) * 2 * dy;
  gb[0] += g * t * 2 * dx;       gb[1] += g * t * 2 * dy;
}

/* gradient of e = edge(p, a, b) w.r.t. a, b scaled by g */
static void edge_bwd(real px, real py, real ax, real ay, real bx, real by, real g, real* ga, real* gb) {
  ga[0] += g * (py - by); ga[1] += g * (bx - px);
  gb[0] += g * (ay - py); gb[1] += g * (px - ax);
}

static void bary2d_bwd(real px, real py, const real* v, const real gw[3], real gv[3][2]) {
  const real area = edge(v[6], v[7], v[0], v[1], v[3], v[4]) + kEps;
  const real e0 = edge(px, py, v[3], v[4], v[6], v[7]);
  const real e1 = edge(px, py, v[6], v[7], v[0], v[1]);
  const real e2 = edge(px, py, v[0], v[1], v[3], v[4]);
  const real darea = -(gw[0] * e0 + gw[1] * e1 + gw[2] * e2) / (area * area);
  edge_bwd(px, py, v[3], v[4], v[6], v[7], gw[0] / area, gv[1], gv[2]);
  edge_bwd(px, py, v[6], v[7], v[0], v[1], gw[1] / area, gv[2], gv[0]);
  edge_bwd(px, py, v[0], v[1], v[3], v[4], gw[2] / area, gv[0], gv[1]);
  /* area = edge(v2, v0, v1): gradient w.r.t. its point argument v2 too */
  gv[2][0] += darea * (v[4] - v[1]);
  gv[2][1] += darea * (v[0] - v[3]);
  edge_bwd(v[6], v[7], v[0], v[1], v[3], v[4], darea, gv[0], gv[1]);
}

static void persp_bwd(const real b[3], real z0, real z1, real z2, const real go[3], real gb[3], real gz[3]) {
  const real t0 = b[0] * z1 * z2, t1 = z0 * b[1] * z2, t2 = z0 * z1 * b[2];
  const real s = t0 + t1 + t2;
  real gt[3];
  if (s > kEps) {
    const real dot = (go[0] * t0 + go[1] * t1 + go[2] * t2) / (s * s);
    gt[0] = go[0] / s - dot; gt[1] = go[1] / s - dot; gt[2] = go[2] / s - dot;
  } else {
    gt[0] = go[0] / kEps; gt[1] = go[1] / kEps; gt[2] = go[2] / kEps;
  }
  gb[0] = gt[0] * z1 * z2; gb[1] = gt[1] * z0 * z2; gb[2] = gt[2] * z0 * z1;
  gz[0] = gt[1] * b[1] * z2 + gt[2] * z1 * b[2];
  gz[1] = gt[0] * b[0] * z2 + gt[2] * z0 * b[2];
  gz[2] = gt[0] * b[0] * z1 + gt[1] * z0 * b[1];
}

static void clip_bwd(const real b[3], const real go[3], real gb[3]) {
  const real w0 = b[0] > 0 ? b[0] : 0, w1 = b[1] > 0 ? b[1] : 0, w2 = b[2] > 0 ? b[2] : 0;
  const real s = w0 + w1 + w2;
  real gw[3];
  if (s > (real)1e-5) {
    const real dot = (go[0] * w0 + go[1] * w1 + go[2] * w2) / (s * s);
    gw[0] = go[0] / s - dot; gw[1] = go[1] / s - dot; gw[2] = go[2] / s - dot;
  } else {
    gw[0] = go[0] / (real)1e-5; gw[1] = go[1] / (real)1e-5; gw[2] = go[2] / (real)1e-5;
  }
  gb[0] = b[0] > 0 ? gw[0] : 0; gb[1] = b[1] > 0 ? gw[1] : 0; gb[2] = b[2] > 0 ? gw[2] : 0;
}

void rast_bwd(const real* fv, int64_t F, const int64_t* p2f, int N, int H, int W, int K, int perspective_correct,
              int clip_bary, const real* gzbuf, const real* gbary, const real* gdists, real* gfv) {
  memset(gfv, 0, sizeof(real) * (size_t)F * 9);
  for (int n = 0; n < N; ++n)
    for (int row = 0; row < H; ++row) {
      const real py = ndc(H - 1 - row, H, W);
      for (int col = 0; col < W; ++col) {
        const real px = ndc(W - 1 - col, W, H);
        const int64_t pix = ((int64_t)n * H + row) * W + col;
        for (int k = 0; k < K; ++k) {
          const int64_t o = pix * K + k;
          const int64_t f = p2f[o];
          if (f < 0) continue;
          const real* v = fv + f * 9;
          const real gz = gzbuf ? gzbuf[o] : 0, gd = gdists ? gdists[o] : 0;
          real gbu[3] = {0, 0, 0};
          if (gbary) { gbu[0] = gbary[o * 3]; gbu[1] = gbary[o * 3 + 1]; gbu[2] = gbary[o * 3 + 2]; }
          real bw[3], bp[3], bc[3];
          bary2d(px, py, v, bw);
          if (perspective_correct) persp(bw, v[2], v[5], v[8], bp); else memcpy(bp, bw, sizeof bp);
          if (clip_bary) clipb(bp, bc); else memcpy(bc, bp, sizeof bc);
          const int inside = bp[0] > 0 && bp[1] > 0 && bp[2] > 0;
          real gv[3][2] = {{0, 0}, {0, 0}, {0, 0}};
          /* signed squared distance */
          {
            const real g = inside ? -gd : gd;
            int which;
            trid2(px, py, v, &which);
            if (which == 0) segd2_bwd(px, py, v[0], v[1], v[3], v[4], g, gv[0], gv[1]);
            else if (which == 1) segd2_bwd(px, py, v[0], v[1], v[6], v[7], g, gv[0], gv[2]);
            else segd2_bwd(px, py, v[3], v[4], v[6], v[7], g, gv[1], gv[2]);
          }
          real gsum[3] = {gbu[0] + gz * v[2], gbu[1] + gz * v[5], gbu[2] + gz * v[8]};
          real gpp[3] = {gsum[0], gsum[1], gsum[2]};
          if (clip_bary) clip_bwd(bp, gsum, gpp);
          real gw[3] = {gpp[0], gpp[1], gpp[2]}, gzp[3] = {0, 0, 0};
          if (perspective_correct) persp_bwd(bw, v[2], v[5], v[8], gpp, gw, gzp);
          bary2d_bwd(px, py, v, gw, gv);
          real* o9 = gfv + f * 9;
          for (int i = 0; i < 3; ++i) {
            o9[i * 3 + 0] += gv[i][0];
            o9[i * 3 + 1] += gv[i][1];
            o9[i * 3 + 2] += gz * bc[i] + gzp[i];
          }
        }
      }
    }
}
