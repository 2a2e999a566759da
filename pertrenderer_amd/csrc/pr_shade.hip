// Phong shading of fragment slots (PyTorch3D 0.4.0 phong_shading + the texel lookup of
// Meshes.sample_textures): the colour producer of RandomPhongShader (random_rasterizer.py:99-110,
// experiments/eval.py:170).  On eval.py's cube frame ~95 % of the 3.3 M slots are padding, whose
// colour depends on the image only, so the kernels separate the two kinds instead of shading
// one thread per slot:
//   forward, counts attached (the renderer's case): pixel blocks -- the padded slots written as
//     16-byte stores of the image's colour pattern, the live slots enumerated from the counts'
//     prefix (shade_fwd_pix_kernel);
//   otherwise, and the backward: per-wave chunks -- liveness flags, the live slots compacted into
//     an LDS list, the padded ones written from per-image terms, the live ones shaded one per lane
//     (wave_compact).
//
#include "pr_common.h"
#include "pr_phong.h"

namespace pr {
namespace {

// (pixel, slot, image) of slot s: 32-bit divisions when the frame's slots fit (idx32, every
// BASELINE configuration), a 64-bit division costs ~4x as many instructions per slot
PR_DEV void slot_index(int64_t s, int K, int64_t HW, bool idx32, int64_t& p, int& k, int& n) {
  if (idx32) {
    const uint32_t p32 = (uint32_t)s / (uint32_t)K;
    p = p32;
    k = (int)((uint32_t)s - p32 * (uint32_t)K);
    n = (int)(p32 / (uint32_t)HW);
  } else {
    p = s / K;
    k = (int)(s - p * K);
    n = (int)(p / HW);
  }
}

PR_DEV Slot load_slot(const PRShadeArgs& a, int64_t s, int64_t HW, bool idx32) {
  Slot sl;
  int64_t p;
  int k;
  slot_index(s, a.K, HW, idx32, p, k, sl.n);
  const bool valid = a.pix_count ? k < a.pix_count[p] : true;
  sl.f = valid ? a.pix_to_face[s] : -1;
  if (sl.f >= 0) {
    sl.b[0] = a.bary[s * 3]; sl.b[1] = a.bary[s * 3 + 1]; sl.b[2] = a.bary[s * 3 + 2];
  } else {
    sl.b[0] = sl.b[1] = sl.b[2] = 0.f;
  }
  return sl;
}


// ---- per-wave compaction of the live slots ---------------------------------------------------
// Each wave takes chunks of 64 R consecutive slots: one pass of flags (the counts, one small read
// per pixel), the live slots compacted into the wave's LDS list, the padded ones written from the
// per-image terms, then the live ones shaded densely.  On eval.py's cube frame ~95 % of the 3.3 M
// slots are padding and every wave over the mesh holds both kinds: shading per slot made each such
// wave pay the interpolation + lighting path and its dependent-load chain for one live lane.  The
// waves run their chunks independently (no workgroup barrier between chunks): the load-chain
// latency of one wave's live slots hides behind the other waves' stores.
// R = slots per lane and chunk: PR_SHADE_ROUNDS (4, 8, 12 or 16), default kRoundsDefault.
constexpr int kRoundsDefault = 4;
constexpr int kPadImgs = 256;  // images whose padded terms sit in LDS (9 floats each); beyond: per slot
constexpr int kWaves = kThreads / 64;

// A lane's position (pixel p, slot k, image n, pixel within the image ph) walked in steps of 64
// slots: one division per chunk instead of two per slot (a runtime integer division is ~20 VALU
// instructions; per slot they were most of the padded slots' arithmetic)
struct SlotPos {
  int64_t p, ph;
  int k, n;
};

PR_DEV SlotPos slot_pos(int64_t s, int K, int64_t HW, bool idx32) {
  SlotPos q;
  slot_index(s, K, HW, idx32, q.p, q.k, q.n);
  q.ph = q.p - (int64_t)q.n * HW;
  return q;
}

// s -> s + 64, with 64 = q64 K + r64
PR_DEV void step64(SlotPos& q, int K, int64_t HW, int q64, int r64) {
  q.k += r64;
  q.p += q64;
  q.ph += q64;
  if (q.k >= K) { q.k -= K; ++q.p; ++q.ph; }
  while (q.ph >= HW) { q.ph -= HW; ++q.n; }
}

// the live flags' lanes as chunk offsets (r * 64 + lane) in list[0, total), in slot order
template <int R>
PR_DEV int wave_compact(const bool (&live)[R], int* list) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int off = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t m = __ballot(live[r]);
    if (live[r]) list[off + __popcll(m & below)] = r * 64 + lane;
    off += __popcll(m);
  }
  __builtin_amdgcn_wave_barrier();
  return off;
}

// The backward's small accumulators (d verts, d normals, d vertex colours, d light, d camera), when
// given to the forward: zeroed by its grid, for a PR_GRAD_PREZEROED pr_shade_bwd (no memsets)
PR_DEV void zero_accumulators(const PRShadeArgs& a) {
  const int64_t t0 = (int64_t)blockIdx.x * kThreads + threadIdx.x, st = (int64_t)gridDim.x * kThreads;
  float* vbuf[3] = {a.grad_verts, a.grad_normals, a.texture == PR_TEX_VERTEX ? a.grad_vert_colors : nullptr};
  float* bbuf[2] = {a.grad_light, a.grad_camera};
  for (int j = 0; j < 3; ++j)
    if (vbuf[j])
      for (int64_t i = t0; i < a.V * 3; i += st) vbuf[j][i] = 0.f;
  for (int j = 0; j < 2; ++j)
    if (bbuf[j])
      for (int64_t i = t0; i < (int64_t)a.N * 3; i += st) bbuf[j][i] = 0.f;
}

// the per-image padded terms (lit, spec, tex: 9 floats per image) of all N images into LDS, once
// per workgroup; false when N exceeds the table (padded slots then shade directly)
// (threads t0.. compute it: the pixel-block kernels leave wave 0 to the counts)
PR_DEV bool pad_table(const PRShadeArgs& a, float* pad, int t0 = 0) {
  if (a.N > kPadImgs) return false;
  for (int n = (int)threadIdx.x - t0; n >= 0 && n < a.N; n += kThreads - t0) {
    const Terms t = slot_terms(a, pad_slot(n), -1, nullptr);
    float* o = pad + n * 9;
    o[0] = t.lit.x; o[1] = t.lit.y; o[2] = t.lit.z;
    o[3] = t.spec.x; o[4] = t.spec.y; o[5] = t.spec.z;
    o[6] = t.tex.x; o[7] = t.tex.y; o[8] = t.tex.z;
  }
  return true;
}

// A padded slot (pix_to_face < 0) shades p = n = 0 at uv = 0 (the reference composition): its
// terms depend on the image only, and its colour on the slot only through a given texel
PR_DEV V3 pad_colour(const PRShadeArgs& a, int64_t s, int n, bool tab, const float* pad) {
  if (!tab) {
    const Terms t = slot_terms(a, pad_slot(n), s, nullptr);
    return colour(t.lit, t.tex, t.spec);
  }
  const float* e = pad + n * 9;
  const V3 tex = a.texture == PR_TEX_GIVEN ? v3(a.texels + s * 3) : V3{e[6], e[7], e[8]};
  return colour(V3{e[0], e[1], e[2]}, tex, V3{e[3], e[4], e[5]});
}

// a wave's chunks: [c0, c0 + 64 R) for c0 = (global wave) * 64 R, striding over the grid's waves
#define PR_WAVE_CHUNKS(R, s0, PK, c0, c1)                                                              \
  for (int64_t c0 = (s0) + ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * (64 * (R)), c1;      \
       c1 = c0 + 64 * (R) < (PK) ? c0 + 64 * (R) : (PK), c0 < (PK); c0 += (int64_t)gridDim.x * kWaves * 64 * (R))

// The padded terms' table is published by the first pass's workgroup barrier, placed after that
// pass's live slots: the table's load chain (light, camera, materials, map) runs beside the
// waves' count -> fragment -> mesh chain instead of before it.  Passes are per workgroup (each
// wave takes its 64 R slots of the workgroup's 4 x 64 R), so every wave meets that barrier.
template <int R>
__global__ void __launch_bounds__(kThreads) shade_fwd_kernel(PRShadeArgs a, int64_t PK, int64_t HW, int idx32) {
  __shared__ int lists[kWaves][64 * R];
  __shared__ float pad[kPadImgs * 9];
  zero_accumulators(a);
  const bool i32 = idx32 != 0;
  const int lane = threadIdx.x & 63;
  int* list = lists[threadIdx.x >> 6];
  const bool tab = pad_table(a, pad);
  const int q64 = 64 / a.K, r64 = 64 - q64 * a.K;
  constexpr int64_t kBlockSlots = (int64_t)kWaves * 64 * R;
  bool first = true;
  for (int64_t b0 = (int64_t)blockIdx.x * kBlockSlots; b0 < PK; b0 += (int64_t)gridDim.x * kBlockSlots) {
    const int64_t c0 = b0 + (threadIdx.x >> 6) * (64 * R);
    const int64_t c1 = c0 + 64 * R < PK ? c0 + 64 * R : PK;
    bool live[R];
    int img[R];
    SlotPos q = slot_pos(c0 + lane, a.K, HW, i32);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t s = c0 + r * 64 + lane;
      live[r] = s < c1 && (a.pix_count ? q.k < a.pix_count[q.p] : a.pix_to_face[s] >= 0);
      img[r] = q.n;
      if (r + 1 < R) step64(q, a.K, HW, q64, r64);
    }
    const int total = wave_compact(live, list);
    for (int i = lane; i < total; i += 64) {
      const int64_t s = c0 + list[i];
      const Slot sl = load_slot(a, s, HW, i32);
      // (a counted slot without a face -- not produced by the rasterizer -- shades as padding,
      // directly: the table may not be published yet)
      const Terms t = slot_terms(a, sl, s, sl.f >= 0 ? a.faces + sl.f * 3 : nullptr);
      const V3 c = colour(t.lit, t.tex, t.spec);
      float* o = a.colors + s * 3;
      o[0] = c.x; o[1] = c.y; o[2] = c.z;
    }
    if (first) {
      __syncthreads();  // the padded terms' table
      first = false;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t s = c0 + r * 64 + lane;
      if (s >= c1 || live[r] || (a.pix_count && (a.flags & PR_SHADE_LIVE_ONLY))) continue;
      const V3 c = pad_colour(a, s, img[r], tab, pad);
      float* o = a.colors + s * 3;
      o[0] = c.x; o[1] = c.y; o[2] = c.z;
    }
    __builtin_amdgcn_wave_barrier();  // the list is rewritten by the wave's next pass
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

// flush the workgroup's partial sums: one global atomic per touched entry
PR_DEV void flush_table(const PRShadeArgs& a, const Tab& tab, const float* lds) {
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

// PR_DETERMINISTIC: instead of scattering, every slot writes its contributions as entries of
// three ordered scatter-adds (pr_detsum.hip): per-vertex (slot corner i: verts | normals |
// vertex colours, 9 components), per-batch (light | camera, 6) and per-texel (bilinear corner,
// 3); padded slots write dropped keys.
struct ShadeDet {
  DetSum v, b, m;  // n == 0: not requested
};

PR_DEV void put3(float* p, V3 g) { p[0] = g.x; p[1] = g.y; p[2] = g.z; }

// padded slot: only the texel term can carry a gradient (p = n = 0: no light, no specular)
template <bool DET>
PR_DEV void pad_bwd(const PRShadeArgs& a, int64_t s, int64_t ds, int n, const ShadeDet& det) {
  if (a.grad_bary && !(a.pix_count && (a.flags & PR_SHADE_LIVE_ONLY))) {
    a.grad_bary[s * 3] = 0.f; a.grad_bary[s * 3 + 1] = 0.f; a.grad_bary[s * 3 + 2] = 0.f;
  }
  if (a.texture == PR_TEX_GIVEN && a.grad_texels) {
    const V3 g = v3(a.ambient + n * 3) * v3(a.grad_colors + s * 3);
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
}

// valid slot whose d colour is exactly 0 (every slot the blend gave no weight: all but the
// winners of some Monte-Carlo sample): every gradient it carries is 0 (finite shading terms times
// 0), so only its zero d bary (and zero d texel) is written -- the chain rule runs for the others
template <bool DET>
PR_DEV void zero_bwd(const PRShadeArgs& a, int64_t s, int64_t ds, const ShadeDet& det) {
  if (a.grad_bary) { a.grad_bary[s * 3] = 0.f; a.grad_bary[s * 3 + 1] = 0.f; a.grad_bary[s * 3 + 2] = 0.f; }
  if (a.texture == PR_TEX_GIVEN && a.grad_texels) {
    float* o = a.grad_texels + s * 3;
    o[0] = 0.f; o[1] = 0.f; o[2] = 0.f;
  }
  if (DET) {
    if (det.v.n)
      for (int i = 0; i < 3; ++i) det.v.keys[ds * 3 + i] = (uint32_t)det.v.M;
    if (det.b.n) det.b.keys[ds] = (uint32_t)det.b.M;
    if (det.m.n)
      for (int c = 0; c < 4; ++c) det.m.keys[ds * 4 + c] = (uint32_t)det.m.M;
  }
}

// live slot: per-slot chain rule in registers (phong_bwd), scatters into the LDS table (or the
// ordered sums)
template <bool DET>
PR_DEV void slot_bwd(const PRShadeArgs& a, const Slot& sl, int64_t s, int64_t ds, const Tab& tab,
                     const ShadeDet& det, float* lds) {
  const int n = sl.n;
  const int64_t* fv = a.faces + sl.f * 3;
  const PhongGrad q = phong_bwd(a, sl, s, fv, v3(a.grad_colors + s * 3));
  const float* b = sl.b;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int64_t vi = fv[i];
    if (DET) {
      if (det.v.n) {
        det.v.keys[ds * 3 + i] = (uint32_t)vi;
        float* e = det.v.vals + (ds * 3 + i) * 9;
        put3(e, b[i] * q.g_P);
        put3(e + 3, b[i] * q.g_Nn);
        put3(e + 6, a.texture == PR_TEX_VERTEX ? b[i] * q.g_tex : V3{0.f, 0.f, 0.f});
      }
      continue;
    }
    if (a.grad_verts) acc(lds, tab.useV, tab.vOff + (int)vi * 3, a.grad_verts, vi, b[i] * q.g_P);
    if (a.grad_normals) acc(lds, tab.useV, tab.nOff + (int)vi * 3, a.grad_normals, vi, b[i] * q.g_Nn);
    if (a.texture == PR_TEX_VERTEX && a.grad_vert_colors)
      acc(lds, tab.useV, tab.cOff + (int)vi * 3, a.grad_vert_colors, vi, b[i] * q.g_tex);
  }
  if (a.texture == PR_TEX_GIVEN) {
    if (a.grad_texels) {
      float* o = a.grad_texels + s * 3;
      o[0] = q.g_tex.x; o[1] = q.g_tex.y; o[2] = q.g_tex.z;
    }
  } else if (a.texture == PR_TEX_UV) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool in = q.ti[c] >= 0;
      if (DET && det.m.n) {
        det.m.keys[ds * 4 + c] = in ? (uint32_t)((int64_t)n * a.Hm * a.Wm + q.ti[c] / 3) : (uint32_t)det.m.M;
        if (in) put3(det.m.vals + (ds * 4 + c) * 3, q.w[c] * q.g_tex);
      }
      if (!DET && in && a.grad_maps) {
        float* gm = a.grad_maps + (int64_t)n * a.Hm * a.Wm * 3 + q.ti[c];
        atomicAdd(&gm[0], q.w[c] * q.g_tex.x); atomicAdd(&gm[1], q.w[c] * q.g_tex.y);
        atomicAdd(&gm[2], q.w[c] * q.g_tex.z);
      }
    }
  }
  if (a.grad_bary) { a.grad_bary[s * 3] = q.gb[0]; a.grad_bary[s * 3 + 1] = q.gb[1]; a.grad_bary[s * 3 + 2] = q.gb[2]; }
  if (DET) {
    if (det.b.n) {
      det.b.keys[ds] = (uint32_t)n;
      put3(det.b.vals + ds * 6, q.g_dir);
      put3(det.b.vals + ds * 6 + 3, q.g_vraw);
    }
    return;
  }
  if (a.grad_light) acc(lds, tab.useB, tab.lOff + n * 3, a.grad_light, n, q.g_dir);
  if (a.grad_camera) acc(lds, tab.useB, tab.camOff + n * 3, a.grad_camera, n, q.g_vraw);
}

// (slots [s0, PK): the deterministic mode runs the frame in batches; the fast path s0 = 0)
template <bool DET, int R>
__global__ void __launch_bounds__(kThreads) shade_bwd_kernel(PRShadeArgs a, int64_t s0, int64_t PK, int64_t HW,
                                                             Tab tab, ShadeDet det, int idx32) {
  extern __shared__ float lds[];
  __shared__ int lists[kWaves][64 * R];
  const bool i32 = idx32 != 0;
  const int lane = threadIdx.x & 63;
  int* list = lists[threadIdx.x >> 6];
  const int q64 = 64 / a.K, r64 = 64 - q64 * a.K;
  if (!DET) {
    for (int i = threadIdx.x; i < tab.size; i += kThreads) lds[i] = 0.f;
    __syncthreads();
  }
  PR_WAVE_CHUNKS(R, s0, PK, c0, c1) {
    bool live[R], zero[R];
    int img[R];
    SlotPos q = slot_pos(c0 + lane, a.K, HW, i32);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t s = c0 + r * 64 + lane;
      const bool valid = s < c1 && (a.pix_count ? q.k < a.pix_count[q.p] : a.pix_to_face[s] >= 0);
      // (the list holds the slots with a non-zero d colour only: on a perturbed-blend frame those are
      // the slots that won a sample, a fraction of the valid ones)
      const float* gc = a.grad_colors + s * 3;
      zero[r] = valid && gc[0] == 0.f && gc[1] == 0.f && gc[2] == 0.f;
      live[r] = valid && !zero[r];
      img[r] = q.n;
      if (r + 1 < R) step64(q, a.K, HW, q64, r64);
    }
    const int total = wave_compact(live, list);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t s = c0 + r * 64 + lane;
      if (zero[r]) zero_bwd<DET>(a, s, s - s0, det);
      else if (s < c1 && !live[r]) pad_bwd<DET>(a, s, s - s0, img[r], det);
    }
    for (int i = lane; i < total; i += 64) {
      const int64_t s = c0 + list[i];
      const Slot sl = load_slot(a, s, HW, i32);
      if (sl.f >= 0) slot_bwd<DET>(a, sl, s, s - s0, tab, det, lds);
      else pad_bwd<DET>(a, s, s - s0, sl.n, det);
    }
    __builtin_amdgcn_wave_barrier();  // the list is rewritten by the wave's next chunk
  }
  if (DET) return;
  __syncthreads();
  flush_table(a, tab, lds);
}

// ---- pixel-block forward: valid-prefix counts attached, texels not given per slot -------------
// A workgroup takes kBlkPix consecutive pixels (kBlkPix K slots).  Wave 0 loads their counts and
// scans them into LDS; the padded slots [count, K) of every pixel are then written as 16-byte
// stores of the image's colour pattern with no per-slot liveness test (fill_padded), and the live
// slots [0, count) are enumerated from the prefix and shaded one per thread.  Measured on the
// eval frame (profiles/r5/shade.md): 18.7 us against 21.4 us for the per-wave chunk kernel.  The
// backward keeps the chunk kernel: the same layout for it (d bary zeros as the padded pattern)
// measured 30 us against 26 us -- its time is the live slots' load chain and arithmetic, which
// the layout does not shorten.
constexpr int kBlkPix = 64;

struct PixBlock {
  int cnt[kBlkPix];   // live slots of the pixel (the count, clamped to [0, K])
  int incl[kBlkPix];  // inclusive prefix of cnt
  int img[kBlkPix];   // image of the pixel
};

// wave 0: the block's counts, their scan and the pixels' images
PR_DEV void pix_block_load(const PRShadeArgs& a, int64_t p0, int npix, int64_t HW, PixBlock& pb) {
  if (threadIdx.x >= 64) return;
  const int l = threadIdx.x;
  int c = 0, n = 0;
  if (l < npix) {
    c = a.pix_count[p0 + l];
    c = c < 0 ? 0 : (c > a.K ? a.K : c);
    n = (int)((p0 + l) / HW);
  }
  int v = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (l >= o) v += t;
  }
  pb.cnt[l] = c;
  pb.incl[l] = v;
  pb.img[l] = n;
}

// live entry i of the block -> its slot (pixel: the first whose inclusive prefix exceeds i)
PR_DEV int64_t live_slot(const PRShadeArgs& a, const PixBlock& pb, int64_t p0, int i, Slot& sl) {
  int pl = 0;
#pragma unroll
  for (int step = kBlkPix / 2; step; step >>= 1)
    if (pb.incl[pl + step - 1] <= i) pl += step;
  const int k = i - (pb.incl[pl] - pb.cnt[pl]);
  const int64_t s = (p0 + pl) * a.K + k;
  sl.n = pb.img[pl];
  sl.f = a.pix_to_face[s];
  if (sl.f >= 0) {
    sl.b[0] = a.bary[s * 3]; sl.b[1] = a.bary[s * 3 + 1]; sl.b[2] = a.bary[s * 3 + 2];
  } else {
    sl.b[0] = sl.b[1] = sl.b[2] = 0.f;
  }
  return s;
}

// x / K for block slot offsets x < kBlkPix K: a multiply-high by mag = ceil(2^32 / K), exact while
// x K < 2^32 (K < 8192 here); mag = 0 divides
PR_DEV int div_k(int x, int K, uint32_t mag) { return mag ? (int)__umulhi((uint32_t)x, mag) : x / K; }

uint32_t k_magic(int K) { return K >= 2 && K < 8192 ? (uint32_t)(((1ull << 32) + K - 1) / K) : 0u; }

// the padded colour c of every image (texture != PR_TEX_GIVEN: no per-slot term) as its three
// 16-byte phases: pat[3 n + j] = (c[j], c[j+1], c[j+2], c[j]) (components mod 3).  Threads t0..
PR_DEV void pad_patterns(const PRShadeArgs& a, float4* pat, int t0) {
  for (int n = (int)threadIdx.x - t0; n >= 0 && n < a.N; n += kThreads - t0) {
    const Terms t = slot_terms(a, pad_slot(n), -1, nullptr);
    const V3 c = colour(t.lit, t.tex, t.spec);
    pat[3 * n] = make_float4(c.x, c.y, c.z, c.x);
    pat[3 * n + 1] = make_float4(c.y, c.z, c.x, c.y);
    pat[3 * n + 2] = make_float4(c.z, c.x, c.y, c.z);
  }
}

// The padded slots of the block as 16-byte stores, consecutive lanes on consecutive float4s (each
// store instruction writes 1 KB of contiguous memory): float4 q holds floats 4q..4q+3, i.e. the
// components ph, ph+1, ph+2, ph (mod 3) of slots sa = 4q / 3 and sa + 1 -- the phase-ph pattern of
// the image.  Both slots padded and of one image: one store; one padded: its floats one by one
// (component j of a slot = float j of the phase-0 pattern).  No loop and no division on either
// path: a wave-instruction spans ~1.7 pixels, so a pixel boundary lane is in nearly every one and
// its path is paid by the whole wave.
PR_DEV void fill_padded(float* out, const PixBlock& pb, int64_t p0, int npix, int K, uint32_t kmag,
                        const float4* pat) {
  const int nf = npix * K * 3, nq = (nf + 3) / 4;
  float* base = out + p0 * K * 3;
  for (int q = threadIdx.x; q < nq; q += kThreads) {
    const int f0 = 4 * q, sa = f0 / 3, ph = f0 - 3 * sa;
    const int pl = div_k(sa, K, kmag), k = sa - pl * K;
    const bool next = k + 1 == K;  // slot sa + 1 opens pixel pl + 1
    const int pl1 = next ? (pl + 1 < npix ? pl + 1 : pl) : pl;
    const int c0 = pb.cnt[pl];
    const bool pad0 = k >= c0;
    const bool pad1 = next ? (pl + 1 < npix && pb.cnt[pl1] == 0) : k + 1 >= c0;
    if (!pad0 && !pad1) continue;
    const int n0 = pb.img[pl], n1 = pb.img[pl1];
    if (pad0 && pad1 && n0 == n1 && f0 + 3 < nf) {
      reinterpret_cast<float4*>(base)[q] = pat[3 * n0 + ph];
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool second = ph + j >= 3;
      if (f0 + j < nf && (second ? pad1 : pad0))
        base[f0 + j] = reinterpret_cast<const float*>(pat + 3 * (second ? n1 : n0))[ph + j - (second ? 3 : 0)];
    }
  }
}

// grid-stride over pixel blocks; every thread runs the same trip count (the barriers)
#define PR_PIX_BLOCKS(P, p0, npix)                                                                     \
  for (int64_t p0 = (int64_t)blockIdx.x * kBlkPix, npix; npix = (P) - p0 < kBlkPix ? (int)((P) - p0) : kBlkPix, \
       p0 < (P); p0 += (int64_t)gridDim.x * kBlkPix)

__global__ void __launch_bounds__(kThreads) shade_fwd_pix_kernel(PRShadeArgs a, int64_t P, int64_t HW,
                                                                  uint32_t kmag) {
  __shared__ PixBlock pb;
  __shared__ float4 pat[kPadImgs * 3];
  zero_accumulators(a);
  pad_patterns(a, pat, 64);
  PR_PIX_BLOCKS(P, p0, npix) {
    pix_block_load(a, p0, (int)npix, HW, pb);
    __syncthreads();  // (the first also publishes the patterns)
    // the padded stores first: they drain while the live slots' load chains run
    if (!(a.flags & PR_SHADE_LIVE_ONLY)) fill_padded(a.colors, pb, p0, (int)npix, a.K, kmag, pat);
    const int total = pb.incl[kBlkPix - 1];
    for (int i = threadIdx.x; i < total; i += kThreads) {
      Slot sl;
      const int64_t s = live_slot(a, pb, p0, i, sl);
      float* o = a.colors + s * 3;
      if (sl.f >= 0) {
        const Terms t = slot_terms(a, sl, s, a.faces + sl.f * 3);
        const V3 c = colour(t.lit, t.tex, t.spec);
        o[0] = c.x; o[1] = c.y; o[2] = c.z;
      } else {  // a counted slot without a face (not produced by the rasterizer): padding
        const float4 c = pat[3 * sl.n];
        o[0] = c.x; o[1] = c.y; o[2] = c.z;
      }
    }
    __syncthreads();  // pb is rewritten by the next block
  }
}

// Pixel-block backward (counts attached, no per-slot texels, fast path): the block's valid slots are
// enumerated from the counts' prefix (the padded ones only get their zero d bary, and none with
// PR_SHADE_LIVE_ONLY), and the chain rule runs for the valid slots with a non-zero d colour: on a
// perturbed-blend frame those are the slots that won a sample (pr_blend_bwd's d colour is wins / Sa
// times g_rgb), a fraction of the valid ones; the chunked kernel walked every slot of the frame.
__global__ void __launch_bounds__(kThreads) shade_bwd_pix_kernel(PRShadeArgs a, int64_t P, int64_t HW, Tab tab,
                                                                 uint32_t kmag) {
  extern __shared__ float lds[];
  __shared__ PixBlock pb;
  for (int i = threadIdx.x; i < tab.size; i += kThreads) lds[i] = 0.f;
  const bool live_only = a.flags & PR_SHADE_LIVE_ONLY;
  PR_PIX_BLOCKS(P, p0, npix) {
    pix_block_load(a, p0, (int)npix, HW, pb);
    __syncthreads();  // (the first also publishes the zeroed table)
    if (!live_only && a.grad_bary) {
      for (int x = threadIdx.x; x < (int)npix * a.K; x += kThreads) {
        const int pl = div_k(x, a.K, kmag), k = x - pl * a.K;
        if (k < pb.cnt[pl]) continue;
        float* o = a.grad_bary + ((p0 + pl) * a.K + k) * 3;
        o[0] = 0.f; o[1] = 0.f; o[2] = 0.f;
      }
    }
    const int total = pb.incl[kBlkPix - 1];
    for (int i = threadIdx.x; i < total; i += kThreads) {
      Slot sl;
      const int64_t s = live_slot(a, pb, p0, i, sl);
      const float* gc = a.grad_colors + s * 3;
      if (sl.f < 0 || (gc[0] == 0.f && gc[1] == 0.f && gc[2] == 0.f)) {
        zero_bwd<false>(a, s, s, ShadeDet{});
        continue;
      }
      slot_bwd<false>(a, sl, s, s, tab, ShadeDet{}, lds);
    }
    __syncthreads();  // pb is rewritten by the next block
  }
  flush_table(a, tab, lds);
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

// the frame's slot indices fit 32-bit arithmetic (shade kernels: slot_index)
int idx32(const PRShadeArgs& a) { return (int64_t)a.N * a.H * a.W * a.K < (int64_t(1) << 31) ? 1 : 0; }

// slots per lane and pass of the shading kernels: PR_SHADE_ROUNDS (4, 8, 12 or 16)
int shade_rounds() {
  static const int r = [] {
    const char* e = getenv("PR_SHADE_ROUNDS");
    const int v = e ? atoi(e) : kRoundsDefault;
    return v == 4 || v == 12 || v == 16 ? v : 8;
  }();
  return r;
}

// the pixel-block kernels apply: counts attached, no per-slot texels, the images' padded colours
// fit the LDS patterns, 16-byte aligned outputs
// (PR_SHADE_PIX=0 forces the per-slot kernels; read per call: tests compare both)
bool pix_path(const PRShadeArgs& a, const float* out) {
  const char* e = getenv("PR_SHADE_PIX");
  if (e && e[0] == '0') return false;
  return a.pix_count && a.texture != PR_TEX_GIVEN && a.N <= kPadImgs &&
         (!out || (reinterpret_cast<uintptr_t>(out) & 15) == 0);
}

int pix_blocks(int64_t P) { return (int)std::min<int64_t>((P + kBlkPix - 1) / kBlkPix, 4096); }

// workgroups of the chunked kernels (64 R slots per wave and chunk): at most 8 per CU, the waves
// stride over the chunks
int shade_blocks(int64_t PK, int R) {
  const int64_t chunk = (int64_t)R * kThreads;
  return (int)std::min<int64_t>((PK + chunk - 1) / chunk, 2048);
}

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
    shade_bwd_kernel<true, kRoundsDefault><<<shade_blocks(nb, kRoundsDefault), kThreads, 0, st>>>(
        a, s0, s0 + nb, (int64_t)a.H * a.W, tab, det, idx32(a));
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
    split_kernel<<<shade_blocks(a.V * 9, 1), kThreads, 0, st>>>(out9, a.V, 9, a.grad_verts, a.grad_normals,
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
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t HW = (int64_t)a.H * a.W;
  if (pix_path(a, a.colors)) {
    const int64_t P = (int64_t)a.N * HW;
    shade_fwd_pix_kernel<<<pix_blocks(P), kThreads, 0, st>>>(a, P, HW, k_magic(a.K));
    return check_launch("shade_fwd");
  }
  const int R = shade_rounds();
  if (R == 4) shade_fwd_kernel<4><<<shade_blocks(PK, 4), kThreads, 0, st>>>(a, PK, HW, idx32(a));
  else if (R == 12) shade_fwd_kernel<12><<<shade_blocks(PK, 12), kThreads, 0, st>>>(a, PK, HW, idx32(a));
  else if (R == 16) shade_fwd_kernel<16><<<shade_blocks(PK, 16), kThreads, 0, st>>>(a, PK, HW, idx32(a));
  else shade_fwd_kernel<8><<<shade_blocks(PK, 8), kThreads, 0, st>>>(a, PK, HW, idx32(a));
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
  // (PR_GRAD_PREZEROED: the forward zeroed the small accumulators; the map gradient is zeroed here)
  const bool pre = a.flags & PR_GRAD_PREZEROED;
  struct Z { float* p; size_t n; } zs[] = {
      {pre ? nullptr : a.grad_verts, (size_t)a.V * 3}, {pre ? nullptr : a.grad_normals, (size_t)a.V * 3},
      {a.texture == PR_TEX_VERTEX && !pre ? a.grad_vert_colors : nullptr, (size_t)a.V * 3},
      {a.texture == PR_TEX_UV ? a.grad_maps : nullptr, (size_t)a.N * a.Hm * a.Wm * 3},
      {pre ? nullptr : a.grad_light, (size_t)a.N * 3}, {pre ? nullptr : a.grad_camera, (size_t)a.N * 3}};
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
  const size_t sh = (size_t)tab.size * sizeof(float);
  const int64_t HW = (int64_t)a.H * a.W;
  if (pix_path(a, nullptr)) {
    const int64_t P = (int64_t)a.N * HW;
    static const int cap_env = getenv("PR_SHADE_BWD_BLOCKS") ? atoi(getenv("PR_SHADE_BWD_BLOCKS")) : 0;
    const int nbp = std::min(pix_blocks(P), cap_env > 0 ? cap_env : (tab.size > 1024 ? 1024 : 4096));
    shade_bwd_pix_kernel<<<nbp, kThreads, sh, st>>>(a, P, HW, tab, k_magic(a.K));
    return check_launch("shade_bwd");
  }
  const int R = shade_rounds();
  const int nb = std::min(shade_blocks(PK, R), tab.size > 1024 ? 1024 : 16384);
  if (R == 4) shade_bwd_kernel<false, 4><<<nb, kThreads, sh, st>>>(a, 0, PK, HW, tab, ShadeDet{}, idx32(a));
  else if (R == 12) shade_bwd_kernel<false, 12><<<nb, kThreads, sh, st>>>(a, 0, PK, HW, tab, ShadeDet{}, idx32(a));
  else if (R == 16) shade_bwd_kernel<false, 16><<<nb, kThreads, sh, st>>>(a, 0, PK, HW, tab, ShadeDet{}, idx32(a));
  else shade_bwd_kernel<false, 8><<<nb, kThreads, sh, st>>>(a, 0, PK, HW, tab, ShadeDet{}, idx32(a));
  return check_launch("shade_bwd");
}
