/*
 * pertrender.h — C ABI of the MI355X-native perturbed differentiable renderer
 * (libpertrender.so, built for gfx950 by pertrenderer_amd/build_native.py).
 *
 * Drop-in boundary for the hot path of quentinll/pertrenderer (reference
 * checkout: randomras/ *.py).  All buffers are device pointers owned by the
 * caller (PyTorch's caching allocator); the library allocates nothing
 * persistent.  Every entry point enqueues on the given HIP stream
 * (hipStream_t passed as void*) and returns 0 on success or a negative
 * PR_ERR_* code; pr_last_error() returns a thread-local message.
 *
 * Layouts are PyTorch3D's: Fragments are (N,H,W,K) row-major, K fastest;
 * pix_to_face is int64, everything else float32; colours (N,H,W,K,3);
 * images (N,H,W,4).  P = N*H*W pixels.
 *
 * Reference interfaces each entry point replaces (the reference is pure
 * Python; these are the calls whose tensor work moves here):
 *   pr_blend_fwd / pr_blend_bwd
 *       random_rasterizer.py:34-56   smooth_rgb_blend with
 *       smoothrast.py:136-147        GaussianRast.rasterize  -> randomHeaviside (:12-59)
 *       smoothagg.py:185-205         GaussianAgg.aggregate   -> randomArgmax   (:10-73)
 *       smoothagg.py:292-337         log_corrected / prod_corrected
 *     flags select the fused shader path (RAST|COLOR) or the standalone
 *     GaussianAgg.aggregate (flags = 0: prob in, weights (N,H,W,K+1) out).
 *   pr_heaviside_fwd / pr_heaviside_bwd
 *       smoothrast.py:144-147 GaussianRast.rasterize standalone (randomHeaviside).
 *   pr_rast_fwd / pr_rast_bwd
 *       PyTorch3D 0.4.0 rasterize_meshes / its backward, as called by
 *       MeshRasterizer at experiments/eval.py:165-168 (requirements.txt:7).
 *   pr_interp_fwd / pr_interp_bwd
 *       PyTorch3D interpolate_face_attributes used by Meshes.sample_textures
 *       for TexturesVertex (random_rasterizer.py:170, experiments/eval.py:251).
 *   pr_vert_normals_fwd / pr_vert_normals_bwd
 *       PyTorch3D Meshes.verts_normals_packed, the vertex normals phong_shading
 *       interpolates for RandomPhongShader (random_rasterizer.py:60-116).
 */
#ifndef PERTRENDER_H_
#define PERTRENDER_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PR_ABI_VERSION 20

/* error codes */
#define PR_OK 0
#define PR_ERR_ARG -1     /* bad shape / null pointer / unsupported value */
#define PR_ERR_HIP -2     /* HIP launch or runtime error */
#define PR_ERR_WORKSPACE -3

/* noise sources */
#define PR_NOISE_PHILOX 0   /* in-kernel Philox4x32-10 keyed by (seed, pixel, slot, sample); */
                            /* N(0,1) by Box-Muller, Cauchy by tan(pi (u - 1/2))             */
#define PR_NOISE_INJECTED 1 /* caller-provided N(0,1) tensors (reference-parity mode) */

#define PR_BLEND_SYNC_BYTES 1024 /* PRBlendFwdArgs.sync */

/* pr_blend flags */
#define PR_BLEND_RAST 1  /* probabilities from dists via the perturbed Heaviside (else `prob` input) */
#define PR_BLEND_COLOR 2 /* colour mix + alpha -> image (else weights (N,H,W,K+1) out) */
#define PR_BLEND_VERTEX 4 /* with COLOR: slot colours interpolated on demand from per-vertex    */
                          /* colours (TexturesVertex.sample_textures fused; no texel tensor)    */
/* noise variants; also valid in PRHeavisideArgs.flags (RAST bits) */
#define PR_BLEND_RAST_CAUCHY 8  /* ArctanRast: Cauchy rast noise, score 2e/(1+e^2) (smoothrast.py:162-173) */
#define PR_BLEND_AGG_CAUCHY 16  /* CauchyAgg: Cauchy agg noise (smoothagg.py:230-250)                    */
#define PR_BLEND_RAST_WOVR 32   /* GaussianRast_wovr: score without the vr baseline (smoothrast.py:61-108) */
#define PR_BLEND_AGG_WOVR 64    /* GaussianAgg_wovr: a_s = <g, w_s> (smoothagg.py:75-141; Cauchy keeps vr) */
/* deterministic SoftRast + SoftAgg (smoothrast.py:126-134, smoothagg.py:165-182; eval.py's
 * "softras" renderer): P = sigmoid(-d / sigma), W = softmax(z / gamma); with RAST | COLOR and
 * texel colours; Sr / Sa / noise fields are ignored, winners / rast_cache are not written */
#define PR_BLEND_SOFT 128
/* UniformAgg: U(-1/2, 1/2) agg noise (smoothagg.py:28-30, 252-271); forward only -- the
 * reference's backward has no uniform branch and fails (smoothagg.py:64-70), so
 * pr_blend_bwd rejects the flag with PR_ERR_ARG */
#define PR_BLEND_AGG_UNIFORM 256
/* Forward only (ABI 16): `winners` (P,Sa) is an INPUT -- the per-sample argmax indices of all Sa
 * samples, gathered from sample shards (pertrenderer_amd.multidevice) -- instead of the Monte-Carlo
 * argmax: the same win counts and the same colour mix, so the image is the one-device image bit
 * for bit.  With !RAST (prob input); no agg noise is read. */
#define PR_BLEND_WINNERS_IN 512
#define PR_BLEND_LIVE_ONLY 1024 /* with RAST and pix_count: pr_blend_bwd leaves the masked slots' d zbuf / d dists / */
                                /* d colour / d bary unwritten, for a caller whose consumers read the valid prefix */
                                /* only (the rasterizer backward, the live-only shading; ABI 19) */
#define PR_BLEND_PHONG 2048     /* pr_blend_fwd with RAST | COLOR (not VERTEX): each slot's colour is Phong-     */
                                /* shaded on demand from `shade` (PRShadeArgs: mesh, vertex normals, TexturesUV */
                                /* map or vertex colours, lights, materials, camera) -- RandomPhongShader's     */
                                /* sample_textures -> phong_shading -> smooth_rgb_blend (random_rasterizer.py:  */
                                /* 99-116) shading only the slots that win a sample.  With `colors` given (an   */
                                /* OUTPUT here) the colours of exactly the slots the backward reads -- the      */
                                /* winners and each pixel's unperturbed argmax -- are written there, nothing    */
                                /* else; the non-null shade.grad_verts / grad_normals / grad_vert_colors        */
                                /* (VERTEX) / grad_light / grad_camera are zeroed, for a PR_GRAD_PREZEROED      */
                                /* pr_shade_bwd (ABI 20)                                                        */
#define PR_BLEND_COLOR_SPARSE 4096 /* pr_blend_bwd with RAST | COLOR: `colors` holds valid values at the slots */
                                /* PR_BLEND_PHONG's forward wrote only; d colors as usual (then pr_shade_bwd)   */

struct PRShadeArgs;

typedef struct PRBlendParams {
  int32_t N, H, W, K;        /* fragment shape */
  int32_t Sr, Sa;            /* rast / agg Monte-Carlo samples of this call (shard) */
  int32_t sample_offset_r;   /* global index of this shard's first rast sample (Philox) */
  int32_t sample_offset_a;   /* global index of this shard's first agg sample (Philox) */
  float sigma, gamma, alpha, eps;
  float background[3];
  int32_t noise_mode;        /* PR_NOISE_* */
  uint64_t seed_r, seed_a;   /* Philox keys */
  const float* noise_r;      /* injected: (Sr,N,H,W,K)   */
  const float* noise_a;      /* injected: (Sa,N,H,W,K+1) */
  const float* znear;        /* (N,) camera near plane per batch element */
  const float* zfar;         /* (N,) */
  int32_t flags;             /* PR_BLEND_* */
  /* graph-capture support (both nullable):                                    */
  const float* scalars[3];   /* nullable device 0-d sigma, gamma, alpha (the leaves' own storage); */
                             /* each non-null one overrides its by-value field                   */
  const uint64_t* seeds;     /* device [base]; Philox keys become mix64(base ^ seed_r/a),  */
                             /* so a captured graph draws fresh noise after pr_seed_advance; */
                             /* a seed_r/seed_a with bit 63 set is used as-is (fixed noise) */
} PRBlendParams;

typedef struct PRBlendFwdArgs {
  PRBlendParams p;
  const int64_t* pix_to_face; /* (N,H,W,K); mask = p2f >= 0.  Either this or `mask`. */
  const uint8_t* mask;        /* (N,H,W,K) bool, used when pix_to_face is NULL */
  const float* dists;         /* RAST: (N,H,W,K) signed squared distances */
  const float* prob;          /* !RAST: (N,H,W,K) probabilities */
  const float* zbuf;          /* (N,H,W,K) */
  const float* colors;        /* COLOR: (N,H,W,K,3) */
  float* image;               /* COLOR out: (N,H,W,4) */
  float* weights;             /* !COLOR out: (N,H,W,K+1) */
  uint8_t* winners;           /* out: (P,Sa) per-sample argmax index, saved for backward */
  float* rast_cache;          /* RAST, nullable out: (N,H,W,K,2) per-slot (prob, rast score mean);  */
                              /* handed to pr_blend_bwd it replaces regenerating the rast noise    */
  /* VERTEX: colour of slot (p,k) = sum_i bary[p,k,i] * vert_colors[faces[p2f[p,k],i]] (0 if p2f<0) */
  const float* bary;          /* (N,H,W,K,3) */
  const int64_t* faces;       /* (F,3) packed vertex indices */
  const float* vert_colors;   /* (V,3) packed per-vertex colours */
  /* nullable (N,H,W) valid-prefix counts of pix_to_face (pr_rast_fwd's pix_count): mask = k < */
  /* count, and no fragment tensor is read at masked slots                                   */
  const int32_t* pix_count;
  /* nullable (needs pix_count), out: >= pr_blend_plan_size(&p) bytes (0: no plan for this call;
   * plans are opt-in, PR_BLEND_SEG=1).  Given, the call first cuts the pixel blocks of the forward
   * and of the backward into entry-balanced segments (a block's valid slots + background entries
   * split into parts of about the same count) and both kernels run one workgroup per segment;
   * keep it for pr_blend_bwd */
  int32_t* plan;
  /* nullable, >= PR_BLEND_SYNC_BYTES: arrival counters the forward zeroes; handed to pr_blend_bwd of
   * the same call, its last workgroup reduces d sigma / d gamma / d alpha (no finalize kernel).
   * Partials are written by device-scope atomic exchanges (no release fence); measured equal to
   * the separate finalize kernel at cfg 2 in graph mode, one launch fewer in eager mode: the
   * package passes it unless PR_BLEND_SYNC=0 */
  int32_t* sync;
  /* PHONG: the shading inputs (texture PR_TEX_UV or PR_TEX_VERTEX; its N,H,W,K, pix_to_face, pix_count, */
  /* bary are the blend's own and ignored; its colors / grad_colors / grad_bary / grad_maps ignored).   */
  /* Host memory, read during the call (the kernels get a copy).  The blend's `bary` is the fragments'  */
  /* barycentrics.                                                                                    */
  const struct PRShadeArgs* shade;
} PRBlendFwdArgs;

typedef struct PRBlendBwdArgs {
  PRBlendParams p;
  const int64_t* pix_to_face;
  const uint8_t* mask;
  const float* dists;
  const float* prob;
  const float* zbuf;
  const float* colors;
  const uint8_t* winners;     /* from pr_blend_fwd */
  const float* grad_image;    /* COLOR: (N,H,W,4) */
  const float* grad_weights;  /* !COLOR: (N,H,W,K+1) */
  float* grad_dists;          /* RAST out (N,H,W,K) */
  float* grad_prob;           /* !RAST out (N,H,W,K) */
  float* grad_zbuf;           /* out (N,H,W,K) */
  float* grad_colors;         /* COLOR out (N,H,W,K,3) */
  float* grad_scalars;        /* out (3,): d sigma, d gamma, d alpha */
  void* workspace;            /* >= pr_blend_bwd_workspace_size(args) bytes */
  size_t workspace_bytes;
  const float* rast_cache;    /* RAST, nullable: pr_blend_fwd's rast_cache of the same call */
  const float* bary;          /* VERTEX: as in PRBlendFwdArgs */
  const int64_t* faces;
  const float* vert_colors;
  float* grad_bary;           /* VERTEX out (N,H,W,K,3) (replaces grad_colors) */
  float* grad_vert_colors;    /* VERTEX out (V,3), nullable, accumulated (caller zeroes) */
  const int32_t* pix_count;   /* nullable: as in PRBlendFwdArgs (the same tensor as the forward's) */
  int32_t* plan;              /* nullable: the forward's plan of the same call (same params, pix_count) */
  int32_t* sync;              /* nullable: the forward's sync buffer of the same call */
  /* PHONG: as in PRBlendFwdArgs; its non-null grad_verts, grad_normals, grad_maps (UV) or     */
  /* grad_vert_colors (VERTEX), grad_light, grad_camera are ACCUMULATED (the caller zeroes them); */
  /* d bary goes to grad_bary (replaces grad_colors)                                            */
} PRBlendBwdArgs;

typedef struct PRHeavisideArgs {
  int32_t N, H, W, K, Sr, sample_offset_r, noise_mode;
  float sigma;
  uint64_t seed_r;
  const float* noise_r;       /* injected (Sr,N,H,W,K) */
  const float* dists;         /* (N,H,W,K); the op is applied to D = -dists */
  float* prob;                /* fwd out (N,H,W,K) */
  const float* grad_prob;     /* bwd in */
  float* grad_dists;          /* bwd out */
  float* grad_sigma;          /* bwd out (1,) */
  void* workspace;
  size_t workspace_bytes;
  const float* sigma_dev;     /* nullable device sigma (overrides `sigma`) */
  const uint64_t* seeds;      /* nullable device seed base (see PRBlendParams.seeds) */
  int32_t flags;              /* PR_BLEND_RAST_CAUCHY | PR_BLEND_RAST_WOVR */
} PRHeavisideArgs;

typedef struct PRRastArgs {
  const float* face_verts;          /* (F,3,3): x,y in NDC, z in view space */
  const int64_t* mesh_first_face;   /* (N,) first packed face of each mesh */
  const int64_t* mesh_num_faces;    /* (N,) */
  int64_t F;
  int32_t N, H, W, K;
  float blur_radius;                /* squared-distance threshold, as PyTorch3D */
  int32_t perspective_correct, clip_barycentric_coords, cull_backfaces;
  /* forward outputs */
  int64_t* pix_to_face; float* zbuf; float* bary; float* dists;
  /* backward */
  const float* grad_zbuf; const float* grad_bary; const float* grad_dists; /* nullable */
  float* grad_face_verts;           /* (F,3,3), overwritten */
  void* workspace;
  size_t workspace_bytes;
  /* nullable (N,H,W) valid-prefix counts: slots 0..count-1 of a pixel hold faces, the rest -1.  */
  /* Forward: written.  Backward: if set (the forward's), pix_to_face is read only below it.    */
  int32_t* pix_count;
  int32_t flags;                    /* PR_GRAD_PREZEROED: pr_rast_bwd does not zero grad_face_verts; */
                                    /* PR_DETERMINISTIC: slot-order face sums (needs the workspace)  */
  /* Coarse binning (forward; PyTorch3D RasterizationSettings.bin_size / max_faces_per_bin,      */
  /* rasterize_meshes.py).  bin_size > 0: the face pass appends every face to the bins of        */
  /* bin_size^2 pixels (rounded up to a multiple of 8) its blur-grown box overlaps, and each      */
  /* tile culls only its bin's list.  max_faces_per_bin bounds a bin's list; a bin that overflows */
  /* falls back to culling the whole mesh (PyTorch3D 0.4.0 writes past the list instead), so the  */
  /* fragments never depend on either knob.  bin_size <= 0: every tile culls the whole mesh.      */
  int32_t bin_size;
  int32_t max_faces_per_bin;
  /* nullable: the forward reads the blur threshold from this device float instead of          */
  /* blur_radius (ABI 18), so a captured graph replays with a blur the caller changes in place   */
  /* (eval.py's adaptive schedule lowers it every 50 iterations, eval.py:389-391)               */
  const float* blur_radius_dev;
} PRRastArgs;

typedef struct PRInterpArgs {
  const int64_t* pix_to_face;  /* (P*K) */
  const float* bary;           /* (P*K,3) */
  const float* face_attr;      /* (F,3,D) */
  int64_t PK, F;
  int32_t D;
  float* out;                  /* fwd (P*K,D) */
  const float* grad_out;       /* bwd in (P*K,D) */
  float* grad_bary;            /* bwd out (P*K,3), nullable */
  float* grad_face_attr;       /* bwd out (F,3,D), overwritten, nullable */
  const int64_t* faces;        /* nullable: if set, face_attr is per-VERTEX (V,D) and the kernel */
  int64_t V;                   /* gathers attr[faces[f][i]] itself; grad_face_attr is then (V,D) */
} PRInterpArgs;

/* World -> NDC projection of every face corner (MeshRasterizer.transform + the
 * face gather of rasterize_meshes, experiments/eval.py:165-168):
 *   v_view = [v,1] @ world_to_view[n] ; v_clip = [v_view,1] @ proj[n]
 *   face_verts[f,i] = (x_clip/w_clip, y_clip/w_clip, z_view)   (row-vector 4x4 matrices,
 *   PyTorch3D Transform3d convention).  Backward scatters d face_verts into d verts. */
typedef struct PRProjectArgs {
  const float* verts;          /* (V,3) packed world vertices */
  const int64_t* faces;        /* (F,3) packed vertex indices */
  const int64_t* mesh_first_face; /* (N,) */
  const int64_t* mesh_num_faces;  /* (N,) */
  const float* world_to_view;  /* (N,4,4) */
  const float* proj;           /* (N,4,4) */
  int64_t V, F;
  int32_t N;
  float* face_verts;           /* fwd out (F,3,3) */
  const float* grad_face_verts;/* bwd in (F,3,3) */
  float* grad_verts;           /* bwd out (V,3), overwritten */
  int32_t flags;               /* PR_GRAD_PREZEROED: pr_project_bwd does not zero grad_verts */
  /* nullable vertex -> face-corner index (CSR): the corners t = 3 f + i of vertex v are        */
  /* vert_corners[vert_corner_start[v] .. vert_corner_start[v+1]), in increasing t.  When set,   */
  /* pr_project_bwd gathers each vertex's corner gradients in that order (the order of the       */
  /* verts[faces] backward, PyTorch3D's face gather) and applies the projection Jacobian once    */
  /* per vertex: deterministic, no atomics.  Else one float atomic per corner component.         */
  const int64_t* vert_corner_start; /* (V+1) */
  const int64_t* vert_corners;      /* (3F) */
  /* nullable: deferred noise-key advances (ABI 16).  pr_project_rast_fwd's face pass applies     */
  /* pr_seed_advance's update to seed_advance[0], seed_advance_n times, before it returns: the    */
  /* caller's per-step key advance (pertrenderer_amd.noise.DeviceSeed) rides on the step's first  */
  /* native kernel instead of a launch of its own.  Ignored by pr_project_fwd / pr_project_bwd.   */
  uint64_t* seed_advance;
  int32_t seed_advance_n;
} PRProjectArgs;

/* Phong shading of every fragment slot: PyTorch3D 0.4.0 phong_shading (+ the texel lookup of
 * Meshes.sample_textures), the colour producer of RandomPhongShader (random_rasterizer.py:99-110,
 * used by experiments/eval.py:170):
 *   p = sum_i b_i verts[f_i],  n = sum_i b_i normals[f_i],  t = texel of the slot,
 *   d^ = normalize(light - p) (point) or normalize(light) (directional),  n^ = normalize(n),
 *   c = n^.d^,  diffuse = diffuse_color * relu(c),
 *   specular = specular_color * (relu(normalize(camera - p) . (2 c n^ - d^)) * [c > 0])^shininess,
 *   colour = (ambient + mat_diffuse * diffuse) * t + mat_specular * specular
 * (normalize(x) = x / max(|x|, 1e-6)).  Padded slots (pix_to_face < 0) shade p = n = 0 at uv = 0,
 * exactly like the reference composition.  All per-batch parameters are (N,3) / (N,) rows. */
#define PR_TEX_GIVEN 0   /* texels (N,H,W,K,3) given (any Textures.sample_textures output) */
#define PR_TEX_UV 1      /* TexturesUV: bilinear map lookup at the interpolated corner UVs */
#define PR_TEX_VERTEX 2  /* TexturesVertex: interpolated per-vertex colours */

typedef struct PRShadeArgs {
  int32_t N, H, W, K;
  const int64_t* pix_to_face;  /* (N,H,W,K) */
  const int32_t* pix_count;    /* nullable valid-prefix counts (N,H,W) */
  const float* bary;           /* (N,H,W,K,3) */
  const int64_t* faces;        /* (F,3) packed vertex indices */
  const float* verts;          /* (V,3) world positions */
  int32_t flags;               /* PR_DETERMINISTIC: the backward's per-vertex / per-texel / per-batch */
                               /* sums in slot order (pr_shade_bwd_workspace_size bytes of workspace) */
                               /* PR_GRAD_PREZEROED (backward): grad_verts / grad_normals / */
                               /* grad_vert_colors / grad_light / grad_camera were zeroed by the */
                               /* forward (below); grad_maps is still zeroed by the call */
  void* workspace;
  size_t workspace_bytes;
  const float* normals;        /* (V,3) vertex normals */
  int64_t V, F;
  int32_t texture;             /* PR_TEX_* */
  const float* texels;         /* GIVEN: (N,H,W,K,3) */
  const float* vert_colors;    /* VERTEX: (V,3) */
  const float* face_uvs;       /* UV: (F,3,2) corner UVs */
  const float* maps;           /* UV: (N,Hm,Wm,3), v = 0 is the bottom row; grid_sample bilinear, */
  int32_t Hm, Wm;              /*     align_corners=True, padding "border" (TexturesUV defaults)  */
  int32_t directional;         /* 0: point lights (light = location), 1: directional (light = direction) */
  const float* light;          /* (N,3) */
  const float* ambient;        /* (N,3) material ambient * light ambient */
  const float* diffuse_color;  /* (N,3) light diffuse colour */
  const float* specular_color; /* (N,3) light specular colour */
  const float* mat_diffuse;    /* (N,3) */
  const float* mat_specular;   /* (N,3) */
  const float* shininess;      /* (N,) */
  const float* camera;         /* (N,3) camera centres */
  float* colors;               /* fwd out (N,H,W,K,3) */
  /* backward: every non-null output is overwritten (accumulators are zeroed by the call, or by */
  /* the forward: pr_shade_fwd zeroes the non-null grad_verts, grad_normals, grad_vert_colors */
  /* (PR_TEX_VERTEX), grad_light and grad_camera it is given, for a PR_GRAD_PREZEROED backward) */
  const float* grad_colors;    /* (N,H,W,K,3) */
  float* grad_bary;            /* (N,H,W,K,3) */
  float* grad_verts;           /* (V,3) */
  float* grad_normals;         /* (V,3) */
  float* grad_texels;          /* GIVEN: (N,H,W,K,3) */
  float* grad_vert_colors;     /* VERTEX: (V,3) */
  float* grad_maps;            /* UV: (N,Hm,Wm,3) */
  float* grad_light;           /* (N,3) */
  float* grad_camera;          /* (N,3) */
} PRShadeArgs;

int pr_shade_fwd(const PRShadeArgs* args, void* stream);
size_t pr_shade_bwd_workspace_size(const PRShadeArgs* args);
int pr_shade_bwd(const PRShadeArgs* args, void* stream);

/* Area-weighted vertex normals of a packed mesh: PyTorch3D Meshes.verts_normals_packed (the
 * normals phong_shading interpolates for RandomPhongShader, random_rasterizer.py:60-116 via
 * eval.py's renderer).  Forward: normals = normalize(sum over each vertex's face corners of
 * cross(v_next - v_c, v_prev - v_c)), F.normalize's max(||n||, 1e-6); `raw` (nullable) keeps
 * the unnormalised sums for the backward.  Backward: grad_verts (overwritten) from
 * grad_normals, through grad_raw (caller scratch, (V,3)). */
typedef struct PRNormalsArgs {
  const float* verts;          /* (V,3) */
  const int64_t* faces;        /* (F,3) */
  int64_t V, F;
  float* normals;              /* fwd out (V,3) */
  float* raw;                  /* fwd out (V,3), nullable; bwd in */
  const float* grad_normals;   /* bwd in (V,3) */
  float* grad_raw;             /* bwd scratch (V,3) */
  float* grad_verts;           /* bwd out (V,3), overwritten */
  /* nullable vertex -> face-corner index (CSR, as in PRProjectArgs) listing each vertex's corners */
  /* in PyTorch3D's accumulation order: all corner-1 entries by face, then corner 2, then corner 0 */
  /* (its three index_adds).  When set, both passes gather per vertex in that order: one kernel    */
  /* per pass, deterministic, no atomics.  Else one thread per face with float atomics.            */
  const int64_t* vert_corner_start; /* (V+1) */
  const int64_t* vert_corners;      /* (3F) */
} PRNormalsArgs;

int pr_vert_normals_fwd(const PRNormalsArgs* args, void* stream);
int pr_vert_normals_bwd(const PRNormalsArgs* args, void* stream);

/* the backward's gradient accumulator was zeroed by the forward (pr_project_rast_fwd) */
#define PR_GRAD_PREZEROED 1
/* deterministic-order backward (PRRastArgs.flags, PRShadeArgs.flags): the sums that
 * the fast path scatters with float atomics are formed by a stable sort of the contributions by
 * target and in-order sums instead (pr_*_bwd_workspace_size reports the workspace they need).
 * pr_rast_bwd then sums every face's slot gradients in slot order, sequentially: the
 * accumulation order of PyTorch3D's CPU backward (and of oracle/rast_oracle.c), bit for bit. */
#define PR_DETERMINISTIC 2
#define PR_RAST_VALID_ONLY 8 /* pr_rast_fwd / pr_project_rast_fwd with pix_count: only each pixel's valid prefix of */
                             /* p2f / zbuf / bary / dists is written (a caller that reads nothing else; ABI 19) */
#define PR_SHADE_LIVE_ONLY 4 /* pr_shade_fwd / _bwd with pix_count: the padded slots' colours (forward) and */
                             /* d bary (backward) are left unwritten -- for a caller that reads the valid  */
                             /* prefix only (the blend and the rasterizer backward with the counts; ABI 19) */

int pr_project_fwd(const PRProjectArgs* args, void* stream);
/* MeshRasterizer.forward's projection (eval.py:165-168: world -> view -> NDC with view z, face
   gather) fused with pr_rast_fwd: one face pass instead of pr_project_fwd + the rasterizer's
   face preparation.  pa->face_verts receives the projected corners and must equal
   ra->face_verts.  Non-null ra->grad_face_verts / pa->grad_verts are zeroed here, for a
   pr_rast_bwd / pr_project_bwd with flags PR_GRAD_PREZEROED. */
int pr_project_rast_fwd(const PRProjectArgs* pa, const PRRastArgs* ra, void* stream);
int pr_project_bwd(const PRProjectArgs* args, void* stream);

/* Pose of the pose-optimisation loop (experiments/eval.py:343-346; PyTorch3D 0.4.0
 * so3_exponential_map and Rotate(R).transform_points):
 *   R[n] = I + sin(t)/t hat(w) + (1-cos t)/t^2 hat(w)^2,  t = sqrt(max(|w|^2, eps))
 *   out[n,p] = points[n,p] @ R[n or 0]                   (row-vector convention)   */
typedef struct PRSO3Args {
  int32_t N;
  float eps;
  const float* log_rot;        /* (N,3) */
  float* R;                    /* fwd out (N,3,3) */
  const float* grad_R;         /* bwd in (N,3,3) */
  float* grad_log_rot;         /* bwd out (N,3) */
} PRSO3Args;

typedef struct PRRotateArgs {
  int32_t N, P;                /* point batches x points per batch */
  int32_t R_batched;           /* 1: R is (N,3,3); 0: one (3,3) shared by every batch */
  const float* points;         /* (N,P,3) */
  const float* R;
  float* out;                  /* fwd out (N,P,3) */
  const float* grad_out;       /* bwd in (N,P,3) */
  float* grad_points;          /* bwd out (N,P,3), nullable */
  float* grad_R;               /* bwd out, R's shape, nullable (deterministic block reduction) */
} PRRotateArgs;

int pr_so3_exp_fwd(const PRSO3Args* args, void* stream);
int pr_so3_exp_bwd(const PRSO3Args* args, void* stream);
int pr_rotate_fwd(const PRRotateArgs* args, void* stream);
int pr_rotate_bwd(const PRRotateArgs* args, void* stream);

/* One optimize_pose iteration's bookkeeping after loss.backward() and before optimizer.step()
 * (experiments/eval.py:356-358, 372-379, 382-385), as one single-thread kernel for a captured
 * graph (ABI 19).  With t = *it:
 *   losses[t] = *loss; if (*loss < *best_loss) { *best_loss = *loss; best = log_rot }
 *   gnorms[t] = |grad|; if (|grad| > 1000) grad = 1e-5 * N(0, 1) (Philox keyed by *seed and t)
 *   acc[i] += *leaf_grad[i]  (the smoothing leaves' gradients accumulate across iterations, as
 *                             their .grad does in eval.py; i < 3, null leaves skipped)
 *   post: v[i] = 0.9 v[i] + 0.1 acc[i]; acc[i] = 0
 *   adam: optimizer.step() of torch.optim.Adam([log_rot], lr) (eval.py:380; betas 0.9 / 0.999,
 *         eps 1e-8, torch's fused-Adam arithmetic): *step += 1; m = b1 m + (1-b1) g;
 *         s = b2 s + (1-b2) g g; log_rot -= (lr / (1 - b1^step)) m / (sqrt(s) / sqrt(1 - b2^step) + eps)
 *   *it = t + 1                                                       (t < niter checked)   */
typedef struct PRPoseStepArgs {
  const float* loss;           /* 0-d */
  float* log_rot;              /* [n] (the Adam step updates it) */
  float* grad;                 /* [n] log_rot's gradient (the guard rewrites it) */
  int64_t* it;                 /* iteration counter */
  float* losses;               /* [niter] */
  float* gnorms;               /* [niter] */
  float* best_loss;            /* 0-d */
  float* best;                 /* [n] */
  float* v;                    /* [3] EMA of the smoothing gradients (post) */
  float* acc;                  /* [3] the smoothing gradients accumulated since the last EMA */
  const float* leaf_grad[3];   /* this iteration's sigma / gamma / alpha gradients, nullable */
  const uint64_t* seed;        /* guard noise key, nullable (then key 0) */
  float* exp_avg;              /* [n] Adam state (adam) */
  float* exp_avg_sq;           /* [n] */
  float* step;                 /* 0-d float step count */
  const float* lr;             /* 0-d learning rate */
  int64_t niter;
  int32_t n;                   /* log_rot's numel (<= 64) */
  int32_t post;                /* eval.py's adapt_reg and i > 100 */
  int32_t adam;                /* 1: also take the Adam step */
} PRPoseStepArgs;

int pr_pose_step(const PRPoseStepArgs* args, void* stream);

/* eval.py's image loss ((images[..., :3] - target) ** 2).mean() (experiments/eval.py:352-353) as
 * two kernels forward (per-workgroup partial sums, one fixed-order finalize) and one backward
 * (ABI 19): image (P, C >= 3) with P = N*H*W pixels, target (P or P / N, 3) (one target frame
 * broadcast over the batch when target_batched == 0).
 *   fwd: *loss = sum_{p, c < 3} (image[p, c] - target[p, c])^2 / (3 P)
 *   bwd: grad_image[p, c] = (*grad_loss / (3 P)) * (2 (image[p, c] - target[p, c])), 0 for c >= 3 */
typedef struct PRRgbMseArgs {
  int64_t P;                   /* pixels */
  int32_t C;                   /* image channels (>= 3) */
  int32_t HW;                  /* pixels per frame (target broadcast) */
  int32_t target_batched;
  const float* image;          /* (P, C) */
  const float* target;         /* (P, 3) or (HW, 3) */
  float* loss;                 /* fwd out, 0-d */
  float* partials;             /* fwd workspace: pr_rgb_mse_workspace floats */
  const float* grad_loss;      /* bwd in, 0-d */
  float* grad_image;           /* bwd out (P, C) */
} PRRgbMseArgs;

size_t pr_rgb_mse_workspace(int64_t P);  /* floats */
int pr_rgb_mse_fwd(const PRRgbMseArgs* args, void* stream);
int pr_rgb_mse_bwd(const PRRgbMseArgs* args, void* stream);

int pr_abi_version(void);
const char* pr_last_error(void);

/* Live per-kernel timing (measurement only; no reference counterpart).  pr_ktimer_arm(slot) makes
 * the next hot-path call of this thread record a pair of HIP events on its launch stream right
 * before and right after its dominant kernel (blend_fwd_kernel, blend_bwd_kernel, rast_fwd_kernel,
 * rast_bwd_kernel); pr_ktimer_read(slot, ...) returns that kernel's duration in ms and its name
 * after the stream has drained.  0 <= slot < 256 (-1 disarms); events are created on the current device.
 * Not armed: no events are recorded (graph capture never sees them). */
int pr_ktimer_arm(int32_t slot);
int pr_ktimer_read(int32_t slot, float* ms, char* name, int32_t name_cap);

int pr_blend_fwd(const PRBlendFwdArgs* args, void* stream);
size_t pr_blend_plan_size(const PRBlendParams* p); /* bytes of PRBlendFwdArgs.plan */
size_t pr_blend_bwd_workspace_size(const PRBlendBwdArgs* args);
int pr_blend_bwd(const PRBlendBwdArgs* args, void* stream);

int pr_heaviside_fwd(const PRHeavisideArgs* args, void* stream);
size_t pr_heaviside_bwd_workspace_size(const PRHeavisideArgs* args);
int pr_heaviside_bwd(const PRHeavisideArgs* args, void* stream);

size_t pr_rast_fwd_workspace_size(const PRRastArgs* args);
int pr_rast_fwd(const PRRastArgs* args, void* stream);
size_t pr_rast_bwd_workspace_size(const PRRastArgs* args);
int pr_rast_bwd(const PRRastArgs* args, void* stream);

int pr_interp_fwd(const PRInterpArgs* args, void* stream);
int pr_interp_bwd(const PRInterpArgs* args, void* stream);

/* seeds[i] <- splitmix64(seeds[i]) for i < n, on the stream (capturable). */
int pr_seed_advance(uint64_t* seeds, int32_t n, void* stream);

/* The kernels' own noise generator on explicit counters (diagnostic / known-answer entry):
 * block i = Philox4x32-R(counters[4i..4i+3], key = keys[i] (lo word, hi word)), R = rounds: 10
 * (Random123's known-answer vectors) or PR_PHILOX_STREAM_ROUNDS (the streams' generator; ABI 20).
 * words (n,4) u32 receives the raw block; normals (n,4) f32 its Box-Muller N(0,1) samples
 * (pr_common.h gauss4), cauchy (n,4) f32 its clamped Cauchy samples (cauchy4).  Each output
 * is nullable.  With R = PR_PHILOX_STREAM_ROUNDS this is exactly the per-(pixel, slot,
 * sample-group) draw of PR_NOISE_PHILOX. */
int pr_philox(const uint32_t* counters, const uint64_t* keys, int64_t n, uint32_t* words, float* normals,
              float* cauchy, int32_t rounds, void* stream);
#define PR_PHILOX_STREAM_ROUNDS 7 /* rounds of the PR_NOISE_PHILOX streams (pr_philox's rounds: 10 or this) */

#ifdef __cplusplus
}
#endif
#endif /* PERTRENDER_H_ */
