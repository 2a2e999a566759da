// C++ autograd layer over the C ABI (include/pertrender.h) for the eager step.
//
// The eager pose-optimisation step (experiments/eval.py:343-376) runs one autograd node per native
// op: so3_exponential_map, Rotate.transform_points, MeshRasterizer (projection + rasterizer), the
// fused perturbed blend (random_rasterizer.py:34-56 with smoothrast.py:12-59 + smoothagg.py:10-73)
// and the smoothing-scalar gradient link.  As Python autograd.Functions each costs ctypes packing
// plus Function.apply (~10-50 us of host time per call); here the nodes are
// torch::autograd::Function subclasses whose forward and backward fill the ABI argument structs
// and launch through the library's own entry points -- the same kernels, arguments and results
// as the Python Functions (pertrenderer_amd/blend.py, renderer/rasterizer.py, renderer/transforms.py),
// which stay the path for HIP-graph capture instrumentation (KernelTimer) and for builds without
// this extension.
//
// The library is not linked: Python hands over the addresses of the entry points of the
// libpertrender.so it loaded (bind()), so both layers drive the one library instance.
#include <torch/extension.h>
#include <torch/csrc/autograd/functions/basic_ops.h>
#include <torch/csrc/autograd/functions/utils.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "pertrender.h"

namespace {

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;
using Opt = c10::optional<Tensor>;

Tensor val(const Opt& t) { return t.has_value() ? *t : Tensor(); }

struct Api {
  decltype(&pr_abi_version) abi_version = nullptr;
  decltype(&pr_last_error) last_error = nullptr;
  decltype(&pr_so3_exp_fwd) so3_exp_fwd = nullptr;
  decltype(&pr_so3_exp_bwd) so3_exp_bwd = nullptr;
  decltype(&pr_rotate_fwd) rotate_fwd = nullptr;
  decltype(&pr_rotate_bwd) rotate_bwd = nullptr;
  decltype(&pr_project_rast_fwd) project_rast_fwd = nullptr;
  decltype(&pr_project_bwd) project_bwd = nullptr;
  decltype(&pr_rast_fwd_workspace_size) rast_fwd_workspace_size = nullptr;
  decltype(&pr_rast_bwd_workspace_size) rast_bwd_workspace_size = nullptr;
  decltype(&pr_rast_bwd) rast_bwd = nullptr;
  decltype(&pr_blend_fwd) blend_fwd = nullptr;
  decltype(&pr_blend_plan_size) blend_plan_size = nullptr;
  decltype(&pr_blend_bwd_workspace_size) blend_bwd_workspace_size = nullptr;
  decltype(&pr_blend_bwd) blend_bwd = nullptr;
  decltype(&pr_shade_fwd) shade_fwd = nullptr;
  decltype(&pr_shade_bwd_workspace_size) shade_bwd_workspace_size = nullptr;
  decltype(&pr_shade_bwd) shade_bwd = nullptr;
  decltype(&pr_vert_normals_fwd) vert_normals_fwd = nullptr;
  decltype(&pr_vert_normals_bwd) vert_normals_bwd = nullptr;
  decltype(&pr_rgb_mse_workspace) rgb_mse_workspace = nullptr;
  decltype(&pr_rgb_mse_fwd) rgb_mse_fwd = nullptr;
  decltype(&pr_rgb_mse_bwd) rgb_mse_bwd = nullptr;
};
Api g_api;
bool g_bound = false;

template <class F>
void bind_one(const std::unordered_map<std::string, int64_t>& addrs, const char* name, F& fn) {
  auto it = addrs.find(name);
  if (it == addrs.end() || it->second == 0) throw std::runtime_error(std::string("pr_torch: missing entry ") + name);
  fn = reinterpret_cast<F>(static_cast<intptr_t>(it->second));
}

void bind(const std::unordered_map<std::string, int64_t>& addrs) {
  Api a;
  bind_one(addrs, "pr_abi_version", a.abi_version);
  bind_one(addrs, "pr_last_error", a.last_error);
  bind_one(addrs, "pr_so3_exp_fwd", a.so3_exp_fwd);
  bind_one(addrs, "pr_so3_exp_bwd", a.so3_exp_bwd);
  bind_one(addrs, "pr_rotate_fwd", a.rotate_fwd);
  bind_one(addrs, "pr_rotate_bwd", a.rotate_bwd);
  bind_one(addrs, "pr_project_rast_fwd", a.project_rast_fwd);
  bind_one(addrs, "pr_project_bwd", a.project_bwd);
  bind_one(addrs, "pr_rast_fwd_workspace_size", a.rast_fwd_workspace_size);
  bind_one(addrs, "pr_rast_bwd_workspace_size", a.rast_bwd_workspace_size);
  bind_one(addrs, "pr_rast_bwd", a.rast_bwd);
  bind_one(addrs, "pr_blend_fwd", a.blend_fwd);
  bind_one(addrs, "pr_blend_plan_size", a.blend_plan_size);
  bind_one(addrs, "pr_blend_bwd_workspace_size", a.blend_bwd_workspace_size);
  bind_one(addrs, "pr_blend_bwd", a.blend_bwd);
  bind_one(addrs, "pr_shade_fwd", a.shade_fwd);
  bind_one(addrs, "pr_shade_bwd_workspace_size", a.shade_bwd_workspace_size);
  bind_one(addrs, "pr_shade_bwd", a.shade_bwd);
  bind_one(addrs, "pr_vert_normals_fwd", a.vert_normals_fwd);
  bind_one(addrs, "pr_vert_normals_bwd", a.vert_normals_bwd);
  bind_one(addrs, "pr_rgb_mse_workspace", a.rgb_mse_workspace);
  bind_one(addrs, "pr_rgb_mse_fwd", a.rgb_mse_fwd);
  bind_one(addrs, "pr_rgb_mse_bwd", a.rgb_mse_bwd);
  if (a.abi_version() != PR_ABI_VERSION)
    throw std::runtime_error("pr_torch: built for ABI " + std::to_string(PR_ABI_VERSION) + ", library has " +
                             std::to_string(a.abi_version()));
  g_api = a;
  g_bound = true;
}

const Api& api() {
  if (!g_bound) throw std::runtime_error("pr_torch: bind() was not called");
  return g_api;
}

void check(int code, const char* what) {
  if (code != 0)
    throw std::runtime_error(std::string(what) + " failed (" + std::to_string(code) + "): " + api().last_error());
}

void* stream_of(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

template <class T>
T* ptr(const Tensor& t) {
  return t.defined() ? static_cast<T*>(t.data_ptr()) : nullptr;
}

// nat.dense: `t` as a contiguous tensor of dtype st (the tensor itself when it already is one)
Tensor dense(const Tensor& t, at::ScalarType st) {
  if (!t.defined()) return t;
  if (t.scalar_type() == st && t.is_contiguous()) return t;
  return t.to(st).contiguous();
}

// nat.require_device: a host pointer handed to a kernel would fault the GPU
void on_device(std::initializer_list<const Tensor*> ts) {
  for (const Tensor* t : ts)
    if (t->defined() && !t->is_cuda())
      throw std::invalid_argument("pertrenderer_amd native ops run on ROCm devices only (got a " +
                                  t->device().str() + " tensor); there is no CPU fallback");
}

Tensor empty(at::IntArrayRef shape, at::ScalarType st, const Tensor& like) {
  return at::empty(shape, like.options().dtype(st));
}

Tensor workspace(size_t bytes, const Tensor& like) {
  return at::empty({static_cast<int64_t>(bytes > 0 ? bytes : 1)}, like.options().dtype(at::kByte));
}

// Tensors a node keeps for its backward go through save_for_backward -- released when the
// backward has run (CppNode::release_variables), version-checked against in-place changes, and a
// second backward without retain_graph raises -- while saved_data holds only each one's index.
struct Keep {
  AutogradContext* ctx;
  std::vector<Tensor> ts;
  explicit Keep(AutogradContext* c) : ctx(c) {}
  void operator()(const char* key, const Tensor& t) {
    ctx->saved_data[key] = static_cast<int64_t>(ts.size());
    ts.push_back(t);  // (undefined tensors are allowed)
  }
  void commit() { ctx->save_for_backward(ts); }
};

struct Saved {
  AutogradContext* ctx;
  variable_list v;
  explicit Saved(AutogradContext* c) : ctx(c), v(c->get_saved_variables()) {}
  Tensor operator()(const char* key) const {
    auto it = ctx->saved_data.find(key);
    if (it == ctx->saved_data.end() || !it->second.isInt()) return Tensor();
    return v.at(static_cast<size_t>(it->second.toInt()));
  }
};

// torch.autograd.function.once_differentiable: with create_graph the returned gradients carry a
// node that refuses a second differentiation instead of silently being constants
variable_list once(const variable_list& grads_in, variable_list out) {
  if (!at::GradMode::is_enabled()) return out;
  bool any = false;
  for (const auto& g : grads_in) any = any || (g.defined() && g.requires_grad());
  if (!any) return out;
  variable_list fake;
  fake.reserve(out.size());
  for (auto& t : out) {
    if (t.defined()) {
      auto d = t.detach();
      d.set_requires_grad(true);
      fake.push_back(d);
    } else {
      fake.push_back(t);
    }
  }
  auto err = std::make_shared<torch::autograd::DelayedError>(
      "trying to differentiate twice a function that was marked with @once_differentiable",
      static_cast<int64_t>(fake.size()));
  return (*err)(std::move(fake));
}

// ------------------------------------------------------------------ smoothing-scalar link
// blend.py's _ScalarLink: the reference's smoothing scalars are CPU 0-d leaves, so every backward
// brings their gradients to the host.  The blend's backward records an event after the kernels
// that write its (3,) gradient buffer; the link's backward (reached after the rasterizer's backward
// is launched: it was created before the rasterizer) waits for that event only, on a side stream.
// Pending entries are keyed by the buffer's address and hold a weak reference to the tensor that
// was marked: a lookup whose tensor is not that one (a freed gradient's address reused, e.g. by a
// summed gradient when the link output feeds two consumers) takes the synchronous copy instead of
// waiting on a stale event.
using WeakImpl = c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>;
struct Pending {
  int dev;
  hipEvent_t event;
  WeakImpl impl;
};
struct Ready {
  std::mutex mu;
  std::unordered_map<const void*, Pending> pending;  // buffer -> (device, event, tensor)
  std::unordered_map<int, std::vector<hipEvent_t>> free;
  std::unordered_map<int, std::pair<hipStream_t, float*>> side;  // device -> side stream, pinned (4,)
};
Ready& ready() {
  static Ready* r = new Ready();  // never destroyed: HIP may be torn down first at exit
  return *r;
}

void mark_ready(const Tensor& buf, void* stream) {
  auto& r = ready();
  const int dev = buf.device().index();
  hipEvent_t e = nullptr;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    auto& fl = r.free[dev];
    if (!fl.empty()) {
      e = fl.back();
      fl.pop_back();
    }
  }
  if (e == nullptr && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
    throw std::runtime_error("pr_torch: hipEventCreateWithFlags failed");
  if (hipEventRecord(e, static_cast<hipStream_t>(stream)) != hipSuccess)
    throw std::runtime_error("pr_torch: hipEventRecord failed");
  std::lock_guard<std::mutex> lk(r.mu);
  // links whose backward never ran (grad taken w.r.t. other inputs) leave entries whose tensor is
  // gone: recycle those (and an entry at this address)
  for (auto it = r.pending.begin(); it != r.pending.end();) {
    if (it->first == buf.data_ptr() || it->second.impl.expired()) {
      r.free[it->second.dev].push_back(it->second.event);
      it = r.pending.erase(it);
    } else {
      ++it;
    }
  }
  r.pending.emplace(buf.data_ptr(), Pending{dev, e, WeakImpl(buf.getIntrusivePtr())});
}

// g (3,) float on the device -> CPU (3,) float, waiting only for the event recorded for g
Tensor host_copy(const Tensor& g) {
  auto& r = ready();
  const int dev = g.device().index();
  hipEvent_t e = nullptr;
  hipStream_t side = nullptr;
  float* pinned = nullptr;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.pending.find(g.data_ptr());
    if (it != r.pending.end()) {
      auto live = it->second.impl.lock();
      if (live.get() == g.unsafeGetTensorImpl()) {
        e = it->second.event;
      } else {  // another tensor at a recycled address: its writer is unknown, copy synchronously
        r.free[it->second.dev].push_back(it->second.event);
      }
      r.pending.erase(it);
    }
    auto s = r.side.find(dev);
    if (s != r.side.end()) {
      side = s->second.first;
      pinned = s->second.second;
    }
  }
  auto gc = g.contiguous();
  if (e == nullptr || gc.scalar_type() != at::kFloat || gc.numel() != 3) return gc.to(at::kCPU);
  if (side == nullptr) {
    if (hipStreamCreateWithFlags(&side, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&pinned), 4 * sizeof(float), hipHostMallocDefault) != hipSuccess)
      throw std::runtime_error("pr_torch: side stream / pinned buffer");
    std::lock_guard<std::mutex> lk(r.mu);
    r.side[dev] = {side, pinned};
  }
  if (hipStreamWaitEvent(side, e, 0) != hipSuccess ||
      hipMemcpyAsync(pinned, gc.data_ptr(), 3 * sizeof(float), hipMemcpyDeviceToHost, side) != hipSuccess ||
      hipStreamSynchronize(side) != hipSuccess)
    throw std::runtime_error("pr_torch: scalar gradient copy failed");
  {
    std::lock_guard<std::mutex> lk(r.mu);
    r.free[dev].push_back(e);
  }
  auto out = at::empty({3}, at::TensorOptions().dtype(at::kFloat));
  std::memcpy(out.data_ptr(), pinned, 3 * sizeof(float));
  return out;
}

struct ScalarMeta {
  bool defined = false;
  at::ScalarType dtype = at::kFloat;
  std::vector<int64_t> shape;
};

ScalarMeta meta_of(const Tensor& t) {
  ScalarMeta m;
  if (t.defined() && t.requires_grad()) {
    m.defined = true;
    m.dtype = t.scalar_type();
    m.shape = t.sizes().vec();
  }
  return m;
}

// The link is a raw autograd Node with sequence number 0: the engine runs ready nodes in
// decreasing sequence order, so once the rasterizer's backward is launched it takes the pose
// backward (Rotate, so3, d log_rot) before the link, and the link's wait for the blend kernels
// overlaps those launches (a Function node made in the renderer would outrank them).
struct ScalarLinkNode : public torch::autograd::Node {
  ScalarMeta meta[3];
  explicit ScalarLinkNode(torch::autograd::edge_list&& next) : Node(/*sequence_nr=*/0, std::move(next)) {}
  std::string name() const override { return "ScalarLinkBackward"; }
  variable_list apply(variable_list&& grads) override {
    variable_list out(3);
    if (grads.empty() || !grads[0].defined()) return out;
    auto host = host_copy(grads[0]);
    for (int i = 0; i < 3; ++i)
      if (meta[i].defined && should_compute_output(i)) out[i] = host[i].to(meta[i].dtype).reshape(meta[i].shape);
    return out;
  }
};

Tensor scalar_link(Opt sigma, Opt gamma, Opt alpha, int64_t device) {
  auto out = at::empty({3}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device));
  const Tensor ts[3] = {val(sigma), val(gamma), val(alpha)};
  bool any = false;
  for (const auto& t : ts) any = any || (t.defined() && t.requires_grad());
  if (!at::GradMode::is_enabled() || !any) return out;
  auto node = std::shared_ptr<ScalarLinkNode>(
      new ScalarLinkNode(torch::autograd::collect_next_edges(ts[0], ts[1], ts[2])), torch::autograd::deleteNode);
  for (int i = 0; i < 3; ++i) node->meta[i] = meta_of(ts[i]);
  torch::autograd::set_history(out, node);
  return out;
}

// ------------------------------------------------------------------ pose: so3 exp, rotate
struct SO3ExpFn : public torch::autograd::Function<SO3ExpFn> {
  static Tensor forward(AutogradContext* ctx, Tensor log_rot, double eps) {
    on_device({&log_rot});
    auto w = dense(log_rot, at::kFloat);
    auto R = empty({w.size(0), 3, 3}, at::kFloat, w);
    PRSO3Args a{};
    a.N = static_cast<int32_t>(w.size(0));
    a.eps = static_cast<float>(eps);
    a.log_rot = ptr<float>(w);
    a.R = ptr<float>(R);
    at::DeviceGuard dg(w.device());
    check(api().so3_exp_fwd(&a, stream_of(w)), "pr_so3_exp_fwd");
    Keep k(ctx);
    k("w", w);
    k.commit();
    ctx->saved_data["eps"] = eps;
    return R;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    if (!grads[0].defined()) return {Tensor(), Tensor()};
    auto w = Saved(ctx)("w");
    auto g = dense(grads[0], at::kFloat);
    auto gw = at::empty_like(w);
    PRSO3Args a{};
    a.N = static_cast<int32_t>(w.size(0));
    a.eps = static_cast<float>(ctx->saved_data["eps"].toDouble());
    a.log_rot = ptr<float>(w);
    a.grad_R = ptr<float>(g);
    a.grad_log_rot = ptr<float>(gw);
    at::DeviceGuard dg(w.device());
    check(api().so3_exp_bwd(&a, stream_of(gw)), "pr_so3_exp_bwd");
    return once(grads, {gw, Tensor()});
  }
};

struct RotateFn : public torch::autograd::Function<RotateFn> {
  static Tensor forward(AutogradContext* ctx, Tensor points, Tensor R) {
    on_device({&points, &R});
    auto p = dense(points, at::kFloat);
    auto r = dense(R, at::kFloat);
    auto out = at::empty_like(p);
    PRRotateArgs a{};
    a.N = static_cast<int32_t>(p.size(0));
    a.P = static_cast<int32_t>(p.size(1));
    a.R_batched = r.size(0) > 1;
    a.points = ptr<float>(p);
    a.R = ptr<float>(r);
    a.out = ptr<float>(out);
    at::DeviceGuard dg(p.device());
    check(api().rotate_fwd(&a, stream_of(out)), "pr_rotate_fwd");
    Keep k(ctx);
    k("p", p);
    k("r", r);
    k.commit();
    return out;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    if (!grads[0].defined()) return {Tensor(), Tensor()};
    const Saved sv(ctx);
    auto p = sv("p"), r = sv("r");
    auto g = dense(grads[0], at::kFloat);
    Tensor gp = ctx->needs_input_grad(0) ? at::empty_like(p) : Tensor();
    Tensor gr = ctx->needs_input_grad(1) ? at::empty_like(r) : Tensor();
    PRRotateArgs a{};
    a.N = static_cast<int32_t>(p.size(0));
    a.P = static_cast<int32_t>(p.size(1));
    a.R_batched = r.size(0) > 1;
    a.points = ptr<float>(p);
    a.R = ptr<float>(r);
    a.grad_out = ptr<float>(g);
    a.grad_points = ptr<float>(gp);
    a.grad_R = ptr<float>(gr);
    at::DeviceGuard dg(p.device());
    check(api().rotate_bwd(&a, stream_of(g)), "pr_rotate_bwd");
    return once(grads, {gp, gr});
  }
};

Tensor so3_exp(const Tensor& log_rot, double eps) { return SO3ExpFn::apply(log_rot, eps); }
Tensor rotate(const Tensor& points, const Tensor& R) { return RotateFn::apply(points, R); }

// ------------------------------------------------------------------ projection + rasterizer
// renderer/rasterizer.py _ProjectRasterizeFn: pr_project_rast_fwd, backward pr_rast_bwd then
// pr_project_bwd into d verts (accumulators zeroed by the forward kernel)
Tensor per_mesh(const Tensor& m, int64_t N, const char* name) {
  // the cameras' cached (N,4,4) float matrices: used as they are (no alias, no copy)
  if (m.scalar_type() == at::kFloat && m.dim() == 3 && m.size(0) == N && m.size(1) == 4 && m.size(2) == 4 &&
      m.is_contiguous())
    return m;
  auto f = m.detach().to(at::kFloat);
  if (f.dim() != 3 || f.size(1) != 4 || f.size(2) != 4 || (f.size(0) != 1 && f.size(0) != N))
    throw std::invalid_argument(std::string(name) + " matrices must be (1,4,4) or (N,4,4)");
  return (f.size(0) != N ? f.expand({N, 4, 4}) : f).contiguous();
}

void rast_common(PRRastArgs& a, const Tensor& fv, const Tensor& first, const Tensor& nfaces,
                 const std::vector<int64_t>& cfg, double blur) {
  a.face_verts = ptr<float>(fv);
  a.mesh_first_face = ptr<int64_t>(first);
  a.mesh_num_faces = ptr<int64_t>(nfaces);
  a.F = fv.size(0);
  a.N = static_cast<int32_t>(first.size(0));
  a.H = static_cast<int32_t>(cfg[0]);
  a.W = static_cast<int32_t>(cfg[1]);
  a.K = static_cast<int32_t>(cfg[2]);
  a.blur_radius = static_cast<float>(blur);
  a.perspective_correct = static_cast<int32_t>(cfg[3]);
  a.clip_barycentric_coords = static_cast<int32_t>(cfg[4]);
  a.cull_backfaces = static_cast<int32_t>(cfg[5]);
  a.bin_size = static_cast<int32_t>(cfg[6]);
  a.max_faces_per_bin = static_cast<int32_t>(cfg[7]);
}

void project_common(PRProjectArgs& pa, const Tensor& v, const Tensor& f, const Tensor& first, const Tensor& nfaces,
                    const Tensor& m1, const Tensor& m2) {
  pa.verts = ptr<float>(v);
  pa.faces = ptr<int64_t>(f);
  pa.mesh_first_face = ptr<int64_t>(first);
  pa.mesh_num_faces = ptr<int64_t>(nfaces);
  pa.world_to_view = ptr<float>(m1);
  pa.proj = ptr<float>(m2);
  pa.V = v.size(0);
  pa.F = f.size(0);
  pa.N = static_cast<int32_t>(first.size(0));
}

struct ProjectRasterizeFn : public torch::autograd::Function<ProjectRasterizeFn> {
  // cfg = (H, W, K, perspective_correct, clip, cull, bin_size, max_faces_per_bin)
  static variable_list forward(AutogradContext* ctx, Tensor verts, Tensor faces, Tensor first, Tensor nfaces,
                               Tensor w2v, Tensor proj, c10::optional<Tensor> csr_start,
                               c10::optional<Tensor> csr_corners, std::vector<int64_t> cfg, double blur,
                               c10::optional<Tensor> blur_dev, bool need, c10::optional<Tensor> seed_adv,
                               int64_t seed_n) {
    if (cfg.size() != 8 && cfg.size() != 9) throw std::invalid_argument("project_rasterize: cfg must have 8 or 9 entries");
    Tensor cs = csr_start.has_value() ? *csr_start : Tensor(), cc = csr_corners.has_value() ? *csr_corners : Tensor();
    on_device({&verts, &faces, &first, &nfaces, &w2v, &proj, &cs, &cc});
    auto v = dense(verts, at::kFloat);
    auto f = dense(faces, at::kLong);
    const int64_t N = first.size(0), F = f.size(0);
    const int64_t H = cfg[0], W = cfg[1], K = cfg[2];
    auto m1 = per_mesh(w2v, N, "world_to_view"), m2 = per_mesh(proj, N, "projection");
    auto fv = empty({F, 3, 3}, at::kFloat, v);
    Tensor gfv = need ? empty({F, 3, 3}, at::kFloat, v) : Tensor();
    Tensor gv = need ? at::empty_like(v) : Tensor();
    PRProjectArgs pa{};
    project_common(pa, v, f, first, nfaces, m1, m2);
    pa.face_verts = ptr<float>(fv);
    pa.grad_verts = ptr<float>(gv);
    const Tensor sa = val(seed_adv);  // the caller's deferred noise-key advances (DeviceSeed)
    if (sa.defined() && seed_n > 0) {
      on_device({&sa});
      pa.seed_advance = static_cast<uint64_t*>(sa.data_ptr());
      pa.seed_advance_n = static_cast<int32_t>(seed_n);
    }
    PRRastArgs a{};
    rast_common(a, fv, first, nfaces, cfg, blur);
    const Tensor bd = val(blur_dev);  // a device blur threshold (graph replays with a changing blur)
    if (bd.defined()) {
      on_device({&bd});
      if (bd.scalar_type() != at::kFloat || bd.numel() != 1)
        throw std::invalid_argument("project_rasterize: a device blur_radius must be one float32");
      a.blur_radius_dev = bd.data_ptr<float>();
    }
    auto p2f = empty({N, H, W, K}, at::kLong, v);
    auto zbuf = empty({N, H, W, K}, at::kFloat, v);
    auto bary = empty({N, H, W, K, 3}, at::kFloat, v);
    auto dists = empty({N, H, W, K}, at::kFloat, v);
    auto counts = empty({N, H, W}, at::kInt, v);
    if (cfg.size() == 9 && cfg[8]) a.flags |= PR_RAST_VALID_ONLY;  // the caller reads the valid prefix only
    a.pix_to_face = ptr<int64_t>(p2f);
    a.zbuf = ptr<float>(zbuf);
    a.bary = ptr<float>(bary);
    a.dists = ptr<float>(dists);
    a.pix_count = ptr<int32_t>(counts);
    a.grad_face_verts = ptr<float>(gfv);
    at::DeviceGuard dg(v.device());
    auto ws = workspace(api().rast_fwd_workspace_size(&a), v);
    a.workspace = ws.data_ptr();
    a.workspace_bytes = static_cast<size_t>(ws.numel());
    check(api().project_rast_fwd(&pa, &a, stream_of(v)), "pr_project_rast_fwd");
    Keep k(ctx);
    k("p2f", p2f);
    k("counts", counts);
    k("v", v);
    k("f", f);
    k("first", first);
    k("nfaces", nfaces);
    k("m1", m1);
    k("m2", m2);
    k("fv", fv);
    k("gfv", gfv);
    k("gv", gv);
    k("csr_start", cs);
    k("csr_corners", cc);
    k.commit();
    ctx->saved_data["cfg"] = cfg;
    ctx->saved_data["blur"] = blur;
    ctx->saved_data["prezeroed"] = true;
    ctx->mark_non_differentiable({p2f, counts});
    ctx->set_materialize_grads(false);
    return {p2f, zbuf, bary, dists, counts};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    variable_list out(14);  // one per forward argument
    const Saved sv(ctx);
    auto gfv = sv("gfv"), gv = sv("gv");
    if (!gfv.defined()) return out;
    auto p2f = sv("p2f"), counts = sv("counts");
    auto v = sv("v"), f = sv("f"), first = sv("first"), nfaces = sv("nfaces");
    auto m1 = sv("m1"), m2 = sv("m2"), fv = sv("fv");
    auto cfg = ctx->saved_data["cfg"].toIntVector();
    // a second backward (retain_graph) finds the accumulators used: zero them again
    const int32_t flags = ctx->saved_data["prezeroed"].toBool() ? PR_GRAD_PREZEROED : 0;
    ctx->saved_data["prezeroed"] = false;
    PRRastArgs a{};
    rast_common(a, fv, first, nfaces, cfg, ctx->saved_data["blur"].toDouble());
    a.pix_to_face = ptr<int64_t>(p2f);
    a.pix_count = ptr<int32_t>(counts);
    a.flags = flags;
    auto gz = dense(grads[1], at::kFloat), gb = dense(grads[2], at::kFloat), gd = dense(grads[3], at::kFloat);
    a.grad_zbuf = ptr<float>(gz);
    a.grad_bary = ptr<float>(gb);
    a.grad_dists = ptr<float>(gd);
    a.grad_face_verts = ptr<float>(gfv);
    at::DeviceGuard dg(v.device());
    Tensor ws;
    if (at::globalContext().deterministicAlgorithms()) {  // nat.deterministic(): slot-order face sums
      a.flags |= PR_DETERMINISTIC;
      ws = workspace(api().rast_bwd_workspace_size(&a), v);
      a.workspace = ws.data_ptr();
      a.workspace_bytes = static_cast<size_t>(ws.numel());
    }
    void* st = stream_of(v);
    check(api().rast_bwd(&a, st), "pr_rast_bwd");
    ws = Tensor();
    PRProjectArgs pa{};
    project_common(pa, v, f, first, nfaces, m1, m2);
    pa.grad_face_verts = ptr<float>(gfv);
    pa.grad_verts = ptr<float>(gv);
    pa.flags = flags;
    auto cs = sv("csr_start"), cc = sv("csr_corners");
    pa.vert_corner_start = ptr<int64_t>(cs);
    pa.vert_corners = ptr<int64_t>(cc);
    check(api().project_bwd(&pa, st), "pr_project_bwd");
    out[0] = gv;
    return once(grads, out);
  }
};

variable_list project_rasterize(const Tensor& verts, const Tensor& faces, const Tensor& first, const Tensor& nfaces,
                                const Tensor& w2v, const Tensor& proj, c10::optional<Tensor> csr_start,
                                c10::optional<Tensor> csr_corners, std::vector<int64_t> cfg, double blur,
                                c10::optional<Tensor> blur_dev, c10::optional<Tensor> seed_adv, int64_t seed_n) {
  // the forward's gradient accumulators are sized when d verts will be wanted (Python's
  // ctx.needs_input_grad[0]; the C++ context has no edges to ask before the node is executable)
  const bool need = at::GradMode::is_enabled() && verts.requires_grad();
  return ProjectRasterizeFn::apply(verts, faces, first, nfaces, w2v, proj, csr_start, csr_corners, cfg, blur,
                                   blur_dev, need, seed_adv, seed_n);
}

// ------------------------------------------------------------------ fused perturbed blend
// blend.py _FusedBlendFn (texel colours) / _FusedVertexBlendFn (vertex colours, vertex = true).
// The parameter block (PRBlendParams: shape, samples, noise keys, by-value / device scalars,
// planes) is packed by the Python caller and read here by address; every tensor it points to is an
// argument of this call and is kept for the backward.
constexpr int kIn = 20;  // forward arguments

struct BlendFn : public torch::autograd::Function<BlendFn> {
  // differentiable: 0 dists, 1 zbuf, 2 colours (texel) / bary (vertex), 3 vertex colours,
  // 4 sigma, 5 gamma, 6 alpha (device or CPU 0-d leaves, undefined when passed by value), 7 link
  // Absent optional arguments are no autograd inputs at all (an undefined tensor cannot be one), so
  // the edges do not line up with the argument positions: the gradient mask is taken here, from
  // requires_grad at the call (the meaning of Python's ctx.needs_input_grad)
  static Tensor forward(AutogradContext* ctx, Tensor dists, Tensor zbuf, Tensor colors, Opt vert_colors_o,
                        Opt sigma_o, Opt gamma_o, Opt alpha_o, Opt link_o, Tensor p2f, Opt faces_o, Opt counts_o,
                        Tensor znear, Tensor zfar, Opt noise_r_o, Opt noise_a_o, Opt seeds_o, int64_t params,
                        bool cache_on, bool sync_on, bool grad_on) {
    const Tensor vert_colors = val(vert_colors_o), sigma = val(sigma_o), gamma = val(gamma_o), alpha = val(alpha_o);
    const Tensor link = val(link_o), faces = val(faces_o), counts = val(counts_o);
    const Tensor noise_r = val(noise_r_o), noise_a = val(noise_a_o), seeds = val(seeds_o);
    on_device({&dists, &zbuf, &colors, &vert_colors, &p2f, &faces, &counts, &znear, &zfar, &noise_r, &noise_a, &seeds});
    const Tensor diff[8] = {dists, zbuf, colors, vert_colors, sigma, gamma, alpha, link};
    int64_t need = 0;
    for (int i = 0; i < 8; ++i)
      need |= (grad_on && diff[i].defined() && diff[i].requires_grad()) ? (int64_t{1} << i) : 0;
    ctx->saved_data["need"] = need;
    PRBlendParams p;
    std::memcpy(&p, reinterpret_cast<const void*>(static_cast<intptr_t>(params)), sizeof(p));
    const bool vertex = (p.flags & PR_BLEND_VERTEX) != 0, soft = (p.flags & PR_BLEND_SOFT) != 0;
    const int64_t N = p.N, H = p.H, W = p.W, K = p.K;
    auto p2f_c = dense(p2f, at::kLong);
    auto d_c = dense(dists, at::kFloat), z_c = dense(zbuf, at::kFloat), c_c = dense(colors, at::kFloat);
    auto v_c = vertex ? dense(vert_colors, at::kFloat) : Tensor();
    auto f_c = vertex ? dense(faces, at::kLong) : Tensor();
    auto image = empty({N, H, W, 4}, at::kFloat, p2f_c);
    auto winners = empty({N * H * W, p.Sa}, at::kByte, p2f_c);
    const bool any_grad = need != 0;
    Tensor cache = cache_on && !soft && any_grad ? empty({N, H, W, K, 2}, at::kFloat, p2f_c) : Tensor();
    PRBlendFwdArgs a{};
    a.p = p;
    a.pix_to_face = ptr<int64_t>(p2f_c);
    a.dists = ptr<float>(d_c);
    a.zbuf = ptr<float>(z_c);
    if (vertex) {
      a.bary = ptr<float>(c_c);
      a.faces = ptr<int64_t>(f_c);
      a.vert_colors = ptr<float>(v_c);
    } else {
      a.colors = ptr<float>(c_c);
    }
    a.image = ptr<float>(image);
    a.winners = ptr<uint8_t>(winners);
    a.rast_cache = ptr<float>(cache);
    a.pix_count = ptr<int32_t>(counts);
    at::DeviceGuard dg(p2f_c.device());
    Tensor plan, sync;
    if (!soft && counts.defined()) {
      const size_t n = api().blend_plan_size(&p);
      if (n) plan = at::empty({static_cast<int64_t>((n + 3) / 4)}, p2f_c.options().dtype(at::kInt));
    }
    if (!soft && sync_on) sync = at::empty({PR_BLEND_SYNC_BYTES / 4}, p2f_c.options().dtype(at::kInt));
    a.plan = ptr<int32_t>(plan);
    a.sync = ptr<int32_t>(sync);
    check(api().blend_fwd(&a, stream_of(image)), "pr_blend_fwd");
    ctx->saved_data["p"] = std::string(reinterpret_cast<const char*>(&p), sizeof(p));
    const char* names[] = {"p2f", "d", "z", "c", "v", "f", "counts", "zn", "zf", "nr", "na", "seeds",
                           "winners", "cache", "plan", "sync", "s0", "s1", "s2"};
    const Tensor ts[] = {p2f_c, d_c, z_c, c_c, v_c, f_c, counts, znear, zfar, noise_r, noise_a, seeds,
                         winners, cache, plan, sync, sigma, gamma, alpha};
    Keep k(ctx);
    for (size_t i = 0; i < sizeof(ts) / sizeof(ts[0]); ++i) k(names[i], ts[i]);
    k.commit();
    return image;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    variable_list out(kIn);
    const auto pb = ctx->saved_data["p"].toStringRef();
    PRBlendParams p;
    std::memcpy(&p, pb.data(), sizeof(p));
    if (p.flags & PR_BLEND_AGG_UNIFORM)
      throw std::runtime_error("UniformAgg: the reference implements no gradient for uniform noise "
                               "(smoothagg.py:64-70)");
    if (!grads[0].defined()) return out;
    const bool vertex = (p.flags & PR_BLEND_VERTEX) != 0;
    const int64_t need = ctx->saved_data["need"].toInt();
    auto needs = [need](int i) { return ((need >> i) & 1) != 0; };
    const Saved sv(ctx);
    auto p2f = sv("p2f"), d = sv("d"), z = sv("z"), c = sv("c");
    auto v = sv("v"), f = sv("f");
    auto g = dense(grads[0], at::kFloat);
    auto gd = at::empty_like(d), gz = at::empty_like(z), gc = at::empty_like(c);
    Tensor gv = vertex && needs(3) ? at::zeros_like(v) : Tensor();
    auto gsc = at::empty({3}, d.options());
    PRBlendBwdArgs a{};
    a.p = p;
    a.pix_to_face = ptr<int64_t>(p2f);
    a.dists = ptr<float>(d);
    a.zbuf = ptr<float>(z);
    if (vertex) {
      a.bary = ptr<float>(c);
      a.faces = ptr<int64_t>(f);
      a.vert_colors = ptr<float>(v);
      a.grad_bary = ptr<float>(gc);
      a.grad_vert_colors = ptr<float>(gv);
    } else {
      a.colors = ptr<float>(c);
      a.grad_colors = ptr<float>(gc);
    }
    a.winners = ptr<uint8_t>(sv("winners"));
    a.grad_image = ptr<float>(g);
    a.rast_cache = ptr<float>(sv("cache"));
    a.grad_dists = ptr<float>(gd);
    a.grad_zbuf = ptr<float>(gz);
    a.grad_scalars = ptr<float>(gsc);
    a.pix_count = ptr<int32_t>(sv("counts"));
    a.plan = ptr<int32_t>(sv("plan"));
    a.sync = ptr<int32_t>(sv("sync"));
    at::DeviceGuard dg(d.device());
    auto ws = workspace(api().blend_bwd_workspace_size(&a), d);
    a.workspace = ws.data_ptr();
    a.workspace_bytes = static_cast<size_t>(ws.numel());
    void* st = stream_of(g);
    check(api().blend_bwd(&a, st), "pr_blend_bwd");
    if (needs(0)) out[0] = gd;
    if (needs(1)) out[1] = gz;
    if (needs(2)) out[2] = gc;
    out[3] = gv;
    // the smoothing scalars (blend.py _scalar_grads): CPU leaves get their three values in ONE copy
    Tensor host;
    for (int i = 0; i < 3; ++i) {
      auto ref = sv(i == 0 ? "s0" : i == 1 ? "s1" : "s2");
      if (!needs(4 + i) || !ref.defined()) continue;
      if (ref.device().is_cpu()) {
        if (!host.defined()) host = gsc.to(at::kCPU);
        out[4 + i] = host[i].to(ref.scalar_type()).reshape(ref.sizes());
      } else {
        out[4 + i] = gsc[i].to(ref.scalar_type()).reshape(ref.sizes());
      }
    }
    if (needs(7)) {  // the link's gradient, marked with the event after its kernels
      mark_ready(gsc, st);
      out[7] = gsc;
    }
    return once(grads, out);
  }
};

Tensor blend(const Tensor& dists, const Tensor& zbuf, const Tensor& colors, Opt vert_colors, Opt sigma, Opt gamma,
             Opt alpha, Opt link, const Tensor& p2f, Opt faces, Opt counts, const Tensor& znear, const Tensor& zfar,
             Opt noise_r, Opt noise_a, Opt seeds, int64_t params, bool cache_on, bool sync_on) {
  return BlendFn::apply(dists, zbuf, colors, vert_colors, sigma, gamma, alpha, link, p2f, faces, counts, znear, zfar,
                        noise_r, noise_a, seeds, params, cache_on, sync_on, at::GradMode::is_enabled());
}

// ------------------------------------------------------------------ Phong shading, vertex normals
// renderer/shading.py _ShadeFn (pr_shade_fwd / pr_shade_bwd) and renderer/mesh.py _VertNormalsFn
// (pr_vert_normals_fwd / pr_vert_normals_bwd): eval.py's RandomPhongShader path
void shade_common(PRShadeArgs& a, const Tensor& p2f, const Tensor& counts, const Tensor& faces, const Tensor& face_uvs,
                  const Tensor* t /* bary verts normals tex light camera */, const Tensor* rows, int64_t mode,
                  bool directional) {
  a.N = static_cast<int32_t>(p2f.size(0));
  a.H = static_cast<int32_t>(p2f.size(1));
  a.W = static_cast<int32_t>(p2f.size(2));
  a.K = static_cast<int32_t>(p2f.size(3));
  a.pix_to_face = ptr<int64_t>(p2f);
  a.pix_count = ptr<int32_t>(counts);
  a.faces = ptr<int64_t>(faces);
  a.bary = ptr<float>(t[0]);
  a.verts = ptr<float>(t[1]);
  a.normals = ptr<float>(t[2]);
  a.V = t[1].size(0);
  a.F = faces.size(0);
  a.texture = static_cast<int32_t>(mode);
  if (mode == PR_TEX_GIVEN) {
    a.texels = ptr<float>(t[3]);
  } else if (mode == PR_TEX_VERTEX) {
    a.vert_colors = ptr<float>(t[3]);
  } else {
    a.maps = ptr<float>(t[3]);
    a.face_uvs = ptr<float>(face_uvs);
    a.Hm = static_cast<int32_t>(t[3].size(1));
    a.Wm = static_cast<int32_t>(t[3].size(2));
  }
  a.directional = directional ? 1 : 0;
  a.light = ptr<float>(t[4]);
  a.camera = ptr<float>(t[5]);
  a.ambient = ptr<float>(rows[0]);
  a.diffuse_color = ptr<float>(rows[1]);
  a.specular_color = ptr<float>(rows[2]);
  a.mat_diffuse = ptr<float>(rows[3]);
  a.mat_specular = ptr<float>(rows[4]);
  a.shininess = ptr<float>(rows[5]);
}

const char* kShadeKeys[6] = {"bary", "verts", "normals", "tex", "light", "camera"};
const char* kShadeRows[6] = {"ambient", "diffuse_color", "specular_color", "mat_diffuse", "mat_specular", "shininess"};

// the small gradient accumulators (d verts, d normals, d vertex colours, d light, d camera) that
// pr_shade_fwd zeroes for a PR_GRAD_PREZEROED backward: inputs 1, 2, 3 (vertex colours), 4, 5
bool prezeroable(int i, int64_t mode) { return i == 1 || i == 2 || i == 4 || i == 5 || (i == 3 && mode == PR_TEX_VERTEX); }

struct ShadeFn : public torch::autograd::Function<ShadeFn> {
  // pz: bit i set = input i will want a gradient (sized and zeroed by the forward's kernel)
  static Tensor forward(AutogradContext* ctx, Tensor bary, Tensor verts, Tensor normals, Tensor tex, Tensor light,
                        Tensor camera, Tensor p2f, Opt counts_o, Tensor faces, Opt face_uvs_o, std::vector<Tensor> rows,
                        int64_t mode, bool directional, bool live_only, int64_t pz) {
    const Tensor counts = val(counts_o), face_uvs = val(face_uvs_o);
    if (rows.size() != 6) throw std::invalid_argument("shade: 6 parameter rows expected");
    on_device({&bary, &verts, &normals, &tex, &light, &camera, &p2f, &counts, &faces, &face_uvs});
    for (const auto& r : rows) on_device({&r});
    Tensor t[6] = {dense(bary, at::kFloat), dense(verts, at::kFloat), dense(normals, at::kFloat),
                   dense(tex, at::kFloat),  dense(light, at::kFloat), dense(camera, at::kFloat)};
    auto p2f_c = dense(p2f, at::kLong);
    auto colors = at::empty({p2f_c.size(0), p2f_c.size(1), p2f_c.size(2), p2f_c.size(3), 3},
                            t[0].options().dtype(at::kFloat));
    PRShadeArgs a{};
    shade_common(a, p2f_c, counts, faces, face_uvs, t, rows.data(), mode, directional);
    a.colors = ptr<float>(colors);
    if (live_only && counts.defined()) a.flags |= PR_SHADE_LIVE_ONLY;
    Tensor acc[6];
    for (int i = 1; i < 6; ++i)
      if ((pz >> i) & 1 && prezeroable(i, mode)) acc[i] = at::empty_like(t[i]);
    a.grad_verts = ptr<float>(acc[1]);
    a.grad_normals = ptr<float>(acc[2]);
    a.grad_vert_colors = ptr<float>(acc[3]);
    a.grad_light = ptr<float>(acc[4]);
    a.grad_camera = ptr<float>(acc[5]);
    at::DeviceGuard dg(colors.device());
    check(api().shade_fwd(&a, stream_of(colors)), "pr_shade_fwd");
    Keep k(ctx);
    for (int i = 0; i < 6; ++i) k(kShadeKeys[i], t[i]);
    const char* kAcc[6] = {"", "acc1", "acc2", "acc3", "acc4", "acc5"};
    for (int i = 1; i < 6; ++i) k(kAcc[i], acc[i]);
    ctx->saved_data["prezeroed"] = true;
    for (int i = 0; i < 6; ++i) k(kShadeRows[i], rows[i]);
    k("p2f", p2f_c);
    k("counts", counts);
    k("faces", faces);
    k("face_uvs", face_uvs);
    k.commit();
    ctx->saved_data["mode"] = mode;
    ctx->saved_data["directional"] = directional;
    ctx->saved_data["live_only"] = live_only && counts.defined();
    return colors;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    variable_list out(15);  // one per forward argument
    if (!grads[0].defined()) return out;
    const Saved sv(ctx);
    Tensor t[6], rows[6];
    for (int i = 0; i < 6; ++i) t[i] = sv(kShadeKeys[i]);
    for (int i = 0; i < 6; ++i) rows[i] = sv(kShadeRows[i]);
    const int64_t mode = ctx->saved_data["mode"].toInt();
    auto g = dense(grads[0], at::kFloat);
    PRShadeArgs a{};
    shade_common(a, sv("p2f"), sv("counts"), sv("faces"), sv("face_uvs"), t, rows,
                 mode, ctx->saved_data["directional"].toBool());
    a.grad_colors = ptr<float>(g);
    // the forward's zeroed accumulators, once: a second backward (retain_graph) sizes and zeroes
    // its own; an accumulator the forward did not size sends the whole call down the zeroing path
    const char* kAcc[6] = {"", "acc1", "acc2", "acc3", "acc4", "acc5"};
    bool pre = ctx->saved_data["prezeroed"].toBool();
    ctx->saved_data["prezeroed"] = false;
    for (int i = 0; i < 6; ++i) {
      if (!ctx->needs_input_grad(i)) continue;
      const Tensor z = i > 0 && pre ? sv(kAcc[i]) : Tensor();
      out[i] = z.defined() ? z : at::empty_like(t[i]);
      if (i > 0 && prezeroable(i, mode) && !z.defined()) pre = false;
    }
    a.grad_bary = ptr<float>(out[0]);
    a.grad_verts = ptr<float>(out[1]);
    a.grad_normals = ptr<float>(out[2]);
    if (mode == PR_TEX_GIVEN) a.grad_texels = ptr<float>(out[3]);
    else if (mode == PR_TEX_VERTEX) a.grad_vert_colors = ptr<float>(out[3]);
    else a.grad_maps = ptr<float>(out[3]);
    a.grad_light = ptr<float>(out[4]);
    a.grad_camera = ptr<float>(out[5]);
    at::DeviceGuard dg(g.device());
    Tensor ws;
    if (at::globalContext().deterministicAlgorithms()) {  // in-order sums, no float atomics
      a.flags = PR_DETERMINISTIC;  // (overwrites its outputs: the pre-zeroing is moot)
      ws = workspace(api().shade_bwd_workspace_size(&a), g);
      a.workspace = ws.data_ptr();
      a.workspace_bytes = static_cast<size_t>(ws.numel());
    }
    if (pre && !(a.flags & PR_DETERMINISTIC)) a.flags |= PR_GRAD_PREZEROED;
    if (ctx->saved_data["live_only"].toBool()) a.flags |= PR_SHADE_LIVE_ONLY;
    check(api().shade_bwd(&a, stream_of(g)), "pr_shade_bwd");
    return once(grads, out);
  }
};

Tensor shade(const Tensor& bary, const Tensor& verts, const Tensor& normals, const Tensor& tex, const Tensor& light,
             const Tensor& camera, const Tensor& p2f, Opt counts, const Tensor& faces, Opt face_uvs,
             std::vector<Tensor> rows, int64_t mode, bool directional, bool live_only) {
  // which inputs will want a gradient (as project_rasterize: the C++ context cannot ask yet)
  int64_t pz = 0;
  if (at::GradMode::is_enabled()) {
    const Tensor* in[6] = {&bary, &verts, &normals, &tex, &light, &camera};
    for (int i = 0; i < 6; ++i) pz |= in[i]->requires_grad() ? (int64_t(1) << i) : 0;
  }
  return ShadeFn::apply(bary, verts, normals, tex, light, camera, p2f, counts, faces, face_uvs, rows, mode,
                        directional, live_only, pz);
}

// ------------------------------------------------------------------ fused Phong blend
// blend.py _FusedPhongBlendFn: RandomPhongShader's sample_textures -> phong_shading ->
// smooth_rgb_blend (random_rasterizer.py:99-116).  Forward: one pr_blend_fwd (PR_BLEND_PHONG) that
// shades a slot only where it wins a sample and keeps the colours of the slots the backward reads
// (winners, unperturbed argmax) in a sparse colour buffer.  Backward: pr_blend_bwd reading those
// (PR_BLEND_COLOR_SPARSE) -> d colours -> pr_shade_bwd, whose chain rule runs for the slots with a
// non-zero d colour only.  Gradients: dists, zbuf, bary (-> rasterizer), verts, normals (-> vertex
// normals), the UV maps or vertex colours, light, camera and the smoothing scalars.
constexpr int kPhongIn = 28;  // forward arguments

struct BlendPhongFn : public torch::autograd::Function<BlendPhongFn> {
  // differentiable: 0 dists, 1 zbuf, 2 bary, 3 verts, 4 normals, 5 tex, 6 light, 7 camera,
  // 8 sigma, 9 gamma, 10 alpha, 11 link
  static Tensor forward(AutogradContext* ctx, Tensor dists, Tensor zbuf, Tensor bary, Tensor verts, Tensor normals,
                        Tensor tex, Tensor light, Tensor camera, Opt sigma_o, Opt gamma_o, Opt alpha_o, Opt link_o,
                        Tensor p2f, Tensor faces, Opt counts_o, Opt face_uvs_o, std::vector<Tensor> rows,
                        Tensor znear, Tensor zfar, Opt noise_r_o, Opt noise_a_o, Opt seeds_o, int64_t params,
                        int64_t mode, bool directional, bool cache_on, bool sync_on, bool grad_on) {
    const Tensor sigma = val(sigma_o), gamma = val(gamma_o), alpha = val(alpha_o), link = val(link_o);
    const Tensor counts = val(counts_o), face_uvs = val(face_uvs_o);
    const Tensor noise_r = val(noise_r_o), noise_a = val(noise_a_o), seeds = val(seeds_o);
    if (rows.size() != 6) throw std::invalid_argument("blend_phong: 6 parameter rows expected");
    on_device({&dists, &zbuf, &bary, &verts, &normals, &tex, &light, &camera, &p2f, &faces, &counts, &face_uvs,
               &znear, &zfar, &noise_r, &noise_a, &seeds});
    for (const auto& r : rows) on_device({&r});
    const Tensor diff[12] = {dists, zbuf, bary, verts, normals, tex, light, camera, sigma, gamma, alpha, link};
    int64_t need = 0;
    for (int i = 0; i < 12; ++i)
      need |= (grad_on && diff[i].defined() && diff[i].requires_grad()) ? (int64_t{1} << i) : 0;
    ctx->saved_data["need"] = need;
    PRBlendParams p;
    std::memcpy(&p, reinterpret_cast<const void*>(static_cast<intptr_t>(params)), sizeof(p));
    const int64_t N = p.N, H = p.H, W = p.W, K = p.K;
    auto p2f_c = dense(p2f, at::kLong), f_c = dense(faces, at::kLong);
    auto d_c = dense(dists, at::kFloat), z_c = dense(zbuf, at::kFloat);
    Tensor t[6] = {dense(bary, at::kFloat),  dense(verts, at::kFloat), dense(normals, at::kFloat),
                   dense(tex, at::kFloat),   dense(light, at::kFloat), dense(camera, at::kFloat)};
    auto image = empty({N, H, W, 4}, at::kFloat, p2f_c);
    auto winners = empty({N * H * W, p.Sa}, at::kByte, p2f_c);
    const bool any_grad = need != 0;
    Tensor cache = cache_on && any_grad ? empty({N, H, W, K, 2}, at::kFloat, p2f_c) : Tensor();
    // the colours the backward reads (written at those slots only: no other slot is touched)
    Tensor colors = any_grad ? empty({N, H, W, K, 3}, at::kFloat, p2f_c) : Tensor();
    PRShadeArgs sh{};
    shade_common(sh, p2f_c, counts, f_c, face_uvs, t, rows.data(), mode, directional);
    // the shading backward's small accumulators, zeroed by the forward's kernel
    Tensor acc[6];
    for (int i = 1; i < 6; ++i)
      if (((need >> (2 + i)) & 1) && prezeroable(i, mode)) acc[i] = at::empty_like(t[i]);
    sh.grad_verts = ptr<float>(acc[1]);
    sh.grad_normals = ptr<float>(acc[2]);
    sh.grad_vert_colors = ptr<float>(acc[3]);
    sh.grad_light = ptr<float>(acc[4]);
    sh.grad_camera = ptr<float>(acc[5]);
    PRBlendFwdArgs a{};
    a.p = p;
    a.pix_to_face = ptr<int64_t>(p2f_c);
    a.dists = ptr<float>(d_c);
    a.zbuf = ptr<float>(z_c);
    a.bary = ptr<float>(t[0]);
    a.colors = ptr<float>(colors);
    a.image = ptr<float>(image);
    a.winners = ptr<uint8_t>(winners);
    a.rast_cache = ptr<float>(cache);
    a.pix_count = ptr<int32_t>(counts);
    a.shade = &sh;
    at::DeviceGuard dg(p2f_c.device());
    Tensor sync = sync_on ? at::empty({PR_BLEND_SYNC_BYTES / 4}, p2f_c.options().dtype(at::kInt)) : Tensor();
    a.sync = ptr<int32_t>(sync);
    check(api().blend_fwd(&a, stream_of(image)), "pr_blend_fwd (phong)");
    ctx->saved_data["p"] = std::string(reinterpret_cast<const char*>(&p), sizeof(p));
    ctx->saved_data["mode"] = mode;
    ctx->saved_data["directional"] = directional;
    ctx->saved_data["prezeroed"] = true;
    Keep k(ctx);
    for (int i = 0; i < 6; ++i) k(kShadeKeys[i], t[i]);
    for (int i = 0; i < 6; ++i) k(kShadeRows[i], rows[i]);
    const char* kAcc[6] = {"", "acc1", "acc2", "acc3", "acc4", "acc5"};
    for (int i = 1; i < 6; ++i) k(kAcc[i], acc[i]);
    const char* names[] = {"p2f", "d", "z", "f", "counts", "face_uvs", "zn", "zf", "nr", "na", "seeds",
                           "winners", "cache", "sync", "colors", "s0", "s1", "s2"};
    const Tensor ts[] = {p2f_c, d_c, z_c, f_c, counts, face_uvs, znear, zfar, noise_r, noise_a, seeds,
                         winners, cache, sync, colors, sigma, gamma, alpha};
    for (size_t i = 0; i < sizeof(ts) / sizeof(ts[0]); ++i) k(names[i], ts[i]);
    k.commit();
    return image;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    variable_list out(kPhongIn);
    const auto pb = ctx->saved_data["p"].toStringRef();
    PRBlendParams p;
    std::memcpy(&p, pb.data(), sizeof(p));
    if (p.flags & PR_BLEND_AGG_UNIFORM)
      throw std::runtime_error("UniformAgg: the reference implements no gradient for uniform noise "
                               "(smoothagg.py:64-70)");
    if (!grads[0].defined()) return out;
    const int64_t need = ctx->saved_data["need"].toInt();
    auto needs = [need](int i) { return ((need >> i) & 1) != 0; };
    const int64_t mode = ctx->saved_data["mode"].toInt();
    const Saved sv(ctx);
    Tensor t[6], rows[6];
    for (int i = 0; i < 6; ++i) t[i] = sv(kShadeKeys[i]);
    for (int i = 0; i < 6; ++i) rows[i] = sv(kShadeRows[i]);
    auto p2f = sv("p2f"), d = sv("d"), z = sv("z"), colors = sv("colors");
    auto g = dense(grads[0], at::kFloat);
    // 1. the blend backward on the sparse colours: d dists, d zbuf, d colours, the scalars
    p.flags = (p.flags & ~PR_BLEND_PHONG) | PR_BLEND_COLOR_SPARSE;
    auto gd = at::empty_like(d), gz = at::empty_like(z), gc = at::empty_like(colors);
    auto gsc = at::empty({3}, d.options());
    PRBlendBwdArgs a{};
    a.p = p;
    a.pix_to_face = ptr<int64_t>(p2f);
    a.dists = ptr<float>(d);
    a.zbuf = ptr<float>(z);
    a.colors = ptr<float>(colors);
    a.grad_colors = ptr<float>(gc);
    a.winners = ptr<uint8_t>(sv("winners"));
    a.grad_image = ptr<float>(g);
    a.rast_cache = ptr<float>(sv("cache"));
    a.grad_dists = ptr<float>(gd);
    a.grad_zbuf = ptr<float>(gz);
    a.grad_scalars = ptr<float>(gsc);
    a.pix_count = ptr<int32_t>(sv("counts"));
    a.sync = ptr<int32_t>(sv("sync"));
    at::DeviceGuard dg(d.device());
    auto ws = workspace(api().blend_bwd_workspace_size(&a), d);
    a.workspace = ws.data_ptr();
    a.workspace_bytes = static_cast<size_t>(ws.numel());
    void* st = stream_of(g);
    check(api().blend_bwd(&a, st), "pr_blend_bwd (phong)");
    // 2. the shading backward: d bary and the mesh / texture / light / camera gradients
    PRShadeArgs sh{};
    shade_common(sh, p2f, sv("counts"), sv("f"), sv("face_uvs"), t, rows, mode,
                 ctx->saved_data["directional"].toBool());
    sh.grad_colors = ptr<float>(gc);
    const char* kAcc[6] = {"", "acc1", "acc2", "acc3", "acc4", "acc5"};
    bool pre = ctx->saved_data["prezeroed"].toBool();
    ctx->saved_data["prezeroed"] = false;
    Tensor sg[6];
    for (int i = 0; i < 6; ++i) {
      if (!needs(2 + i)) continue;
      const Tensor zt = i > 0 && pre ? sv(kAcc[i]) : Tensor();
      sg[i] = zt.defined() ? zt : at::empty_like(t[i]);
      if (i > 0 && prezeroable(i, mode) && !zt.defined()) pre = false;
    }
    sh.grad_bary = ptr<float>(sg[0]);
    sh.grad_verts = ptr<float>(sg[1]);
    sh.grad_normals = ptr<float>(sg[2]);
    if (mode == PR_TEX_VERTEX) sh.grad_vert_colors = ptr<float>(sg[3]);
    else sh.grad_maps = ptr<float>(sg[3]);
    sh.grad_light = ptr<float>(sg[4]);
    sh.grad_camera = ptr<float>(sg[5]);
    Tensor sws;
    if (at::globalContext().deterministicAlgorithms()) {  // in-order sums, no float atomics
      sh.flags = PR_DETERMINISTIC;
      sws = workspace(api().shade_bwd_workspace_size(&sh), g);
      sh.workspace = sws.data_ptr();
      sh.workspace_bytes = static_cast<size_t>(sws.numel());
    }
    if (pre && !(sh.flags & PR_DETERMINISTIC)) sh.flags |= PR_GRAD_PREZEROED;
    if ((p.flags & PR_BLEND_LIVE_ONLY) && sh.pix_count) sh.flags |= PR_SHADE_LIVE_ONLY;
    if (needs(2) || needs(3) || needs(4) || needs(5) || needs(6) || needs(7))
      check(api().shade_bwd(&sh, st), "pr_shade_bwd (phong)");
    if (needs(0)) out[0] = gd;
    if (needs(1)) out[1] = gz;
    for (int i = 0; i < 6; ++i) out[2 + i] = sg[i];
    Tensor host;
    for (int i = 0; i < 3; ++i) {
      auto ref = sv(i == 0 ? "s0" : i == 1 ? "s1" : "s2");
      if (!needs(8 + i) || !ref.defined()) continue;
      if (ref.device().is_cpu()) {
        if (!host.defined()) host = gsc.to(at::kCPU);
        out[8 + i] = host[i].to(ref.scalar_type()).reshape(ref.sizes());
      } else {
        out[8 + i] = gsc[i].to(ref.scalar_type()).reshape(ref.sizes());
      }
    }
    if (needs(11)) {
      mark_ready(gsc, st);
      out[11] = gsc;
    }
    return once(grads, out);
  }
};

Tensor blend_phong(const Tensor& dists, const Tensor& zbuf, const Tensor& bary, const Tensor& verts,
                   const Tensor& normals, const Tensor& tex, const Tensor& light, const Tensor& camera, Opt sigma,
                   Opt gamma, Opt alpha, Opt link, const Tensor& p2f, const Tensor& faces, Opt counts, Opt face_uvs,
                   std::vector<Tensor> rows, const Tensor& znear, const Tensor& zfar, Opt noise_r, Opt noise_a,
                   Opt seeds, int64_t params, int64_t mode, bool directional, bool cache_on, bool sync_on) {
  return BlendPhongFn::apply(dists, zbuf, bary, verts, normals, tex, light, camera, sigma, gamma, alpha, link, p2f,
                             faces, counts, face_uvs, rows, znear, zfar, noise_r, noise_a, seeds, params, mode,
                             directional, cache_on, sync_on, at::GradMode::is_enabled());
}

struct VertNormalsFn : public torch::autograd::Function<VertNormalsFn> {
  static Tensor forward(AutogradContext* ctx, Tensor verts, Tensor faces, Opt csr_start_o, Opt csr_corners_o) {
    const Tensor cs = val(csr_start_o), cc = val(csr_corners_o);
    on_device({&verts, &faces, &cs, &cc});
    auto v = verts.contiguous();
    auto f = dense(faces, at::kLong);
    auto n = at::empty_like(v), raw = at::empty_like(v);
    PRNormalsArgs a{};
    a.verts = ptr<float>(v);
    a.faces = ptr<int64_t>(f);
    a.V = v.size(0);
    a.F = f.size(0);
    a.normals = ptr<float>(n);
    a.raw = ptr<float>(raw);
    a.vert_corner_start = ptr<int64_t>(cs);
    a.vert_corners = ptr<int64_t>(cc);
    at::DeviceGuard dg(v.device());
    check(api().vert_normals_fwd(&a, stream_of(v)), "pr_vert_normals_fwd");
    Keep k(ctx);
    k("v", v);
    k("f", f);
    k("raw", raw);
    k("cs", cs);
    k("cc", cc);
    k.commit();
    return n;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    variable_list out(4);
    if (!grads[0].defined()) return out;
    const Saved sv(ctx);
    auto v = sv("v"), f = sv("f"), raw = sv("raw");
    auto cs = sv("cs"), cc = sv("cc");
    auto g = dense(grads[0], at::kFloat);
    auto graw = at::empty_like(v), gv = at::empty_like(v);
    PRNormalsArgs a{};
    a.verts = ptr<float>(v);
    a.faces = ptr<int64_t>(f);
    a.V = v.size(0);
    a.F = f.size(0);
    a.raw = ptr<float>(raw);
    a.grad_normals = ptr<float>(g);
    a.grad_raw = ptr<float>(graw);
    a.grad_verts = ptr<float>(gv);
    a.vert_corner_start = ptr<int64_t>(cs);
    a.vert_corners = ptr<int64_t>(cc);
    at::DeviceGuard dg(g.device());
    check(api().vert_normals_bwd(&a, stream_of(g)), "pr_vert_normals_bwd");
    out[0] = gv;
    return once(grads, out);
  }
};

Tensor vert_normals(const Tensor& verts, const Tensor& faces, Opt csr_start, Opt csr_corners) {
  return VertNormalsFn::apply(verts, faces, csr_start, csr_corners);
}

// ------------------------------------------------------------------ RGB loss
// pose_opt._RgbMse: eval.py:352-353's ((images[..., :3] - target) ** 2).mean() on pr_rgb_mse_fwd /
// _bwd (fixed-order sums), the caller's loss of the bench / pose step
PRRgbMseArgs rgb_mse_args(const Tensor& img, const Tensor& t) {
  if (img.dim() != 4 || img.scalar_type() != at::kFloat || t.scalar_type() != at::kFloat || img.size(3) < 3 ||
      t.size(-1) != 3)
    throw std::invalid_argument("rgb_mse: float32 (N,H,W,C>=3) images and (..,H,W,3) target expected");
  const int64_t N = img.size(0), H = img.size(1), W = img.size(2);
  if (t.numel() != H * W * 3 && t.numel() != N * H * W * 3)
    throw std::invalid_argument("rgb_mse: target does not broadcast to the images");
  PRRgbMseArgs a{};
  a.P = N * H * W;
  a.C = static_cast<int32_t>(img.size(3));
  a.HW = static_cast<int32_t>(H * W);
  a.target_batched = (t.numel() == N * H * W * 3 && N > 1) ? 1 : 0;
  a.image = ptr<float>(img);
  a.target = ptr<float>(t);
  return a;
}

struct RgbMseFn : public torch::autograd::Function<RgbMseFn> {
  static Tensor forward(AutogradContext* ctx, Tensor images, Tensor target) {
    on_device({&images, &target});
    auto img = images.contiguous(), t = target.contiguous();
    PRRgbMseArgs a = rgb_mse_args(img, t);
    auto loss = at::empty({}, img.options());
    auto part = at::empty({static_cast<int64_t>(api().rgb_mse_workspace(a.P))}, img.options());
    a.loss = ptr<float>(loss);
    a.partials = ptr<float>(part);
    at::DeviceGuard dg(img.device());
    check(api().rgb_mse_fwd(&a, stream_of(img)), "pr_rgb_mse_fwd");
    Keep k(ctx);
    k("img", img);
    k("t", t);
    k.commit();
    return loss;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    variable_list out(2);
    if (!grads[0].defined()) return out;
    const Saved sv(ctx);
    auto img = sv("img"), t = sv("t");
    PRRgbMseArgs a = rgb_mse_args(img, t);
    auto gl = dense(grads[0], at::kFloat);
    auto gi = at::empty_like(img);
    a.grad_loss = ptr<float>(gl);
    a.grad_image = ptr<float>(gi);
    at::DeviceGuard dg(img.device());
    check(api().rgb_mse_bwd(&a, stream_of(gi)), "pr_rgb_mse_bwd");
    out[0] = gi;
    return once(grads, out);
  }
};

Tensor rgb_mse(const Tensor& images, const Tensor& target) { return RgbMseFn::apply(images, target); }

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "C++ autograd layer over libpertrender's C ABI (eager step host path)";
  m.attr("ABI_VERSION") = PR_ABI_VERSION;
  m.attr("PARAMS_BYTES") = static_cast<int64_t>(sizeof(PRBlendParams));
  m.def("bind", &bind, "entry-point addresses {name: address} of the loaded libpertrender");
  m.def("so3_exp", &so3_exp);
  m.def("rotate", &rotate);
  m.def("project_rasterize", &project_rasterize);
  m.def("blend", &blend);
  m.def("scalar_link", &scalar_link);
  m.def("shade", &shade);
  m.def("blend_phong", &blend_phong);
  m.def("rgb_mse", &rgb_mse);
  m.def("vert_normals", &vert_normals);
}
