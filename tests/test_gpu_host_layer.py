"""The C++ autograd layer (host_layer.py, csrc/pr_torch.cpp) against the Python autograd Functions
it replaces in the eager step: the same kernels with the same arguments, so the same results.

The bench step (pose -> rasterizer -> fused vertex-colour blend -> L2 loss -> backward) in
deterministic mode (the rasterizer / projection backwards then sum in a fixed order) is bitwise
equal through both layers: image, loss, d log_rot and the CPU smoothing-scalar gradients that come
back through the C++ link.  The texel-colour and SoftRas blends are compared on their own."""
import pytest
import torch

import pertrenderer_amd as pa
from pertrenderer_amd import host_layer

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _cpp_layer():
    assert host_layer.layer() == "c++", host_layer.error()


def _step(device, size=96, K=30, seed=3, eval_scene=False):
    import bench
    torch.manual_seed(seed)
    wl = bench.Workload(device, image_size=size, K=K, samples=8, eval_scene=eval_scene,
                        rast_samples=16 if eval_scene else None)
    torch.manual_seed(seed + 1)  # the Philox keys of the blend
    loss = wl.forward()
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), wl.log_rot.grad.clone(), [p.grad.clone() for p in wl.params()[1:]]


@pytest.mark.parametrize("size,K,eval_scene", [(96, 30, False), (256, 50, False), (128, 50, True)])
def test_eager_step_matches_python_layer(device, size, K, eval_scene):
    """eval_scene: eval.py's renderer (RandomPhongShader over the TexturesUV cube: the C++ shading
    and vertex-normal nodes too)."""
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        a = _step(device, size, K, eval_scene=eval_scene)
        with host_layer.disabled():
            b = _step(device, size, K, eval_scene=eval_scene)
    finally:
        torch.use_deterministic_algorithms(False)
    assert torch.equal(a[0], b[0]), "loss"
    assert torch.equal(a[1], b[1]), "d log_rot"
    for x, y, n in zip(a[2], b[2], ("sigma", "gamma", "alpha")):
        assert x.device.type == "cpu" and y.device.type == "cpu", n
        assert torch.equal(x, y), n
    assert a[1].abs().sum() > 0


def _frags(device, size=64, K=20):
    import bench
    wl = bench.Workload(device, image_size=size, K=K, samples=8)
    frag = wl.renderer.rasterizer(wl.base, cameras=wl.cameras)
    return wl, frag


@pytest.mark.parametrize("soft", [False, True])
def test_texel_blend_matches_python_layer(device, soft):
    wl, frag = _frags(device)
    cols = torch.rand(frag.pix_to_face.shape + (3,), device=device, generator=torch.Generator(device).manual_seed(0))
    g = torch.randn(frag.pix_to_face.shape[:3] + (4,), device=device, generator=torch.Generator(device).manual_seed(1))

    def run():
        d = frag.dists.detach().requires_grad_(True)
        z = frag.zbuf.detach().requires_grad_(True)
        c = cols.clone().requires_grad_(True)
        s, gm, al = (torch.tensor(v, requires_grad=True) for v in (1e-3, 1e-2, 1.0))
        torch.manual_seed(7)
        if soft:
            img = pa.soft_blend(c, frag.pix_to_face, d, z, s, gm, al, background=(0.1, 0.2, 0.3))
        else:
            img = pa.perturbed_blend(c, frag.pix_to_face, d, z, s, gm, al, 8, 8, background=(0.1, 0.2, 0.3))
        (img * g).sum().backward()
        return [img.detach(), d.grad, z.grad, c.grad, s.grad, gm.grad, al.grad]

    a = run()
    with host_layer.disabled():
        b = run()
    for x, y, n in zip(a, b, ("image", "dists", "zbuf", "colors", "sigma", "gamma", "alpha")):
        assert torch.equal(x, y), n


def test_device_scalars_and_retain_graph(device):
    """Device smoothing leaves (graph mode's) through the C++ blend: gradients stay on the device;
    a second backward of the same graph reproduces the first (the rasterizer's accumulators are
    zeroed again)."""
    wl, _ = _frags(device)
    wl.device_scalars()
    torch.use_deterministic_algorithms(True)
    try:
        torch.manual_seed(2)
        loss = wl.forward()
        loss.backward(retain_graph=True)
        first = [wl.log_rot.grad.clone()] + [p.grad.clone() for p in wl.params()[1:]]
        wl.zero_grad()
        loss.backward()
        second = [wl.log_rot.grad.clone()] + [p.grad.clone() for p in wl.params()[1:]]
    finally:
        torch.use_deterministic_algorithms(False)
    for x, y in zip(first, second):
        assert x.is_cuda and torch.equal(x, y)


def test_graph_capture_through_cpp_layer(device):
    """bench.py's captured step records the C++ nodes' launches (device smoothing leaves, DeviceSeed
    keys): a replay runs the whole step and moves the pose."""
    import bench
    wl = bench.Workload(device, image_size=64, K=20, samples=8)
    try:
        step = bench.build_step(wl, 1, "graph", device, 1.0)
        before = wl.log_rot.detach().clone()
        step()
        torch.cuda.synchronize()
    finally:
        pa.noise.use_device_seed(None)  # build_step routes Philox draws through its DeviceSeed
    assert not torch.equal(before, wl.log_rot.detach())
    assert torch.isfinite(wl.log_rot).all()


def test_layer_is_used_in_eager_step(device):
    """The eager step's graph holds the C++ nodes (no Python Function of this package)."""
    import bench
    wl = bench.Workload(device, image_size=64, K=20, samples=8)
    loss = wl.forward()
    names, stack, seen, held = [], [loss.grad_fn], set(), []
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        held.append(fn)  # the node wrappers are made per access: hold them so ids stay unique
        seen.add(id(fn))
        names.append(type(fn).__name__ if not hasattr(fn, "name") else fn.name())
        stack.extend(f for f, _ in fn.next_functions)
    assert not any(n.startswith("_") and n.endswith("Backward") for n in names), names
    assert any("BlendFn" in n for n in names), names
    assert any("ProjectRasterizeFn" in n for n in names), names


@pytest.mark.parametrize("deterministic", [False, True])
def test_eval_scene_uses_cpp_shading_and_normals(device, deterministic):
    """eval.py's renderer in the C++ layer: the fused Phong blend node (BlendPhongFn) and the vertex
    normals, in deterministic mode too (its shading backward then sums in order)."""
    import bench
    wl = bench.Workload(device, image_size=64, K=20, samples=8, eval_scene=True, rast_samples=16)
    torch.use_deterministic_algorithms(deterministic, warn_only=True)
    try:
        loss = wl.forward()
    finally:
        torch.use_deterministic_algorithms(False)
    names, stack, seen, held = [], [loss.grad_fn], set(), []
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        held.append(fn)
        seen.add(id(fn))
        names.append(fn.name())
        stack.extend(f for f, _ in fn.next_functions)
    shading = "BlendPhongFn"
    assert any(shading in n for n in names) and any("VertNormalsFn" in n for n in names), names
    assert not any(n.startswith("_") and n.endswith("Backward") for n in names), names
