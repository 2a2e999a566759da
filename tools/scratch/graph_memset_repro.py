"""Scratch: graph replays after an eager matmul -- memset node vs torch global reduce, and whether
a matmul before the captures (BLAS initialised) avoids the corruption."""
import sys, ctypes, torch
case, pre = sys.argv[1], sys.argv[2] == "pre"
dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
torch.manual_seed(0)
if pre:
    _ = torch.randn(3, device=dev) @ torch.randn(3, device=dev)
    torch.cuda.synchronize()
x = torch.randn(1, 256, 256, 4, device=dev)
t = torch.randn(1, 256, 256, 3, device=dev)
buf = torch.ones(64, device=dev)
rec = torch.zeros(1000, device=dev)
it = torch.zeros((), dtype=torch.int64, device=dev)
w = torch.ones((), device=dev)

def body():
    if case == "memset":
        s = torch.cuda.current_stream().cuda_stream
        assert hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, ctypes.c_size_t(256), ctypes.c_void_p(s)) == 0
        buf.add_(1.0)
        v = buf.sum()
    else:
        v = ((x[..., :3] * w - t) ** 2).mean()
    rec.index_copy_(0, it.view(1), v.view(1))
    w.add_(0.01)
    it.add_(1)

def capture():
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
        body()
    return g

g0 = capture()
for _ in range(5): g0.replay()
g1 = capture()
for _ in range(5): g1.replay()
torch.cuda.synchronize()
_ = torch.randn(3, device=dev) @ torch.randn(3, device=dev)
torch.cuda.synchronize()
for _ in range(5): g0.replay()
torch.cuda.synchronize()
r = rec[:15].tolist()
if case == "memset":
    exp = [64.0] * 15
else:
    exp = [float(((x[..., :3] * (1 + 0.01 * i) - t) ** 2).double().mean()) for i in range(15)]
bad = [i for i in range(15) if abs(r[i] - exp[i]) > 1e-4 * abs(exp[i])]
print(case, "pre" if pre else "nopre", "bad iterations:", bad, [round(v, 4) for v in r[9:12]], flush=True)
