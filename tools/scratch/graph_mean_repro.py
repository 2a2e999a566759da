"""Scratch: does a replayed torch.cuda graph keep computing a large mean() correctly after another
graph was captured and eager work ran?  (the cfg5 GraphSession stale-loss symptom)
argv: reduce (mean | twostage)  eager (none | matmul | bigsum | randn)"""
import sys, torch
red, eager = sys.argv[1], sys.argv[2]
dev = torch.device("cuda:0")
torch.manual_seed(0)
x = torch.randn(1, 256, 256, 4, device=dev)
t = torch.randn(1, 256, 256, 3, device=dev)
rec = torch.zeros(1000, device=dev)
it = torch.zeros((), dtype=torch.int64, device=dev)
w = torch.ones((), device=dev)

def loss_of():
    d = (x[..., :3] * w - t) ** 2
    if red == "mean":
        return d.mean()
    return d.reshape(256, -1).sum(1).sum() / d.numel()

def body():
    loss = loss_of()
    rec.index_copy_(0, it.view(1), loss.view(1))
    w.add_(0.01)
    it.add_(1)

def capture():
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        loss_of()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
        body()
    return g

g0 = capture()
for _ in range(5): g0.replay()
g1 = capture()
for _ in range(5): g1.replay()
torch.cuda.synchronize()
if eager == "matmul":
    _ = torch.randn(3, device=dev) @ torch.randn(3, device=dev)
elif eager == "bigsum":
    _ = torch.randn(1 << 20, device=dev).sum()
elif eager == "randn":
    _ = torch.randn(1 << 20, device=dev) * 2
torch.cuda.synchronize()
for _ in range(5): g0.replay()
torch.cuda.synchronize()
r = rec[:15].tolist()
exp = [float(((x[..., :3] * (1 + 0.01 * i) - t) ** 2).double().mean()) for i in range(15)]
bad = [i for i in range(15) if abs(r[i] - exp[i]) > 1e-4 * exp[i]]
print(red, eager, "bad iterations:", bad, [round(v, 4) for v in r[9:12]], [round(v, 4) for v in exp[9:12]], flush=True)
