"""Store-bandwidth probe: torch fill_ of 39 / 78 / 156 MB float32 buffers (rocprofv3 gives the kernel times)."""
import torch
d = torch.device("cuda")
for mb in (39, 78, 156):
    x = torch.empty(mb * 1000 * 1000 // 4, device=d)
    for _ in range(20):
        x.fill_(1.5)
    torch.cuda.synchronize()
    print(mb, "MB ok")
