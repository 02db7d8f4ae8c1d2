"""Pure-write HBM bandwidth on this GPU (torch fill_ / zero_ of a buffer the size of the SMOTE
output, 8M rows x 64 B), the ceiling to compare smote_generate's write stream against."""
import torch

dev = torch.device("cuda", 0)
for mb in (510, 2048):
    n = mb * (1 << 20) // 4
    t = torch.empty(n, dtype=torch.float32, device=dev)
    for fn, name in ((lambda: t.fill_(1.0), "fill"), (lambda: t.zero_(), "zero")):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name} {mb} MB: {us:.1f} us, {mb * (1 << 20) / us / 1e6:.2f} TB/s", flush=True)
