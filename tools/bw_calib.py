#!/usr/bin/env python3
"""HBM calibration on this box: device-to-device copy and fill of 4 GiB (torch/hip runtime
kernels), to read our kernels' GB/s against what the box actually sustains."""
import torch

n = 1 << 32
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
a.fill_(1)
torch.cuda.synchronize()
for name, fn, nbytes in (("copy", lambda: b.copy_(a), 2 * n), ("fill", lambda: b.fill_(3), n)):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    print(f"{name}: median {ts[5]:.3f} ms  {nbytes / ts[5] / 1e6:.0f} GB/s  (best {nbytes / ts[0] / 1e6:.0f})")
