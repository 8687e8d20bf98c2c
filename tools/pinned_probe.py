#!/usr/bin/env python3
"""Host-side cost of the adaptive path's level chain on page-locked buffers
(diagnostic): np.add / np.log10 / np.multiply over C3's 827 k frame r values
read from / written to torch pin_memory blocks vs ordinary numpy arrays."""
import time
import numpy as np
import torch

n = 826_880
rng = np.random.default_rng(0)
r = (rng.random(n).astype(np.float32) * 0.1 + 1e-4)
pin_in = torch.empty(n, dtype=torch.float32, pin_memory=True)
pin_out = torch.empty(n, dtype=torch.float32, pin_memory=True)
pin_in.numpy()[:] = r
tmp = np.empty(n, np.float32)
out = np.empty(n, np.float32)


def chain(src, dst):
    np.add(src, 1e-12, out=tmp)
    np.log10(tmp, out=tmp)
    np.multiply(tmp, 20.0, out=dst)


for name, src, dst in (("plain -> plain", r, out), ("pinned -> plain", pin_in.numpy(), out),
                       ("plain -> pinned", r, pin_out.numpy()),
                       ("pinned -> pinned", pin_in.numpy(), pin_out.numpy())):
    best = 1e9
    for _ in range(20):
        t0 = time.perf_counter()
        chain(src, dst)
        best = min(best, time.perf_counter() - t0)
    print(f"{name:18s} {best * 1e6:8.0f} us")
for name, src in (("copy pinned->plain", pin_in.numpy()), ("copy plain->plain", r)):
    best = 1e9
    for _ in range(20):
        t0 = time.perf_counter()
        np.copyto(out, src)
        best = min(best, time.perf_counter() - t0)
    print(f"{name:18s} {best * 1e6:8.0f} us")
