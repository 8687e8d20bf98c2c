"""Host level chain (add EPS, log10, x20 -> f64) timing: numpy buffers vs page-locked torch buffers."""
import time
import numpy as np
import torch
n = 825_000
EPS = 1e-12
r = (np.random.default_rng(0).random(n).astype(np.float32) * 0.1 + 1e-4)
pin_r = torch.empty(n, dtype=torch.float32, pin_memory=True)
pin_o = torch.empty(n, dtype=torch.float64, pin_memory=True)
pin_r.numpy()[:] = r
tmp = np.empty(n, np.float32)
out = np.empty(n, np.float64)
def chain(rr, oo):
    np.add(rr, EPS, out=tmp)
    np.log10(tmp, out=tmp)
    np.multiply(tmp, 20.0, out=oo, dtype=np.float32, casting="unsafe")
for name, rr, oo in (("numpy", r, out), ("pinned", pin_r.numpy(), pin_o.numpy())):
    best = 1e9
    for _ in range(20):
        t = time.perf_counter(); chain(rr, oo); best = min(best, time.perf_counter() - t)
    print(f"{name}: {best*1e6:.0f} us")
for step in ("add", "log10", "mul"):
    best = 1e9
    for _ in range(20):
        t = time.perf_counter()
        if step == "add": np.add(r, EPS, out=tmp)
        elif step == "log10": np.log10(tmp, out=tmp)
        else: np.multiply(tmp, 20.0, out=out, dtype=np.float32, casting="unsafe")
        best = min(best, time.perf_counter() - t)
    print(f"{step}: {best*1e6:.0f} us")
