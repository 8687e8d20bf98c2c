"""Host numpy log10 throughput over threads (the adaptive path's host step)."""
import time, os
from concurrent.futures import ThreadPoolExecutor
import numpy as np
n = 825_000
r = (np.random.default_rng(0).random(n).astype(np.float32) * 0.1 + 1e-4)
out = np.empty(n, np.float32)
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for k in (1, 2, 4, 8, 16):
    pool = ThreadPoolExecutor(k)
    edges = np.linspace(0, n, k + 1).astype(np.int64)
    def part(i):
        a, b = edges[i], edges[i + 1]
        np.log10(r[a:b], out=out[a:b])
    best = 1e9
    for _ in range(20):
        t = time.perf_counter()
        if k == 1:
            np.log10(r, out=out)
        else:
            list(pool.map(part, range(k)))
        best = min(best, time.perf_counter() - t)
    print(f"threads {k}: {best * 1e6:.0f} us for {n} float32 log10")
    pool.shutdown()
r64 = r.astype(np.float64); o64 = np.empty(n)
t = time.perf_counter(); np.log10(r64, out=o64); print(f"f64 1 thread {1e6 * (time.perf_counter() - t):.0f} us")
