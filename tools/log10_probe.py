#!/usr/bin/env python3
"""Host log10 throughput on this machine (the adaptive path's only host
arithmetic): single thread vs the engine's thread pool, allocating vs in-place
ufunc chains.  One JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from concurrent.futures import ThreadPoolExecutor
    from tomatis_audio_processor_amd import dsp
    n = 1653632
    r = (np.random.default_rng(0).random(n).astype(np.float32) * 0.3)
    ref = dsp.r_to_level(r)
    out = {}

    def best(f, k=5):
        ts = []
        for _ in range(k):
            t = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t)
        return round(min(ts) * 1e3, 3)

    out["single_alloc_ms"] = best(lambda: dsp.r_to_level(r))

    def inplace(a, b, o, tmp):
        np.add(r[a:b], dsp.EPS, out=tmp[a:b])
        np.log10(tmp[a:b], out=tmp[a:b])
        np.multiply(tmp[a:b], 20.0, out=tmp[a:b])
        o[a:b] = tmp[a:b]

    o = np.empty(n)
    tmp = np.empty(n, np.float32)
    out["single_inplace_ms"] = best(lambda: inplace(0, n, o, tmp))
    assert np.array_equal(o, ref)
    for T in (4, 8, 16, 32):
        pool = ThreadPoolExecutor(T)
        k = T
        e = np.linspace(0, n, k + 1).astype(np.int64)
        out[f"pool{T}_inplace_ms"] = best(
            lambda: list(pool.map(lambda i: inplace(e[i], e[i + 1], o, tmp), range(k))))
        assert np.array_equal(o, ref)
        pool.shutdown()
    out["cpus"] = len(os.sched_getaffinity(0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
