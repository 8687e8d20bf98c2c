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
    try:   # reading from / writing to page-locked (torch pin_memory) blocks
        import torch
        rp = torch.empty(n, dtype=torch.float32, pin_memory=True)
        op = torch.empty(n, dtype=torch.float64, pin_memory=True)
        rp.numpy()[:] = r
        rpn, opn = rp.numpy(), op.numpy()
        tmp2 = np.empty(n, np.float32)

        def pinned():
            np.add(rpn, dsp.EPS, out=tmp2)
            np.log10(tmp2, out=tmp2)
            np.multiply(tmp2, 20.0, out=tmp2)
            opn[:] = tmp2

        out["pinned_in_out_ms"] = best(pinned)
        out["pinned_read_copy_ms"] = best(lambda: np.copy(rpn))
        out["pinned_write_ms"] = best(lambda: opn.__setitem__(slice(None), o))
    except Exception as e:  # no ROCm runtime: skip
        out["pinned"] = str(e)[:80]
    out["cpus"] = len(os.sched_getaffinity(0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
