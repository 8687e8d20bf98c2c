#!/usr/bin/env python3
"""Diagnostic: one-hot gain rows (bin b passes, every other bin 0) through the
register STFT-OLA at n_fft 4096 / hop 1024 against the float64 numpy filter;
prints the relative interior error per probed bin (a bin the device applies
elsewhere shows ~1)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.diag_fft import ref_filter  # noqa: E402


def main():
    import torch  # noqa: F401
    from tomatis_audio_processor_amd import engine
    sr, n_fft, hop = 48000, 4096, 1024
    n = sr * 2 + 77
    ss = engine.StreamSet.synthetic(1, n, 2, sr, seed0=3)
    x = ss.x.cpu().numpy().reshape(n, 2).astype(np.float64)
    probes = [0, 1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 63, 64, 65, 96, 127, 128, 512, 1000, 1023,
              1024, 1025, 1500, 2000, 2016, 2032, 2040, 2047, 2048]
    bad = []
    for b in probes:
        g = np.zeros(n_fft // 2 + 1)
        g[b] = 1.0
        pipe = engine.StaticEqPipeline(ss, g, n_fft=n_fft, hop=hop, pad=True)
        y = pipe.run().output(0).astype(np.float64)
        yr = ref_filter(x, g, n_fft, hop)
        m = min(len(y), len(yr))
        a, e = 2 * n_fft, m - 2 * n_fft
        rel = np.abs(y[a:e] - yr[a:e]).max() / max(1e-30, np.abs(yr[a:e]).max())
        print(f"bin {b}: rel err {rel:.3e}", flush=True)
        if rel > 1e-3:
            bad.append(b)
    print("bad bins:", bad)


if __name__ == "__main__":
    main()
