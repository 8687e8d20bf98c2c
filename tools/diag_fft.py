#!/usr/bin/env python3
"""Diagnostic: a random real gain row through the register kernels' STFT-OLA
(StaticEqPipeline, head pad) against a float64 numpy STFT filter of the same
frames; prints the max interior error per (n_fft, hop) and the frame-grid
position (lane = pos mod P, register = pos // P) of the worst samples."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ref_filter(x, g, n_fft, hop):
    w = np.hanning(n_fft).astype(np.float32).astype(np.float64)
    pl = n_fft // 2
    xp = np.concatenate([np.zeros((pl, x.shape[1])), x, np.zeros((pl, x.shape[1]))])
    F = (len(xp) - n_fft) // hop + 1
    y = np.zeros(((F - 1) * hop + n_fft, x.shape[1]))
    ws = np.zeros(len(y))
    for f in range(F):
        s = f * hop
        fr = xp[s:s + n_fft] * w[:, None]
        y[s:s + n_fft] += np.fft.irfft(np.fft.rfft(fr, axis=0) * g[:, None], n_fft, axis=0) * w[:, None]
        ws[s:s + n_fft] += w * w
    return y / (ws[:, None] + 1e-12)


def main():
    import torch
    from tomatis_audio_processor_amd import engine
    sr = 48000
    rng = np.random.default_rng(5)
    for n_fft, hop, P in ((2048, 512, 64), (4096, 1024, 128), (4096, 2048, 128)):
        n = sr * 4 + 77
        ss = engine.StreamSet.synthetic(1, n, 2, sr, seed0=3)
        ss.x.mul_(0.1)
        x = ss.x.cpu().numpy().reshape(n, 2).astype(np.float64)
        g = rng.uniform(0.2, 3.0, n_fft // 2 + 1)
        pipe = engine.StaticEqPipeline(ss, g, n_fft=n_fft, hop=hop, pad=True)
        yr = ref_filter(x, g.astype(np.float32).astype(np.float64), n_fft, hop)
        for rep in range(3):
            y = pipe.run().output(0).astype(np.float64)
            m = min(len(y), len(yr))
            a, b = 2 * n_fft, m - 2 * n_fft
            err = np.abs(y[a:b] - yr[a:b]).max(axis=1)
            bad = np.nonzero(err > 1e-4)[0] + a
            lanes = np.bincount((bad % hop) % P, minlength=P)
            print(f"n_fft {n_fft} hop {hop} rep {rep}: max interior err {err.max():.3e}, "
                  f"{len(bad)} samples > 1e-4; lanes hit: {np.nonzero(lanes)[0].tolist()[:40]}; "
                  f"hop blocks hit: {np.unique(bad // hop).tolist()[:20]}", flush=True)


if __name__ == "__main__":
    main()
