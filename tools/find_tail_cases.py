#!/usr/bin/env python3
"""Sweep stream lengths with the oracle (bit-exact with the reference) for the
tail class of SURVEY.md §7 hard part 4: the last limiter chunk's scale set by
a sample whose OLA window sum is < 1e-3 (src/process_tomatis.py:447-453).
For each length it also evaluates the conditioning flag, and reports both, so
the flag can be checked to fire on exactly the affected lengths.

Usage: python tools/find_tail_cases.py [--seeds 2 9] [--n0 250000] [--count 220] [--step 7]
(Found std_48k_st_tail_ill: seed 2, N = 250875; 1 of 440 lengths, flagged 1.)
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import tomatis_oracle as orc  # noqa: E402
from tomatis_audio_processor_amd import conditioning as cd  # noqa: E402
from tomatis_audio_processor_amd.synth import synth_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[2, 9])
    ap.add_argument("--n0", type=int, default=250000)
    ap.add_argument("--count", type=int, default=220)
    ap.add_argument("--step", type=int, default=7)
    ap.add_argument("--sr", type=int, default=48000)
    ap.add_argument("--n_fft", type=int, default=2048)
    ap.add_argument("--hop", type=int, default=512)
    a = ap.parse_args()
    n_fft, hop, sr = a.n_fft, a.hop, a.sr
    tot = hits = flagged = missed = 0
    for seed in a.seeds:
        for N in range(a.n0, a.n0 + a.count * a.step, a.step):
            x = synth_stream(seed, N, 2, sr)
            ref = orc.process_standard(x, sr, gate_ui=50, n_fft=n_fft, hop=hop)
            b, sc = ref["bounds"], ref["scales"]
            ranges = [(max(0, int(b[c])), min(N, int(b[c + 1]))) for c in range(len(b) - 1)]
            pre = ref["y"].astype(np.float64).copy()
            peaks = []
            for c, (lo, hi) in enumerate(ranges):
                pre[lo:hi] /= sc[c] or 1.0
                peaks.append(float(np.abs(pre[lo:hi]).max()) if hi > lo else 0.0)
            q = cd.edge_index(N, n_fft)
            fl = cd.chunk_flags(pre[q], q, out_begin=0, first_start=-(n_fft // 2),
                                n_frames=len(ref["states"]), n_fft=n_fft, hop=hop, norm="eps",
                                chunk_lo=[r[0] for r in ranges], chunk_hi=[r[1] for r in ranges],
                                peaks=peaks, limit=0.999)[-1]["flagged"]
            pad = ref["pad"]
            w = ref["wsum"][pad:pad + N]
            lo, hi = ranges[-1]
            ill = w[lo:hi] < cd.TAU
            p = np.abs(pre[lo:hi]).max(axis=1)
            hit = bool(sc[-1] not in (None, 1.0) and ill.any() and p[ill].max() > p[~ill].max())
            tot += 1
            hits += hit
            flagged += fl
            missed += hit and not fl
            if hit or fl:
                print(f"seed {seed} N {N} (N-n_fft)%hop={(N - n_fft) % hop} tail-set={hit} "
                      f"flagged={fl}", flush=True)
    print(f"{tot} lengths: {hits} tail-set scales, {flagged} flagged, {missed} missed")


if __name__ == "__main__":
    main()
