"""Adaptive Tomatis processor — MI355X drop-in for
src/process_tomatis_adaptive.py (``process()`` :157-373, CLI :376-420).

Head-room pre-attenuation, per-frame levels, bisection for the threshold that
puts ``target_c2`` of the frames in C2, min-hold gate, alpha cross-fade with a
dB-domain gain mix per frame, OLA normalised by max(sum w^2, 1e-8), restore and
a global 0.999 limiter.  The reference's NEP-50 precision switch (float32 for
loud input, float64 for input at or below -(max_gain+margin) dBFS)
is kept for the levels and the gate; the spectral path runs in float32 on the
GPU in both cases (<=1e-6 relative difference, inside the 1e-4 contract).

Also exports the reference's gate helpers (``compute_frame_levels``,
``simulate_gate``, ``find_optimal_threshold``) backed by the GPU kernels.
"""
from __future__ import annotations

import argparse
import csv
import sys

import numpy as np

from . import audio_io, dsp
from .engine import compute_frame_levels, find_optimal_threshold, simulate_gate  # noqa: F401

EPS = dsp.EPS
PEAK_LIMIT = dsp.PEAK_LIMIT
rms_dbfs = dsp.rms_dbfs
build_tilt_gain_db = dsp.build_tilt_gain_db


def db_to_lin(db):
    """10 ** (db / 20) in the input's precision (adaptive variant, no cast)."""
    return 10 ** (np.asarray(db) / 20.0)


def process(
    in_path,
    out_path,
    fc=1000.0,
    slope=12.0,
    c1_low=15.0, c1_high=-15.0,
    c2_low=-15.0, c2_high=15.0,
    target_c2=0.5,
    hyst_db=3.0,
    min_hold_ms=250.0,
    xfade_ms=500.0,
    headroom_margin=2.0,
    n_fft=4096,
    hop=2048,
    state_csv_path=None,
):
    """Adaptive gate + cross-fade tilt processing of ``in_path`` -> ``out_path``."""
    from . import engine, fileio
    import torch
    print("=" * 60 + "\nTomatis 自适应处理器 (MI355X)\n" + "=" * 60)
    print(f"\n读取输入: {in_path}")
    x, N, ch, sr = fileio.read_device(in_path)
    print(f"  采样率: {sr} Hz\n  声道数: {ch}\n  时长: {N / sr:.2f} s")
    ss = fileio.device_stream_set(x, N, ch, sr)
    pipe = engine.AdaptivePipeline(ss, fc=fc, slope=slope, c1_low=c1_low, c1_high=c1_high,
                                   c2_low=c2_low, c2_high=c2_high, target_c2=target_c2,
                                   hyst_db=hyst_db, min_hold_ms=min_hold_ms, xfade_ms=xfade_ms,
                                   headroom_margin=headroom_margin, n_fft=n_fft, hop=hop)
    res = pipe.run()
    torch.cuda.synchronize()
    y_dev = res.y[res.out_offs[0]:res.out_offs[0] + res.out_lens[0] * ch]
    states = res.stream_states(0)
    alpha = res.stream_alpha(0)
    a = res.frame_base[0]
    levels = res.extra["levels"][a:a + res.n_frames[0]].cpu().numpy()
    T = float(res.extra["thresholds"].cpu().numpy()[0])
    atten = pipe.atten[0]
    F = len(states)
    c2_ratio = int(np.count_nonzero(states == 2)) / F if F else 0.0
    switches = int(np.count_nonzero(states[1:] != states[:-1])) if F else 0
    print(f"\n门控参数:\n  hyst_db: {hyst_db} dB\n  min_hold: {min_hold_ms} ms "
          f"({pipe.mh} 帧)\n  xfade: {xfade_ms} ms ({pipe.xf} 帧)")
    print(f"\n预衰减: {-atten:.2f} dB\n  最优阈值 T: {T:.2f} dBFS\n  C2 占比: {c2_ratio * 100:.1f}%"
          f"\n  切换次数: {switches}")
    if out_path.lower().endswith(".wav"):
        audio_io.write(out_path, y_dev.cpu().numpy().reshape(-1, ch), sr, "WAV", "PCM_24")
        written = out_path
    else:  # reference: sf.write(out_path, y, sr, subtype='PCM_24')
        written, _ = fileio.write_device(out_path, y_dev, res.out_lens[0], ch, sr,
                                         log=lambda m: None)
    print(f"\n输出已保存: {written}")
    if state_csv_path:
        frame_sec = hop / sr
        with open(state_csv_path, "w", newline="", encoding="utf-8") as f:
            w = csv.writer(f)
            w.writerow(["frame_idx", "time_sec", "level_dbfs", "state", "alpha"])
            for i in range(F):
                t = (i + 1) * frame_sec
                w.writerow([i + 1, f"{t:.6f}", f"{levels[i]:.4f}",
                            "C1" if states[i] == 1 else "C2", f"{alpha[i]:.4f}"])
        print(f"状态已保存: {state_csv_path}")
    return 0


def build_parser():
    p = argparse.ArgumentParser(description="Tomatis 自适应处理器 (MI355X)")
    p.add_argument("-i", "--input", required=True, help="输入音频")
    p.add_argument("-o", "--output", required=True, help="输出音频")
    p.add_argument("--state_csv", help="状态 CSV 输出路径")
    p.add_argument("--fc", type=float, default=1000)
    p.add_argument("--slope", type=float, default=12)
    p.add_argument("--c1_low", type=float, default=15.0)
    p.add_argument("--c1_high", type=float, default=-15.0)
    p.add_argument("--c2_low", type=float, default=-15.0)
    p.add_argument("--c2_high", type=float, default=15.0)
    p.add_argument("--target_c2", type=float, default=0.5, help="目标 C2 占比")
    p.add_argument("--hyst_db", type=float, default=3.0, help="回差 dB（默认 3.0）")
    p.add_argument("--min_hold_ms", type=float, default=250.0, help="最短保持 ms（默认 250）")
    p.add_argument("--xfade_ms", type=float, default=500.0, help="Crossfade 过渡时间 ms（默认 500）")
    p.add_argument("--headroom_margin", type=float, default=2.0, help="预衰减余量 dB")
    p.add_argument("--n_fft", type=int, default=4096)
    p.add_argument("--hop", type=int, default=2048)
    return p


def main(argv=None):
    a = build_parser().parse_args(argv)
    return process(a.input, a.output, fc=a.fc, slope=a.slope, c1_low=a.c1_low,
                   c1_high=a.c1_high, c2_low=a.c2_low, c2_high=a.c2_high,
                   target_c2=a.target_c2, hyst_db=a.hyst_db, min_hold_ms=a.min_hold_ms,
                   xfade_ms=a.xfade_ms, headroom_margin=a.headroom_margin, n_fft=a.n_fft,
                   hop=a.hop, state_csv_path=a.state_csv)


if __name__ == "__main__":
    sys.exit(main())
