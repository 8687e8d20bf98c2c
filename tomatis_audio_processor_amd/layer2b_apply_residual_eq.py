"""Layer-2b residual EQ — MI355X drop-in for src/layer2b_apply_residual_eq.py
(``smooth_on_logfreq`` :12-35, ``build_eq_from_residual`` :37-55, CLI :57-165).

diff_spectrum.csv -> log-frequency moving average -> clamped per-bin gain ->
the same fused STFT/OLA with no padding (frames at k*hop over the input; the
tail beyond the last full frame is dropped, as the reference).
"""
from __future__ import annotations

import argparse

import numpy as np

from . import audio_io, dsp

EPS = dsp.EPS
smooth_on_logfreq = dsp.smooth_on_logfreq
build_eq_from_residual = dsp.build_eq_from_residual


def db_to_lin(db):
    return 10.0 ** (db / 20.0)


def run_residual_eq(in_audio, out_audio, eq_lin, n_fft, hop):
    from . import engine, fileio
    import torch
    sr, ch, _ = audio_io.info(in_audio)
    assert ch == 2, "只支持双声道"
    x, n, ch, sr = fileio.read_device(in_audio)
    ss = fileio.device_stream_set(x, n, ch, sr)
    pipe = engine.StaticEqPipeline(ss, eq_lin, n_fft=n_fft, hop=hop, pad=False)
    res = pipe.run()
    torch.cuda.synchronize()
    y = res.y[res.out_offs[0]:res.out_offs[0] + res.out_lens[0] * ch]
    written, _ = fileio.write_device(out_audio, y, res.out_lens[0], ch, sr, log=lambda m: None)
    return written


def build_parser(safe=False):
    ap = argparse.ArgumentParser()
    if safe:
        ap.add_argument("--in_audio", required=True)
        ap.add_argument("--out_audio", required=True)
        ap.add_argument("--diff_csv", default="diff_spectrum.csv")
        ap.add_argument("--n_fft", type=int, default=4096)
        ap.add_argument("--hop", type=int, default=2048)
        ap.add_argument("--smooth_win", type=int, default=61)
        ap.add_argument("--clamp_hi", type=float, default=1.0)
        ap.add_argument("--hf_start", type=float, default=3000.0)
        return ap
    ap.add_argument("--in_audio", required=True, help="候选音频（例如 D_MNF_matched_v2_eq_gp.flac）")
    ap.add_argument("--out_audio", required=True, help="输出音频")
    ap.add_argument("--diff_csv", default="diff_spectrum.csv", help="对比生成的 diff_spectrum.csv")
    ap.add_argument("--n_fft", type=int, default=4096)
    ap.add_argument("--hop", type=int, default=2048)
    ap.add_argument("--smooth_win", type=int, default=41)
    ap.add_argument("--clamp_hi", type=float, default=6.0)
    ap.add_argument("--mid_start", type=float, default=3000.0)
    ap.add_argument("--mid_clamp_hi", type=float, default=2.0)
    ap.add_argument("--hf_start", type=float, default=8000.0)
    ap.add_argument("--hf_clamp_hi", type=float, default=0.0)
    return ap


def main(argv=None):
    args = build_parser().parse_args(argv)
    res_freq, res_db = dsp.read_diff_csv(args.diff_csv)
    res_db_s = smooth_on_logfreq(res_freq, res_db, win=args.smooth_win)
    sr, ch, _ = audio_io.info(args.in_audio)
    freqs = np.fft.rfftfreq(args.n_fft, 1.0 / sr)
    eq_lin, _ = build_eq_from_residual(freqs, res_freq, res_db_s, clamp_lo=-6.0,
                                       clamp_hi=args.clamp_hi, mid_start=args.mid_start,
                                       mid_clamp_hi=args.mid_clamp_hi, hf_start=args.hf_start,
                                       hf_clamp_hi=args.hf_clamp_hi)
    run_residual_eq(args.in_audio, args.out_audio, eq_lin, args.n_fft, args.hop)
    print(f"[DONE] Applied residual EQ to {args.out_audio}")


if __name__ == "__main__":
    main()
