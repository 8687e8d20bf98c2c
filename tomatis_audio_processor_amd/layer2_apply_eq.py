"""Layer-2 static EQ through the STFT/OLA — MI355X drop-in for
src/layer2_apply_eq.py (``load_eq_csv`` :11-46, ``build_gain_per_bin`` :48-64,
``apply_eq_stft`` :66-237, CLI :239-263).

One static gain row per file through the same fused kernel, on the device
file path (``fileio``: FLAC bytes -> HBM -> FLAC); the head pad is kept in the
output (padded coordinates), and gain protection writes a ``*_gp.flac`` copy
scaled by ``peak_target / peak`` when the output peak exceeds ``peak_target``:
like the reference, the copy scales the PCM_24 samples of the main output
(re-quantised on the device instead of re-read from the file).
"""
from __future__ import annotations

import argparse

import numpy as np

from . import audio_io, dsp  # noqa: F401  (audio_io: format probe)

EPS = dsp.EPS
load_eq_csv = dsp.load_eq_csv
build_gain_per_bin = dsp.build_gain_per_bin


def db_to_lin(db):
    return 10.0 ** (db / 20.0)


def apply_eq_stft(
    in_path,
    out_path,
    eq_csv,
    n_fft=4096,
    hop=2048,
    pad=True,
    global_gain_db=0.0,
    auto_gain_protect=True,
    peak_target=0.99,
    allow_any_format=False,
):
    from . import engine, fileio
    import torch
    sr, ch, _ = audio_io.info(in_path)
    if not allow_any_format:
        if sr != 48000:
            raise ValueError(f"期望 48kHz，实际 {sr}")
        if ch != 2:
            raise ValueError(f"期望双声道，实际 {ch}")
    # the device file path: FLAC bytes -> HBM, the fused STFT/OLA, HBM -> FLAC
    x, n, ch, sr = fileio.read_device(in_path)
    eq_freqs, eq_db = load_eq_csv(eq_csv)
    gain_bins = build_gain_per_bin(sr, n_fft, eq_freqs, eq_db)
    ss = fileio.device_stream_set(x, n, ch, sr)
    pipe = engine.StaticEqPipeline(ss, gain_bins, n_fft=n_fft, hop=hop, pad=pad,
                                   global_gain_db=global_gain_db)
    res = pipe.run()
    n_out = res.out_lens[0]
    y_dev = res.y[res.out_offs[0]:res.out_offs[0] + n_out * ch]
    written, is_flac = fileio.write_device(out_path, y_dev, n_out, ch, sr, log=lambda m: None)
    if not is_flac:
        print(f"[WARN] FLAC 写入失败，先写 WAV: {written}")
    peak_seen = float(res.stream_peaks(0)[0])
    if auto_gain_protect and peak_seen > peak_target:
        scale = peak_target / max(peak_seen, EPS)
        print(f"[GAIN_PROTECT] peak={peak_seen:.4f} > {peak_target}, apply scale={scale:.4f}")
        # the reference re-reads its PCM_24 output and scales that
        # (src/layer2_apply_eq.py:220-231): the same samples, on the device
        ygp = engine.scale_copy(fileio.requantize_device(y_dev, n_out, ch, 24), scale)
        tmp_out = out_path.replace(".flac", "_gp.flac")
        gp_written, _ = fileio.write_device(tmp_out, ygp, n_out, ch, sr, log=lambda m: None)
        print(f"[DONE] gain-protected file: {gp_written}")
    torch.cuda.synchronize()
    print("[DONE] EQ applied.")
    if not is_flac:
        print(f"[NOTE] 输出为 WAV: {written}，可用 ffmpeg 转 FLAC。")
    return dict(out=written, peak_seen=peak_seen)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-i", "--input", required=True)
    ap.add_argument("-o", "--output", required=True)
    ap.add_argument("--eq_csv", required=True)
    ap.add_argument("--n_fft", type=int, default=4096)
    ap.add_argument("--hop", type=int, default=2048)
    ap.add_argument("--no_pad", action="store_true")
    ap.add_argument("--gain_db", type=float, default=0.0,
                    help="额外整体增益（dB），想完全匹配录音电平可用 -17.77")
    ap.add_argument("--no_gain_protect", action="store_true")
    ap.add_argument("--allow_any_format", action="store_true")
    a = ap.parse_args(argv)
    apply_eq_stft(a.input, a.output, a.eq_csv, n_fft=a.n_fft, hop=a.hop, pad=(not a.no_pad),
                  global_gain_db=a.gain_db, auto_gain_protect=(not a.no_gain_protect),
                  allow_any_format=a.allow_any_format)


if __name__ == "__main__":
    main()


__all__ = ["apply_eq_stft", "load_eq_csv", "build_gain_per_bin", "db_to_lin", "np"]
