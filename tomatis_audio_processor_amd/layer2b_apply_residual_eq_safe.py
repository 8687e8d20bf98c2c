"""'Safe' layer-2b residual EQ — MI355X drop-in for
src/layer2b_apply_residual_eq_safe.py: +-1 dB clamp, 0 dB at and above 3 kHz,
smoothing window 61 by default."""
from __future__ import annotations

import numpy as np

from . import audio_io, dsp
from .layer2b_apply_residual_eq import build_parser, run_residual_eq

EPS = dsp.EPS
smooth_on_logfreq = dsp.smooth_on_logfreq
build_eq_from_residual_safe = dsp.build_eq_from_residual_safe


def main(argv=None):
    args = build_parser(safe=True).parse_args(argv)
    res_freq, res_db = dsp.read_diff_csv(args.diff_csv)
    res_db_s = smooth_on_logfreq(res_freq, res_db, win=args.smooth_win)
    sr, ch, _ = audio_io.info(args.in_audio)
    freqs = np.fft.rfftfreq(args.n_fft, 1.0 / sr)
    eq_lin, _ = build_eq_from_residual_safe(freqs, res_freq, res_db_s, clamp_lo=-1.0,
                                            clamp_hi=args.clamp_hi, hf_start=args.hf_start)
    run_residual_eq(args.in_audio, args.out_audio, eq_lin, args.n_fft, args.hop)
    print(f"[DONE] Applied SafeB residual EQ to {args.out_audio}")


if __name__ == "__main__":
    main()
