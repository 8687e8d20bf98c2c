"""Golden-fixture case table (shared by tools/make_goldens.py and the tests).

Every case is a seeded synthetic input (``tomatis_audio_processor_amd.synth``)
plus reference parameters (``in_scale`` scales it, ``silence`` zeroes that many
samples at both ends).  ``bypass`` marks configurations outside the
reference's 48 kHz-stereo guard, run through the guard bypass.
Lengths are chosen so that standard-mode cases cover every tail residue class
that matters (N - n_fft mod hop = 0, 9, 259, 777) and at least one case spans
several 240000-sample limiter chunks.
"""
import numpy as np

S48, S44, S96 = 48000, 44100, 96000

CASES = [
    # --- standard (src/process_tomatis.py) ---------------------------------
    dict(name="std_c1_mono44k_2048_512", mode="standard", sr=S44, ch=1, N=441000,
         seed=1, bypass=True, params=dict(gate_ui=50, n_fft=2048, hop=512)),
    dict(name="std_48k_st_2048_512_tail259", mode="standard", sr=S48, ch=2,
         N=288000 + 2048 + 259, seed=2, params=dict(gate_ui=50, n_fft=2048, hop=512)),
    dict(name="std_48k_st_4096_2048_linear_gain", mode="standard", sr=S48, ch=2,
         N=144000 + 4096 + 777, seed=3,
         params=dict(gate_ui=50, gate_mode="linear", gate_offset=-90,
                     output_gain_db=3.0)),
    dict(name="std_44k_st_4096_1024_d0", mode="standard", sr=S44, ch=2,
         N=176400 + 4096 + 9, seed=4, bypass=True,
         params=dict(gate_ui=50, n_fft=4096, hop=1024, up_delay_ms=0.0,
                     hysteresis_db=2.0)),
    dict(name="std_96k_st_4096_1024_tail0", mode="standard", sr=S96, ch=2,
         N=4096 + 1024 * 230, seed=5, bypass=True,
         params=dict(gate_ui=50, n_fft=4096, hop=1024)),
    dict(name="std_48k_st_nolimit", mode="standard", sr=S48, ch=2, N=150000,
         seed=6, params=dict(gate_ui=30, n_fft=2048, hop=512, output_gain_db=-12.0)),
    dict(name="std_48k_st_hop300", mode="standard", sr=S48, ch=2, N=96000,
         seed=7, params=dict(gate_ui=50, n_fft=2048, hop=300)),
    dict(name="std_48k_st_short", mode="standard", sr=S48, ch=2, N=3000,
         seed=8, params=dict(gate_ui=0, n_fft=2048, hop=512)),
    # tail class where the reference's last-chunk limiter scale is set by an
    # ill-conditioned tail sample (sum w^2 < 1e-3; SURVEY F7, process_tomatis.py:447-453):
    # found by tools/find_tail_cases.py (1 of 440 lengths near 250 k)
    dict(name="std_48k_st_tail_ill", mode="standard", sr=S48, ch=2, N=250875,
         seed=2, params=dict(gate_ui=50, n_fft=2048, hop=512)),
    # any-size LDS path (n_fft other than 2048/4096; SURVEY §8 b "any --n_fft")
    dict(name="std_48k_st_1024_256", mode="standard", sr=S48, ch=2, N=96000 + 1024 + 77,
         seed=9, params=dict(gate_ui=50, n_fft=1024, hop=256)),
    dict(name="std_48k_st_8192_2048", mode="standard", sr=S48, ch=2, N=288000 + 8192 + 555,
         seed=10, params=dict(gate_ui=50, n_fft=8192, hop=2048)),
    # n_fft that is not a power of two (Bluestein) and 16384 (round 3)
    dict(name="std_48k_st_3000_750", mode="standard", sr=S48, ch=2, N=192000 + 3000 + 91,
         seed=51, params=dict(gate_ui=50, n_fft=3000, hop=750)),
    dict(name="std_48k_st_16384_4096", mode="standard", sr=S48, ch=2, N=288000 + 16384 + 313,
         seed=52, params=dict(gate_ui=50, n_fft=16384, hop=4096)),
    dict(name="xfade_48k_st_2400_600", mode="xfade", sr=S48, ch=2, N=144000 + 2400 + 7,
         seed=54, params=dict(gate_ui=50, gate_offset=-90, n_fft=2400, hop=600,
                              xfade_ms=200.0)),
    # --- xfade (src/process_tomatis_xfade.py) ------------------------------
    dict(name="xfade_48k_st_2048_512_500ms", mode="xfade", sr=S48, ch=2,
         N=288000 + 5000, seed=11,
         params=dict(gate_ui=50, gate_offset=-90, n_fft=2048, hop=512,
                     xfade_ms=500.0)),
    dict(name="xfade_96k_st_4096_1024_500ms", mode="xfade", sr=S96, ch=2,
         N=96000 * 3 + 333, seed=12, bypass=True,
         params=dict(gate_ui=50, gate_offset=-90, n_fft=4096, hop=1024,
                     xfade_ms=500.0)),
    dict(name="xfade_48k_st_0ms", mode="xfade", sr=S48, ch=2, N=120000, seed=13,
         params=dict(gate_ui=50, gate_offset=-90, n_fft=2048, hop=512,
                     xfade_ms=0.0)),
    # --- adaptive (src/process_tomatis_adaptive.py) ------------------------
    dict(name="adapt_44k_st_2048_512", mode="adaptive", sr=S44, ch=2, N=44100 * 8,
         seed=21, params=dict(n_fft=2048, hop=512)),
    dict(name="adapt_44k_st_quiet_f64", mode="adaptive", sr=S44, ch=2,
         N=44100 * 6 + 123, seed=22, in_scale=0.01, params=dict(n_fft=2048, hop=512)),
    dict(name="adapt_48k_mono_4096_2048", mode="adaptive", sr=S48, ch=1,
         N=48000 * 7, seed=23, params=dict()),
    # the adaptive processor takes any channel count (no guard, adaptive.py:179-183)
    dict(name="adapt_48k_4ch_2048_512", mode="adaptive", sr=S48, ch=4, N=48000 * 5 + 321,
         seed=24, params=dict(n_fft=2048, hop=512)),
    # more channels than the L + iR register path (round 3: 10 channels, and a
    # prime n_fft on the adaptive path)
    dict(name="adapt_48k_10ch_2048_512", mode="adaptive", sr=S48, ch=10, N=48000 * 3 + 77,
         seed=53, params=dict(n_fft=2048, hop=512)),
    dict(name="adapt_44k_st_1999_500", mode="adaptive", sr=S44, ch=2, N=44100 * 4 + 5,
         seed=55, params=dict(n_fft=1999, hop=500)),
    dict(name="adapt_44k_st_512_128", mode="adaptive", sr=S44, ch=2, N=44100 * 4 + 99,
         seed=25, params=dict(n_fft=512, hop=128)),
    # --- layer 2 (src/layer2_apply_eq.py) -----------------------------------
    dict(name="l2_48k_st_pad_gp", mode="layer2", sr=S48, ch=2, N=150000 + 17,
         seed=31, params=dict(n_fft=2048, hop=512)),
    dict(name="l2_48k_st_nopad_gain", mode="layer2", sr=S48, ch=2, N=100000,
         seed=32, params=dict(pad=False, global_gain_db=-6.0,
                              auto_gain_protect=False)),
    # gain protect set by a well-conditioned sample: digital silence at both
    # ends keeps the ill-conditioned head/tail samples exactly 0, so peak_seen
    # (layer2_apply_eq.py:177,213) and the _gp scale are determined
    dict(name="l2_48k_st_pad_gp_silent_edges", mode="layer2", sr=S48, ch=2, N=150000,
         seed=33, silence=4096, params=dict(n_fft=2048, hop=512, global_gain_db=12.0)),
    # --- layer 2b (src/layer2b_apply_residual_eq*.py) -----------------------
    dict(name="l2b_96k_st_4096_1024", mode="layer2b", sr=S96, ch=2,
         N=96000 * 2 + 1500, seed=41, params=dict(n_fft=4096, hop=1024)),
    dict(name="l2b_safe_48k_st", mode="layer2b_safe", sr=S48, ch=2, N=120000,
         seed=42, params=dict(n_fft=2048, hop=512)),
]

BY_NAME = {c["name"]: c for c in CASES}


def eq_curve(n=48):
    """Synthetic layer-2 EQ curve (freq_hz, delta_db), float-exact formula."""
    f = np.geomspace(20.0, 20000.0, n)
    d = 4.0 * np.sin(np.linspace(0.0, 3.0 * np.pi, n)) - 1.5
    return f, d


def eq_csv_rows(case=None):
    f, d = eq_curve()
    lines = ["freq_hz,delta_db"] + [f"{float(a)!r},{float(b)!r}" for a, b in zip(f, d)]
    return "\n".join(lines) + "\n"


def diff_curve(sr=48000, n_fft=4096):
    """Synthetic ``diff_spectrum.csv`` in compare_audio.py's layout."""
    freqs = np.fft.rfftfreq(n_fft, 1 / sr)
    lf = np.log10(np.maximum(freqs, 1.0))
    d = 5.0 * np.sin(2.1 * lf) + 1.5 * np.cos(37.0 * lf) - 0.5
    return freqs, d


def diff_csv_rows(case=None):
    f, d = diff_curve()
    lines = ["freq_hz,delta_db_base_minus_cand"]
    lines += ["%.18e,%.18e" % (a, b) for a, b in zip(f, d)]
    return "\n".join(lines) + "\n"
