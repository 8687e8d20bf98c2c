"""Host logic of the ill-conditioned-scale flags (conditioning.py), on the oracle.

The flag decides whether a limiter / gain-protect scale is determined by
well-conditioned samples (SURVEY.md F7, §8(c) "whole-chunk scale mismatches
... are flagged").  These CPU tests pin (1) the window sums against the
reference's own float32 sums, (2) the error model against the reference's
float32 arithmetic, and (3) the flags on the reference's golden outputs.
"""
import numpy as np
import pytest

from tests.golden_util import BY_NAME, CASES, case_input, load_fixture, run_oracle
from tomatis_audio_processor_amd import conditioning as cd


def _std_flags(c, ref):
    N = c["N"]
    n_fft, hop = c["params"].get("n_fft", 4096), c["params"].get("hop", 2048)
    b = ref["bounds"]
    ranges = [(max(0, int(b[i])), min(N, int(b[i + 1]))) for i in range(len(b) - 1)]
    pre = ref["y"].astype(np.float64).copy()
    peaks = []
    for i, (a, e) in enumerate(ranges):
        s = ref["scales"][i] or 1.0
        pre[a:e] /= s
        peaks.append(float(np.abs(pre[a:e]).max()) if e > a else 0.0)
    q = cd.edge_index(N, n_fft)
    fl = cd.chunk_flags(pre[q], q, out_begin=0, first_start=-(n_fft // 2),
                        n_frames=len(ref["states"]), n_fft=n_fft, hop=hop, norm="eps",
                        chunk_lo=[r[0] for r in ranges], chunk_hi=[r[1] for r in ranges],
                        peaks=peaks, limit=0.999)
    return [f["flagged"] for f in fl]


@pytest.mark.parametrize("name", ["std_48k_st_2048_512_tail259", "std_96k_st_4096_1024_tail0",
                                  "std_48k_st_hop300"])
def test_window_sums_match_reference(name):
    c = BY_NAME[name]
    ref = run_oracle(c)
    p = c["params"]
    n_fft, hop = p.get("n_fft", 4096), p["hop"]
    pos = np.arange(-(n_fft // 2), len(ref["wsum"]) - n_fft // 2)
    s1, s2 = cd.window_sums(n_fft, hop, -(n_fft // 2), len(ref["states"]), pos)
    np.testing.assert_allclose(s2, ref["wsum"], rtol=1e-5, atol=1e-9)


def test_error_model_bounds_reference_float32():
    """|reference float32 - exact| <= (KAPPA_INT * A + KAPPA_EDGE * A * S1/den) / 4
    on loud random streams (the constants' 8x margin, checked at 4x here)."""
    from oracle import tomatis_oracle as orc
    rng = np.random.default_rng(3)
    for n_fft, hop in ((2048, 512), (4096, 1024)):
        win, win2 = orc.hann_sym(n_fft)
        w64 = win.astype(np.float64)
        for _ in range(3):
            N = int(rng.integers(4 * n_fft, 9 * n_fft))
            x = (rng.standard_normal((N, 2)) * rng.uniform(0.1, 3)).astype(np.float32)
            pad, pe, F, starts = orc._std_schedule(N, n_fft, hop)
            xpad = np.concatenate([np.zeros((pad, 2), np.float32), x,
                                   np.zeros((pe, 2), np.float32)])
            frames = orc.frame_view(xpad, n_fft, hop, F)
            g = orc.db_to_lin_f32(rng.uniform(-15, 15, n_fft // 2 + 1))[None, :]
            g = np.broadcast_to(g, (F, n_fft // 2 + 1))
            y32 = orc.spectral_filter(frames, win, g)
            length = int(starts[-1]) + n_fft + pad
            o32, w = orc.ola(y32, starts, n_fft, win2, length, origin=-pad)
            X = np.fft.rfft(frames.astype(np.float64) * w64[None, :, None], axis=1)
            y64 = np.fft.irfft(X * g[:, :, None], n=n_fft, axis=1) * w64[None, :, None]
            o64 = np.zeros((length, 2))
            for k in range(F):
                o64[starts[k] + pad:starts[k] + pad + n_fft] += y64[k]
            pos = np.arange(length) - pad
            s1, s2 = cd.window_sums(n_fft, hop, -pad, F, pos)
            err = np.abs(o32 / (w[:, None] + 1e-12) - o64 / (s2[:, None] + 1e-12)).max(axis=1)
            yab = np.abs(o64 / (s2[:, None] + 1e-12)).max(axis=1) * (s2 >= cd.TAU)
            from scipy.ndimage import maximum_filter1d
            A = maximum_filter1d(yab, 2 * n_fft + 1)
            bound = (cd.KAPPA_INT * A + cd.KAPPA_EDGE * A * s1 / (s2 + 1e-12)) / 4
            assert np.all(err[bound > 0] <= bound[bound > 0])


# goldens whose limiter scale is set by an ill-conditioned tail sample: the
# 2-5 % tail class (found by tools/find_tail_cases.py) and the pe = 0 case
# whose last frame ends exactly at N (sum w^2 = 3.5e-13 at N-2: the peak is
# z/w of the filter's time-aliased tail, 37.6 before the limiter)
FLAGGED = {"std_48k_st_tail_ill": [False, True], "std_96k_st_4096_1024_tail0": [True]}


@pytest.mark.parametrize("case", [c for c in CASES if c["mode"] in ("standard", "xfade")],
                         ids=lambda c: c["name"])
def test_golden_chunk_flags(case):
    """Flags on the reference's own outputs: only the two tail-set scales."""
    ref = run_oracle(case, load_fixture(case["name"]), case_input(case))
    fl = _std_flags(case, ref)
    assert fl == FLAGGED.get(case["name"], [False] * len(fl))
    # and where flagged, an ill-conditioned sample does reach the chunk peak's order
    if any(fl):
        N = case["N"]
        pad = ref["pad"]
        w = ref["wsum"][pad:pad + N]
        b = ref["bounds"]
        c = fl.index(True)
        a, e = max(0, int(b[c])), min(N, int(b[c + 1]))
        p = np.abs(ref["y"][a:e]).max(axis=1)
        assert p[w[a:e] < cd.TAU].max() >= 0.5 * p.max()


@pytest.mark.parametrize("name,flagged", [("l2_48k_st_pad_gp", True),
                                          ("l2_48k_st_pad_gp_silent_edges", False)])
def test_gain_protect_flag(name, flagged):
    c = BY_NAME[name]
    fx = load_fixture(name)
    ref = run_oracle(c, fx, case_input(c))
    y = ref["y"]
    p = c["params"]
    n_fft, hop = p.get("n_fft", 4096), p.get("hop", 2048)
    pl = n_fft // 2 if p.get("pad", True) else 0
    q = cd.edge_index(len(y), n_fft)
    fl = cd.chunk_flags(y[q], q, out_begin=-pl, first_start=-pl, n_frames=ref["frames"],
                        n_fft=n_fft, hop=hop, norm="eps", chunk_lo=[0], chunk_hi=[len(y)],
                        peaks=[float(np.abs(y).max())], limit=0.99)
    assert fl[0]["flagged"] is flagged


def test_flag_logic_synthetic():
    """A peak set by a sample with a tiny window sum is flagged; the same chunk
    with that sample quiet is not; an unlimited chunk is never flagged."""
    n_fft, hop, N = 2048, 512, 2048 + 512 * 35   # pe = 0: the last frame ends at N
    q = cd.edge_index(N, n_fft)
    y = np.full((len(q), 1), 0.5)
    kw = dict(out_begin=0, first_start=-1024, n_frames=(1024 + N - n_fft) // hop + 1,
              n_fft=n_fft, hop=hop, norm="eps", chunk_lo=[0], chunk_hi=[N])
    last = len(q) - 2                              # sum w^2 ~ 5e-12 there
    y2 = y.copy()
    y2[last] = 3.0
    assert cd.chunk_flags(y2, q, peaks=[3.0], limit=0.999, **kw)[0]["flagged"]
    assert not cd.chunk_flags(y, q, peaks=[1.5], limit=0.999, **kw)[0]["flagged"]
    assert not cd.chunk_flags(y2, q, peaks=[3.0], limit=np.inf, **kw)[0]["flagged"]
