"""GPU parity of the analysis spectra through the C ABI.

* vs the reference's own outputs (tests/golden/an_*.npz): frame counts / used
  frames exact; spectra within float32 FFT rounding (tolerances below: the
  device FFT is this build's own, pocketfft's rounding differs by ~1e-7 rel.);
* the exact pieces bit-for-bit vs the oracle / numpy: per-frame r (numpy
  pairwise order), the level-gated frame masks, the median over frames
  (np.median, both parities, negatives, ties, masks) and the mean over frames;
* any n_fft (Bluestein lengths, 16384, tiny frames): reference goldens at
  3000/1000/1500/6000/100/16384, bit-exact r for numpy's tree at any length,
  band tilts vs the reference formula, and the size bounds.
"""
import json
import os

import numpy as np
import pytest

from tests.golden.an_cases import AN_CASES, an_inputs
from oracle import tomatis_oracle as orc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAG_RTOL = 2e-5      # |mag_gpu - mag_ref| <= MAG_RTOL * max(mag_ref)
DB_ATOL = 2e-3       # dB, medians of log-power / ratio spectra


def load(name):
    with np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


@pytest.fixture(scope="module")
def an():
    import torch
    assert torch.cuda.is_available()
    from tomatis_audio_processor_amd import analysis, _lib
    _lib.lib()
    return analysis


@pytest.mark.parametrize("c", AN_CASES, ids=[c["name"] for c in AN_CASES])
def test_device_vs_reference(an, c):
    fx = load(c["name"])
    x, y, states = an_inputs(c)
    if c["fn"] == "stft_mag_avg":
        ref = fx["mag"]
        for m in (an.stft_mag_avg(orc.power_mono(x), c["sr"], c["n_fft"], c["hop"]),
                  an.stft_mag_avg(x, c["sr"], c["n_fft"], c["hop"], premix="power_mono")):
            assert m.dtype == np.float32 and m.shape == ref.shape
            err = float(np.max(np.abs(m - ref)))
            assert err <= MAG_RTOL * float(ref.max()), err
    elif c["fn"] == "stft_logpower_median":
        f, med, used = an.stft_logpower_median(x, c["sr"], c["n_fft"], c["hop"], c["music_dbfs"])
        assert used == int(fx["used"])
        assert np.array_equal(f, fx["freqs"])
        err = float(np.max(np.abs(med - fx["med"])))
        assert err <= DB_ATOL, err
    else:
        f, c1, c2, n1, n2 = an.compute_conditional_spectrum(x, y, c["sr"], states, c["n_fft"],
                                                            c["hop"], c["level_threshold"])
        assert (n1, n2) == (int(fx["n1"]), int(fx["n2"]))
        for a, b in ((c1, fx["c1_db"]), (c2, fx["c2_db"])):
            err = float(np.max(np.abs(a - b)))
            assert err <= DB_ATOL, err


@pytest.mark.parametrize("n_fft,hop,ch,mode", [(2048, 512, 2, 0), (4096, 1024, 1, 0),
                                                (8192, 4096, 2, 1), (256, 100, 2, 1),
                                                (1024, 300, 2, 0),
                                                # numpy's tree for any length (program)
                                                (3000, 750, 2, 0), (12000, 3000, 2, 1),
                                                (16384, 4096, 1, 0), (100, 30, 2, 1),
                                                (16, 5, 1, 0), (1500, 375, 1, 0)])
def test_frame_r_bit_exact(an, n_fft, hop, ch, mode):
    from tomatis_audio_processor_amd.synth import synth_stream
    x = synth_stream(40 + n_fft, n_fft * 7 + 3 * hop + 11, ch, 48000)
    xd = an._dev(x, ch=True)
    r = an._frame_r(xd, len(x), ch, n_fft, hop, mode).cpu().numpy()
    ref = orc.analyze_frame_r(x, n_fft, hop) if mode == 1 else orc.conditional_frame_r(x, n_fft, hop)
    assert r.dtype == ref.dtype and np.array_equal(r.view(np.uint32), ref.view(np.uint32))


def test_select_matches_oracle_levels(an):
    import torch
    from tomatis_audio_processor_amd import dsp
    from tomatis_audio_processor_amd.synth import synth_stream
    x = synth_stream(77, 48000 * 8, 2, 48000)
    n_fft, hop = 2048, 512
    r = orc.conditional_frame_r(x, n_fft, hop)
    lv = orc.r_to_level(r)
    rd = torch.from_numpy(r).cuda()
    cls = (np.arange(len(r)) % 3).astype(np.int8)
    for T in (-60.0, -45.5, -25.0, float(np.median(lv))):
        on_bits, on_exc, off_bits, off_exc = dsp.gate_bits(T, T)
        m, cnt = an._select(rd, on_bits, on_exc, 1)
        assert np.array_equal(m.cpu().numpy().astype(bool), lv >= T) and cnt == int((lv >= T).sum())
        m, cnt = an._select(rd, off_bits, off_exc, 0, torch.from_numpy(cls).cuda(), 2)
        want = (lv > T) & (cls == 2)
        assert np.array_equal(m.cpu().numpy().astype(bool), want) and cnt == int(want.sum())


@pytest.mark.parametrize("F,nb,masked", [(1, 5, False), (2, 65, False), (7, 130, True),
                                         (1000, 1025, True), (5001, 300, False),
                                         (20000, 70, True)])
def test_median_and_mean_bit_exact(an, F, nb, masked):
    import torch
    rng = np.random.default_rng(F * 7 + nb)
    a = (rng.standard_normal((F, nb)) * 30).astype(np.float32)
    a[:, ::7] = np.round(a[:, ::7])          # ties
    a[:, 3 % nb] = -np.abs(a[:, 3 % nb])     # all-negative column
    a[: F // 2 + 1, 4 % nb] = -0.0              # signed zeros
    if F > 1:
        a[F // 2, :] = a[0, :]               # repeated rows
    ad = torch.from_numpy(a).cuda()
    if masked:
        keep = rng.random(F) < 0.6
        keep[0] = True
        mask = torch.from_numpy(keep.astype(np.uint8)).cuda()
        n_sel = int(keep.sum())
        ref = np.median(a[keep], axis=0)
    else:
        mask, n_sel, ref = None, F, np.median(a, axis=0)
    med = an.frame_median(ad, mask, n_sel).cpu().numpy()
    assert np.array_equal(med.view(np.uint32), ref.astype(np.float32).view(np.uint32))
    mean = an.frame_mean(ad).cpu().numpy()
    assert np.array_equal(mean.view(np.uint32), a.mean(axis=0).view(np.uint32))


def test_errors_like_reference(an):
    x = np.zeros((48000, 2), np.float32)
    with pytest.raises(ValueError):
        an.stft_logpower_median(x[:4096 * 5], 48000, 4096, 2048, -65.0)
    with pytest.raises(ValueError, match="50|帧"):
        an.stft_logpower_median(x, 48000, 2048, 512, -65.0)
    with pytest.raises(ValueError):
        an.stft_mag_avg(np.zeros(100, np.float32), 48000, 4096, 2048)


@pytest.mark.parametrize("n_fft,hop", [(3000, 1500), (1000, 250), (16384, 8192), (100, 50)])
def test_band_tilts_any_n_fft(n_fft, hop):
    """calibrate_to_baseline_v2.stft_band_tilt (:17-31) per frame at lengths the
    calibration golden does not use (Bluestein / 16384), against that formula in
    numpy (pocketfft, float32 P, float sums)."""
    import torch
    assert torch.cuda.is_available()
    from tomatis_audio_processor_amd import calibrate_to_baseline_v2 as cal
    from tomatis_audio_processor_amd.synth import synth_stream
    sr = 48000
    x = synth_stream(90 + n_fft, 8 * n_fft + 3 * hop + 5, 2, sr)
    got = cal.band_tilts(x, sr, n_fft, hop)
    F = 1 + (len(x) - n_fft) // hop
    win = np.hanning(n_fft).astype(np.float32)
    freqs = np.fft.rfftfreq(n_fft, 1 / sr)
    lo = (freqs >= 200) & (freqs < 1000)
    hi = (freqs >= 2000) & (freqs < 8000)
    want = []
    for f in range(F):
        X = np.fft.rfft(orc.power_mono(x[f * hop:f * hop + n_fft]) * win)
        P = (X.real * X.real + X.imag * X.imag).astype(np.float32)
        elo, ehi = float(np.sum(P[lo]) + 1e-12), float(np.sum(P[hi]) + 1e-12)
        want.append(10 * np.log10(ehi / elo + 1e-12))
    want = np.asarray(want, np.float32)
    assert got.shape == want.shape
    assert float(np.abs(got - want).max()) < 1e-3


def test_n_fft_bounds(an):
    """Any n_fft np.fft.rfft takes within the LDS: powers of two 16..16384,
    other lengths 16..8192 (Bluestein over >= 2n - 1 points); outside that the
    wrappers refuse before any launch."""
    x = np.zeros((48000, 2), np.float32)
    for bad in (8, 15, 8193, 9000, 32768):
        with pytest.raises(ValueError, match="n_fft"):
            an.stft_mag_avg(x[:, 0], 48000, bad, bad // 2)
    assert an.stft_mag_avg(x[:, 0], 48000, 16, 8).shape == (9,)
    assert an.stft_mag_avg(x[:, 0], 48000, 8191, 4000).shape == (4096,)
