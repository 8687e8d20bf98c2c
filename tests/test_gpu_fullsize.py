"""Full-size (BASELINE.json config) properties on the GPU, checked without
running the whole oracle on 60-min streams:

* the gate TF-scan states equal the reference automaton re-run on the host
  over the GPU's own frame r (levels via numpy log10, exactly as the reference);
* randomly sampled interior hop blocks equal the oracle's spectral filter +
  OLA of the 4 covering frames, given the GPU's states (tolerance 1e-4);
* every limiter chunk's output peak is <= 0.999 (+1 ulp), and chunks the
  kernel reported above 0.999 peak at 0.999 after the fix-up;
* the synthetic input equals the host generator on sampled windows;
* an all-0-dB tilt reproduces the input in the interior (identity round trip).
"""
import numpy as np
import pytest

from oracle import tomatis_oracle as orc
from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine
    return torch, engine


@pytest.mark.parametrize("secs,sr,n_fft,hop", [(3600, 44100, 2048, 512),   # C2
                                               (300, 96000, 4096, 1024)])   # C5 stage shape
def test_fullsize_standard(secs, sr, n_fft, hop):
    torch, E = _engine()
    n = secs * sr
    ss = E.StreamSet.synthetic(1, n, 2, sr, seed0=1000)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=n_fft, hop=hop)
    res = pipe.run()
    torch.cuda.synchronize()
    pipe.plan.check_device()  # fused-limiter waits all completed
    rng = np.random.default_rng(secs)
    # input generator parity on sampled windows
    for a in rng.integers(0, n - 4096, 4):
        a = int(a)
        dev = ss.x[2 * a:2 * (a + 4096)].cpu().numpy().reshape(-1, 2)
        assert np.array_equal(dev, synth_stream(1000, 4096, 2, sr, start=a))
    # gate states vs the reference automaton over the GPU r
    r = res.stream_r(0)
    levels = orc.r_to_level(r)
    starts = res.first_start[0] + hop * np.arange(len(r), dtype=np.int64)
    st_ref = orc.gate_standard(levels, starts, pipe.Ton, pipe.Toff, pipe.up_delay_samples)
    st = res.stream_states(0)
    assert np.array_equal(st, st_ref)
    # sampled interior blocks vs oracle frames (before the limiter scale)
    peaks = res.stream_peaks(0)
    bounds = res.extra["bounds"][0]
    win, win2 = orc.hann_sym(n_fft)
    g = [pipe.gains[0].cpu().numpy()[:n_fft // 2 + 1], pipe.gains[1].cpu().numpy()[:n_fft // 2 + 1]]
    y_all = None
    R = n_fft // hop
    for k in rng.integers(R, len(r) - R, 6):
        k = int(k)
        s_k = int(starts[k])
        if s_k < 0 or s_k + hop > n:
            continue
        frames_k = list(range(k - R + 1, k + 1))
        lo = int(starts[frames_k[0]])
        xw = synth_stream(1000, n_fft + (R - 1) * hop, 2, sr, start=lo) if lo >= 0 else None
        if xw is None:
            continue
        fr = orc.frame_view(xw, n_fft, hop, R)
        gains = np.stack([g[0] if st[j] == 1 else g[1] for j in frames_k]).astype(np.float32)
        yk = orc.spectral_filter(fr, win, gains)
        out = np.zeros((hop, 2), np.float32)
        w = np.zeros(hop, np.float32)
        for q, j in enumerate(frames_k):
            off = s_k - int(starts[j])
            out += yk[q, off:off + hop]
            w += win2[off:off + hop]
        ref = out / (w[:, None] + np.float32(1e-12))
        c = sum(1 for b in bounds[1:-1] if b <= s_k)
        sc = np.float32(0.999) / peaks[c] if peaks[c] > 0.999 else np.float32(1.0)
        got = res.y[2 * s_k:2 * (s_k + hop)].cpu().numpy().reshape(-1, 2)
        assert np.max(np.abs(got - ref * sc)) <= 1e-4
    # limiter property on every chunk
    y = res.y[:2 * n].cpu().numpy().reshape(-1, 2)
    for c, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        a, b = max(0, a), min(n, b)
        if b <= a:
            continue
        pk = float(np.max(np.abs(y[a:b])))
        assert pk <= 0.999 * (1 + 2e-7)
        if peaks[c] > 0.999:
            assert pk >= 0.999 * (1 - 1e-6)


def test_identity_round_trip_fullsize():
    """0 dB gains: framing/window/FFT/IFFT/OLA/normalise is the identity in the interior."""
    torch, E = _engine()
    sr, n = 48000, 48000 * 300
    ss = E.StreamSet.synthetic(2, n, 2, sr, seed0=77)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512, c1_low=0.0, c1_high=0.0,
                          c2_low=0.0, c2_high=0.0)
    res = pipe.run()
    torch.cuda.synchronize()
    for i in range(2):
        y = res.output(i)
        x = ss.x[ss.offs[i]:ss.offs[i] + 2 * n].cpu().numpy().reshape(-1, 2)
        sl = slice(4096, n - 4096)
        assert np.max(np.abs(y[sl] - x[sl])) <= 2e-6
