"""GPU parity of the any-size transform path beyond the reference goldens.

The goldens pin the oracle at n_fft 3000/750 (Bluestein, M = 8192 in LDS),
2400/600 xfade, 1999/500 adaptive, 16384/4096 (LDS, M = 16384) and 10 channels
(tests/golden/cases.py).  Here the HIP path is checked against that oracle on
the shapes the goldens do not reach: Bluestein and power-of-two lengths whose
FFT exceeds the LDS (per-block HBM buffers, M = 32768 / 65536), tiny frames
(n_fft 3, 16, 100) and 16 channels.  Same contract as test_gpu_parity: r and
states bit-exact, samples within 1e-4 where sum w^2 >= 1e-3.
Reference: src/process_tomatis.py:394-406 (np.fft.rfft / irfft of any length),
src/process_tomatis_adaptive.py:179-183 (no channel guard).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import _check_chunks, _engine, TAU

pytestmark = pytest.mark.gpu


def _run(mode, x, sr, **p):
    torch, E = _engine()
    from oracle import tomatis_oracle as orc
    ss = E.StreamSet.from_arrays([x], sr)
    if mode == "standard":
        pipe = E.GatePipeline(ss, **p)
        ref = orc.process_standard(x, sr, **p)
    else:
        pipe = E.AdaptivePipeline(ss, **p)
        ref = orc.process_adaptive(x, sr, **p)
    res = pipe.run()
    torch.cuda.synchronize()
    return res, ref


@pytest.mark.parametrize("n_fft,hop,secs", [
    (12000, 3000, 3.0),    # Bluestein, M = 32768: HBM buffers
    (32768, 8192, 4.0),    # power of two above the LDS: HBM buffers
    (40000, 10000, 4.0),   # Bluestein, M = 131072: the largest HBM buffers
    (65536, 16384, 4.0),   # kMaxNfft, power of two
    (100, 25, 0.5),        # Bluestein in LDS, M = 256
    (16, 4, 0.1),
    (3, 1, 0.02),
])
def test_standard_any_n_fft(n_fft, hop, secs):
    from tomatis_audio_processor_amd.synth import synth_stream
    sr = 48000
    N = int(sr * secs) + n_fft + 17
    x = synth_stream(600 + n_fft, N, 2, sr)
    res, ref = _run("standard", x, sr, gate_ui=50, n_fft=n_fft, hop=hop)
    r = res.stream_r(0)
    np.testing.assert_array_equal(r.view(np.uint32), ref["r"].view(np.uint32))
    np.testing.assert_array_equal(res.stream_states(0), ref["states"])
    y = res.output(0)
    yr = np.asarray(ref["y"], np.float64)
    assert y.shape == yr.shape
    m = ref["wsum"][ref["pad"]:ref["pad"] + N] >= TAU
    _check_chunks(res, ref, y, yr, m, "standard")


@pytest.mark.parametrize("ch,n_fft,hop", [(16, 2048, 512), (9, 1500, 375), (3, 4096, 1024)])
def test_adaptive_many_channels(ch, n_fft, hop):
    from tomatis_audio_processor_amd.synth import synth_stream
    sr = 48000
    N = sr * 3 + 101
    x = synth_stream(700 + ch, N, ch, sr)
    res, ref = _run("adaptive", x, sr, n_fft=n_fft, hop=hop)
    np.testing.assert_array_equal(res.stream_states(0), ref["states"])
    np.testing.assert_array_equal(res.stream_alpha(0), ref["alpha"])
    assert float(res.extra["thresholds"].cpu().numpy()[0]) == ref["threshold"]
    y = res.output(0)
    yr = np.asarray(ref["y"], np.float64)
    assert y.shape == yr.shape
    _check_chunks(res, ref, y, yr, ref["wsum"] >= TAU, "adaptive")


def test_adaptive_quiet_f64_8192():
    """float64 levels at n_fft 8192: a frame larger than the f64 level block's
    LDS takes the pairwise-program kernel (k_levels_any<double>)."""
    from tomatis_audio_processor_amd.synth import synth_stream
    sr = 48000
    N = sr * 4 + 11
    x = (synth_stream(811, N, 2, sr) * np.float32(0.01)).astype(np.float32)
    res, ref = _run("adaptive", x, sr, n_fft=8192, hop=2048)
    np.testing.assert_array_equal(res.stream_states(0), ref["states"])
    assert float(res.extra["thresholds"].cpu().numpy()[0]) == ref["threshold"]


@pytest.mark.parametrize("secs,n_fft,hop", [(120, 2048, 512), (300, 2048, 512), (60, 4096, 2048)])
def test_adaptive_quiet_long_stream(secs, n_fft, hop):
    """Quiet input takes the reference's float64 pipeline (SURVEY F6,
    src/process_tomatis_adaptive.py:201-215): levels, threshold, states and
    alpha run in float64 here too (bit-exact); the spectral path runs in
    float32.  Bounds that deviation on long streams against the oracle's
    float64 spectral path: within 1e-4 where sum w^2 >= 1e-3 (and reports the
    measured maximum)."""
    from tomatis_audio_processor_amd.synth import synth_stream
    sr = 44100
    N = sr * secs + 77
    x = (synth_stream(1200 + secs, N, 2, sr) * np.float32(0.01)).astype(np.float32)
    res, ref = _run("adaptive", x, sr, n_fft=n_fft, hop=hop)
    assert res.extra["atten_db"][0] == 0  # the float64 pipeline (F64 levels)
    np.testing.assert_array_equal(res.stream_states(0), ref["states"])
    np.testing.assert_array_equal(res.stream_alpha(0), ref["alpha"])
    assert float(res.extra["thresholds"].cpu().numpy()[0]) == ref["threshold"]
    y = res.output(0)
    yr = np.asarray(ref["y"], np.float64)
    m = ref["wsum"] >= TAU
    err = float(np.max(np.abs(y[m] - yr[m])))
    print(f"quiet {secs} s {n_fft}/{hop}: max |f32 - f64 oracle| = {err:.2e}, "
          f"peak {float(np.max(np.abs(yr))):.3f}")
    assert ref["scale"] is None  # quiet: the limiter stays off
    assert err <= 1e-4
