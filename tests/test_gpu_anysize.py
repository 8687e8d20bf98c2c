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


@pytest.mark.parametrize("hop,ch,mode", [(1024, 2, "standard"), (2048, 2, "standard"),
                                         (1024, 2, "xfade"), (2048, 1, "adaptive"),
                                         (512, 2, "standard")])
def test_half_frames_4096(hop, ch, mode, monkeypatch):
    """n_fft 4096 as two P = 64 waves per frame (sample parities, one spectral
    exchange; tm_transform.hip H) against the oracle and against the two-wave
    P = 128 kernel (TOMATIS_HALF4096=0) on 4 streams with many limiter chunks.
    Reference: src/process_tomatis.py:394-406 (4096/2048 is its default)."""
    torch, E = _engine()
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd.synth import synth_stream
    sr = 48000
    lens = [sr * 12 + 333, sr * 5, sr * 9 + 4096 + 7, sr * 3]
    xs = [synth_stream(900 + i, n, ch, sr) for i, n in enumerate(lens)]
    kw = dict(n_fft=4096, hop=hop)
    outs = []
    for half in ("1", "0"):
        monkeypatch.setenv("TOMATIS_HALF4096", half)
        ss = E.StreamSet.from_arrays(xs, sr)
        if mode == "adaptive":
            pipe = E.AdaptivePipeline(ss, **kw)
        else:
            pipe = E.GatePipeline(ss, gate_ui=50, **kw, **({"xfade_ms": 300.0} if mode == "xfade" else {}))
        res = pipe.run()
        torch.cuda.synchronize()
        outs.append(res)
    r1, r0 = outs
    for i, (x, n) in enumerate(zip(xs, lens)):
        y1, y0 = r1.output(i), r0.output(i)
        # the two kernels differ only by float rounding of the transform
        assert np.max(np.abs(y1 - y0)) <= 2e-5 * max(1.0, float(np.max(np.abs(y0))))
        if i < 2:  # and against the oracle
            if mode == "adaptive":
                ref = orc.process_adaptive(x, sr, **kw)
                mk = ref["wsum"] >= TAU
                np.testing.assert_array_equal(r1.stream_states(i), ref["states"])
            else:
                ref = orc.process_standard(x, sr, gate_ui=50, **kw,
                                           **({"xfade_ms": 300.0} if mode == "xfade" else {}))
                mk = ref["wsum"][ref["pad"]:ref["pad"] + n] >= TAU
                np.testing.assert_array_equal(r1.stream_states(i), ref["states"])
            _check_chunks_stream(r1, i, ref, y1, mk, mode)


def _check_chunks_stream(res, i, ref, y, m, mode):
    """test_gpu_parity._check_chunks for stream i of a multi-stream result."""
    from tomatis_audio_processor_amd import conditioning
    from tests.test_gpu_parity import _scale_of, TOL
    flags = res.scale_flags(i)
    ranges = res.chunk_ranges(i)
    peaks = res.stream_peaks(i)
    yr = np.asarray(ref["y"], np.float64)
    ref_scales = ref["scales"] if mode != "adaptive" else [ref["scale"] or 1.0]
    assert len(ranges) == len(ref_scales)
    for c, (a, b) in enumerate(ranges):
        if b <= a:
            continue
        gs, rs = _scale_of(peaks[c]), float(ref_scales[c] or 1.0)
        mm = m[a:b]
        if abs(gs / rs - 1.0) > conditioning.ETA:
            assert flags[c]
        err = (np.abs(y[a:b][mm] - yr[a:b][mm]) if not flags[c]
               else np.abs(y[a:b][mm] / gs - yr[a:b][mm] / rs) * min(gs, rs))
        assert float(err.max(initial=0.0)) <= TOL, f"chunk {c}: {err.max()}"
