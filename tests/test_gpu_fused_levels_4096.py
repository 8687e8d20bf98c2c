"""GPU: in-kernel levels + gate + cross-fade alpha at n_fft 4096 / hop 1024
(tomatis_stft_ola_gated on two-wave frames, DESIGN.md §5 "Fused levels at
4096"; opt-in through TOMATIS_DEV_FUSED_4096, as it measured slower than the
two-pass chain) against the two-pass chain (tomatis_levels -> tomatis_gate_std
with alpha -> tomatis_stft_ola_limited).

A frame's 32 leaves are 128-sample registers across both waves of the
sequence: each wave writes the m^2 of its half of the new hop block to LDS,
the forward FFT's pair barrier orders both halves, and both waves sum numpy's
8 chains of 16 per leaf in order, the 32-leaf perfect tree, r, the gate step
and (cross-fade) the float64 alpha step of src/process_tomatis_xfade.py:
237-278.  Each run starts from k_gate_carry's state and alpha (a run of
xf + 2 equal states pins alpha).  r, states, alpha, output and chunk peaks
must equal the two-pass chain bit for bit; a run whose look-back does not
resolve re-runs the pass on the two-pass chain (same results).
"""
import numpy as np
import pytest

from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_4096():
    """the path is opt-in (measured slower than the two-pass chain)"""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd._lib import set_dev_option
    set_dev_option("FUSED_4096", 1)
    yield
    set_dev_option("FUSED_4096", -1)


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine
    return torch, engine


def _scale(ss, gains, n, ch):
    for i, g in enumerate(gains):
        if g != 1.0:
            o = ss.offs[i]
            ss.x[o:o + n * ch] *= g


def _pair(E, ss, **kw):
    """(gated pipe after run, two-pass y / r / states / peaks / alpha)"""
    two = E.GatePipeline(ss, fused_levels=False, **kw)
    two.run()
    assert not two.gated_used
    ref = (two.y.clone(), two.r.clone(), two.states.clone(), two.peaks.clone(),
           two.alpha.clone() if two.alpha is not None else None)
    del two
    pipe = E.GatePipeline(ss, **kw)
    pipe.run()
    return pipe, ref


def _assert_same(torch, pipe, ref, y=None, peaks=None, r=None, states=None, alpha=None):
    ry, rr, rst, rpk, ral = ref
    F = pipe.plan.total_frames
    st = pipe.states if states is None else states
    assert torch.equal(st[:F], rst[:F]), "gate states differ"
    rv = pipe.r if r is None else r
    assert torch.equal(rv[:F].view(torch.int32), rr[:F].view(torch.int32)), "r differs"
    if ral is not None:
        al = pipe.alpha if alpha is None else alpha
        assert torch.equal(al[:F], ral[:F]), "alpha differs"
    assert torch.equal(pipe.peaks if peaks is None else peaks, rpk), "chunk peaks differ"
    assert torch.equal(pipe.y if y is None else y, ry), "output differs"


@pytest.mark.parametrize("case", [
    # (name, streams, seconds, ch, sr, xfade_ms (None: standard), up_delay_ms, gains)
    ("c5x_like", 4, 40, 2, 96000, 500.0, 250.0, [1.0, 0.3, 1.0, 0.05]),
    ("xfade_48k", 3, 30, 2, 48000, 500.0, 250.0, [1.0, 0.2, 0.6]),
    ("xfade_mono", 2, 30, 1, 96000, 500.0, 250.0, [1.0, 0.1]),
    ("xfade_0ms", 2, 20, 2, 48000, 0.0, 250.0, [1.0, 0.4]),
    # 5 s cross-fade: xf + 2 = 218 equal states, longer than any of this signal's
    # state runs, pin alpha only from the stream start -- the later runs' look-backs
    # do not resolve and the pass re-runs on the two-pass chain (checked below)
    ("xfade_long", 1, 60, 2, 44100, 5000.0, 250.0, [0.8]),
    ("xfade_no_delay", 2, 20, 2, 96000, 300.0, 0.0, [1.0, 0.15]),
    ("standard", 3, 30, 2, 96000, None, 250.0, [1.0, 0.25, 0.05]),
    ("short", 4, 1, 2, 48000, 500.0, 250.0, [1.0, 0.5, 0.1, 1.0]),
    ("tiny", 2, 10, 2, 96000, 500.0, 250.0, [1e-18, 1.0]),
])
def test_gated4096_bit_identical(case):
    torch, E = _engine()
    _, ns, secs, ch, sr, xms, ud, gains = case
    n = sr * secs + 517
    ss = E.StreamSet.synthetic(ns, n, ch, sr, seed0=910)
    _scale(ss, gains, n, ch)
    kw = dict(gate_ui=50, gate_offset=-90, n_fft=4096, hop=1024, up_delay_ms=ud)
    if xms is not None:
        kw["xfade_ms"] = xms
    pipe, ref = _pair(E, ss, **kw)
    if case[0] == "xfade_long":
        assert pipe.gate_fallbacks == 1 and not pipe.gated_used
    else:
        assert pipe.gated_used, "an eligible 4096 / 1024 plan takes the fused gate"
        assert pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)


def test_gated4096_ragged():
    """Ragged lengths (edge runs, a stream shorter than a frame) under the
    fused cross-fade gate."""
    torch, E = _engine()
    sr = 96000
    xs = [synth_stream(41 + i, n, 2, sr) for i, n in
          enumerate([sr * 50 + 13, 3000, sr * 3 + 1, 4096, sr * 21 + 999])]
    ss = E.StreamSet.from_arrays(xs, sr)
    pipe, ref = _pair(E, ss, gate_ui=50, gate_offset=-90, n_fft=4096, hop=1024, xfade_ms=500.0)
    assert pipe.gated_used
    _assert_same(torch, pipe, ref)


def _hover(n, sr, T=-40.0):
    t = np.arange(n) / sr
    s = (np.sqrt(2.0) * 10.0 ** (T / 20.0) * np.sin(2 * np.pi * 1000.0 * t)).astype(np.float32)
    return np.stack([s, s], 1)


def _flicker(seed, n, sr, on_s, off_s):
    """synthetic audio switched between full level and -40 dB"""
    t = np.arange(n) / sr
    env = np.where((t % (on_s + off_s)) < on_s, 1.0, 0.01).astype(np.float32)
    return synth_stream(seed, n, 2, sr) * env[:, None]


def test_gated4096_no_alpha_pin():
    """A stream at the threshold for minutes (the look-back finds no anchor)
    and one whose state alternates faster than the cross-fade settles (on
    0.53 s, off 0.21 s at 96 kHz / 1024: C2 and C1 stretches both shorter
    than xf + 2 = 49 frames, so no run of equal states pins alpha): the
    look-backs do not resolve and the pass re-runs on the two-pass chain --
    results bit-identical either way."""
    torch, E = _engine()
    sr, n = 96000, 96000 * 40
    ss = E.StreamSet.from_arrays([synth_stream(76, n, 2, sr), _flicker(77, n, sr, 0.533, 0.213),
                                  _hover(n, sr)], sr)
    pipe, ref = _pair(E, ss, gate_ui=50, gate_offset=-90, n_fft=4096, hop=1024, xfade_ms=500.0)
    _assert_same(torch, pipe, ref)


def test_gated4096_switching_streams():
    """Streams switching between C1 and C2 every 1.5 s / 2.3 s: every run's
    look-back finds a run of equal states before it (alpha pinned) -- no
    fallback, bit-identical alpha through the cross-fades."""
    torch, E = _engine()
    sr, n = 96000, 96000 * 60
    ss = E.StreamSet.from_arrays([_flicker(78, n, sr, 1.5, 1.5), _flicker(79, n, sr, 2.3, 0.9),
                                  synth_stream(80, n, 2, sr)], sr)
    pipe, ref = _pair(E, ss, gate_ui=50, gate_offset=-90, n_fft=4096, hop=1024, xfade_ms=500.0)
    assert pipe.gated_used and pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)


def test_gated4096_pipelined():
    """Pipelined passes (tomatis_stft_ola_gated_pipelined at 4096: the partner
    blocks through VGPRs next to the in-kernel gate) over distinct inputs,
    queued without host synchronisation: every pass equals an unpipelined
    two-pass pass bit for bit."""
    torch, E = _engine()
    sr, ns = 96000, 4
    n = sr * 30 + 99
    xs = []
    for k in range(3):
        s = E.StreamSet.synthetic(ns, n, 2, sr, seed0=500 + 17 * k)
        _scale(s, [1.0, 0.3 * (k + 1), 1.0, 0.05], n, 2)
        xs.append(s.x.clone())
    ss = E.StreamSet(x=xs[0].clone(), offs=[i * n * 2 for i in range(ns)], lens=[n] * ns,
                     ch=2, sr=sr)
    kw = dict(gate_ui=50, gate_offset=-90, n_fft=4096, hop=1024, xfade_ms=500.0)
    two = E.GatePipeline(ss, fused_levels=False, **kw)
    refs = []
    for x in xs:
        ss.x.copy_(x)
        two.run()
        refs.append((two.y.clone(), two.r.clone(), two.states.clone(), two.peaks.clone(),
                     two.alpha.clone()))
    del two
    pipe = E.GatePipeline(ss, pipelined=True, **kw)
    got, cur = [], None
    for x in xs:
        ss.x.copy_(x)
        assert pipe.run(check_device=False) is None and pipe.pending and pipe.gated_used
        if cur is not None:
            got.append((cur[0].clone(), cur[1].clone()) + cur[2:])
        cur = (pipe.y, pipe.peaks, pipe.r.clone(), pipe.states.clone(), pipe.alpha.clone())
    res = pipe.result()
    got.append((res.y, res.chunk_peaks) + cur[2:])
    assert pipe.finish() == 0 and pipe.gate_fallbacks == 0
    for k, (y, pk, r, st, al) in enumerate(got):
        _assert_same(torch, pipe, refs[k], y=y, peaks=pk, r=r, states=st, alpha=al)
