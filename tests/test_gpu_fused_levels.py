"""GPU: in-kernel levels + gate (tomatis_stft_ola_gated, DESIGN.md §5 "Fused
levels") against the two-pass chain (tomatis_levels -> tomatis_gate_std ->
tomatis_stft_ola_limited) and the oracle.

The fused kernel computes every frame's r from the samples it loads for the FFT
(the 16 128-sample leaves of numpy's pairwise sum, src/process_tomatis.py:373-376
via dsp.frame_rms) and steps the gate automaton (:377-385) from the state a
look-back pre-kernel found before its run; r, states, output and chunk peaks
must equal the two-pass chain bit for bit.  A stream whose level hovers inside
the hysteresis band chains its runs' carries (k_gate_chain); only runs that
cannot chain stay unresolved: the pass is flagged (TOMATIS_ERR_GATE_CARRY) and
re-run on the two-pass chain.
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


def _dev_opts(**kw):
    from tomatis_audio_processor_amd._lib import dev_options
    return dev_options(**kw)


def _pair(E, ss, **kw):
    """(gated pipe after run, two-pass y/r/states/peaks)"""
    two = E.GatePipeline(ss, fused_levels=False, **kw)
    two.run()
    assert not two.gated_used
    ref = (two.y.clone(), two.r.clone(), two.states.clone(), two.peaks.clone())
    del two
    pipe = E.GatePipeline(ss, **kw)
    pipe.run()
    return pipe, ref


def _assert_same(torch, pipe, ref):
    y, r, st, pk = ref
    F = pipe.plan.total_frames
    assert torch.equal(pipe.states[:F], st[:F]), "gate states differ"
    assert torch.equal(pipe.r[:F].view(torch.int32), r[:F].view(torch.int32)), "r differs"
    assert torch.equal(pipe.peaks, pk), "chunk peaks differ"
    assert torch.equal(pipe.y, y), "output differs"


@pytest.mark.parametrize("case", [
    # (streams, seconds, ch, sr, hop, up_delay_ms, per-stream input gains)
    ("c2_like", 1, 600, 2, 44100, 512, 250.0, [1.0]),
    ("batch", 6, 45, 2, 48000, 512, 250.0, [1.0, 0.05, 0.3, 1.0, 0.15, 0.6]),
    ("mono_hop256", 3, 40, 1, 44100, 256, 250.0, [1.0, 0.2, 0.02]),
    ("no_delay", 2, 30, 2, 44100, 512, 0.0, [1.0, 0.1]),
    ("long_delay", 1, 60, 2, 22050, 256, 2000.0, [0.7]),
    ("short", 4, 1, 2, 44100, 512, 250.0, [1.0, 0.5, 0.1, 1.0]),
    # near-silent non-zero samples (mean square < 2^-96): the sqrtf branch
    ("tiny", 3, 20, 2, 44100, 512, 250.0, [1e-18, 1.0, 3e-16]),
    ("tiny_mono", 1, 20, 1, 44100, 256, 250.0, [1e-17]),
])
def test_gated_bit_identical(case):
    torch, E = _engine()
    _, ns, secs, ch, sr, hop, ud, gains = case
    n = sr * secs + 391
    ss = E.StreamSet.synthetic(ns, n, ch, sr, seed0=900)
    for i, g in enumerate(gains):
        if g != 1.0:
            o = ss.offs[i]
            ss.x[o:o + n * ch] *= g
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=hop, up_delay_ms=ud)
    assert pipe.gated_used, "an eligible standard-mode plan takes the fused gate"
    assert pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)


def test_gated_digital_silence():
    """Exact zeros (digital silence) inside interior runs, next to loud and
    near-silent stretches: hop blocks of zeros and loud samples take the short
    correctly rounded sqrt, blocks holding a near-silent sample (mean square
    below 2^-96) the scaled form; the approximate look-back decides the loud
    and silent frames and hands near-threshold ones to the exact walk.  All
    must equal the two-pass chain bit for bit."""
    torch, E = _engine()
    sr, n = 44100, 44100 * 30 + 77
    ss = E.StreamSet.synthetic(2, n, 2, sr, seed0=321)
    for i in range(2):
        o = ss.offs[i]
        a, b = o + 2 * (sr * 5 + 100 * (i + 1)), o + 2 * (sr * 9)
        ss.x[a:b] = 0.0                               # silence
        ss.x[b:b + 2 * sr] *= 1e-20                   # near-silent (mean square < 2^-96)
        ss.x[o + 2 * sr * 15:o + 2 * sr * 15 + 2 * 700:7] = 0.0  # scattered zeros in loud audio
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=512)
    assert pipe.gated_used and pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)


def test_gated_ragged():
    """Ragged stream lengths (edge runs, streams shorter than a frame) under
    the fused gate."""
    torch, E = _engine()
    sr = 44100
    xs = [synth_stream(31 + i, n, 2, sr) for i, n in
          enumerate([sr * 70 + 13, 1500, sr * 3 + 1, 2048, sr * 41 + 999])]
    ss = E.StreamSet.from_arrays(xs, sr)
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=512)
    assert pipe.gated_used
    _assert_same(torch, pipe, ref)


def test_gated_vs_oracle():
    torch, E = _engine()
    sr, n = 44100, 44100 * 120 + 333
    x = synth_stream(21, n, 2, sr)
    ss = E.StreamSet.from_arrays([x], sr)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    res = pipe.run()
    assert pipe.gated_used
    ref = orc.process_standard(x, sr, gate_ui=50, n_fft=2048, hop=512)
    assert np.array_equal(res.stream_states(0), ref["states"])
    assert np.array_equal(res.stream_r(0).view(np.uint32),
                          np.asarray(ref["r"], np.float32).view(np.uint32))
    y = res.output(0)
    m = ref["wsum"][ref["pad"]:ref["pad"] + n] >= 1e-3
    ok = np.ones(n, dtype=bool)
    for (a, b), f in zip(res.chunk_ranges(0), res.scale_flags(0)):
        if f:
            ok[a:b] = False
    err = float(np.max(np.abs(y[m & ok] - ref["y"][m & ok])))
    assert err <= 1e-4, err


def _hover(n, sr, T=-40.0):
    """a stereo sine whose level sits at the gate threshold T (gate_ui 50,
    log_percent: inside the +-1.5 dB hysteresis band, neither "on" nor "off")"""
    amp = np.sqrt(2.0) * 10.0 ** (T / 20.0)
    s = (amp * np.sin(2 * np.pi * 1000.0 * np.arange(n) / sr)).astype(np.float32)
    return np.stack([s, s], 1)


def test_gated_chained_hovering_level():
    """A level hovering inside the hysteresis band for ~1400 frames: no run
    after the quiet first frame finds a state-fixing frame, so each run's
    look-back stops at the previous run's first frame and chains (its transfer
    function over the frames between, composed in run order by k_gate_chain).
    No fallback; bit-identical to the two-pass chain; a loud stream in the same
    batch is unaffected."""
    torch, E = _engine()
    sr, hop = 44100, 512
    n = hop * 1400
    ss = E.StreamSet.from_arrays([_hover(n, sr), synth_stream(8, n, 2, sr)], sr)
    with _dev_opts(RUN_FRAMES=48):  # many runs: long chains of chained runs
        pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=hop)
    assert pipe.gated_used and pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)
    st = pipe.result().stream_states(0)
    assert (st == 1).all()  # stays C1 after its quiet start (never D + 1 frames on)


def test_gated_fallback_unchainable():
    """Chaining needs up_delay_frames + 2 <= 1024 transfer-table states; with a
    longer up-delay a hovering stream's runs stay unresolved after 512 frames of
    look-back: the pass is flagged and re-run on the two-pass chain, with the
    two-pass results, and the next run() tries the fused gate again."""
    torch, E = _engine()
    sr, hop = 44100, 256
    n = hop * 2400
    ud = 1100 * hop / sr * 1000.0  # 1100 frames of up-delay
    ss = E.StreamSet.from_arrays([_hover(n, sr), synth_stream(8, n, 2, sr)], sr)
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=hop, up_delay_ms=ud)
    assert pipe.up_delay_frames + 2 > 1024
    assert pipe.gate_fallbacks == 1, "the unresolved carry must re-run the pass"
    assert not pipe.gated_used
    _assert_same(torch, pipe, ref)
    pipe.run()
    assert pipe.gate_fallbacks == 2
    _assert_same(torch, pipe, ref)


def test_gated_hovering_stream_in_c4_batch():
    """BASELINE C4 as benched per GPU (64 x 5 min stereo 48 kHz) with one stream
    hovering at the threshold for all 5 minutes: every run of it chains, the
    pass takes the fused gate (no fallback), equals the two-pass chain bit for
    bit, and costs about what a clean batch does."""
    torch, E = _engine()
    sr = 48000
    n = 300 * sr
    ss = E.StreamSet.synthetic(64, n, 2, sr, seed0=1000)
    clean = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)

    def timed(pipe, k=4):
        pipe.run()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(k):
            pipe.run(check_device=False)
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / k

    t_clean = timed(clean)
    del clean
    o = ss.offs[17]
    ss.x[o:o + 2 * n] = torch.from_numpy(_hover(n, sr).reshape(-1)).to(ss.x.device)
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=512)
    assert pipe.gated_used and pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)
    t_hover = timed(pipe)
    assert pipe.gate_fallbacks == 0
    # (the look-back of the hovering stream's runs walks their whole span once;
    # a whole-batch two-pass re-run would double the pass)
    assert t_hover <= 1.3 * t_clean, (t_hover, t_clean)


def test_gated_declines_other_shapes():
    """Shapes outside the fused gate (n_fft 4096 unless TOMATIS_DEV_FUSED_4096,
    n_fft 2048 with hop 1024, cross-fade at 2048) run two passes."""
    torch, E = _engine()
    sr, n = 44100, 44100 * 20
    ss = E.StreamSet.synthetic(1, n, 2, sr, seed0=5)
    for kw in (dict(n_fft=4096, hop=1024), dict(n_fft=4096, hop=1024, xfade_ms=500.0),
               dict(n_fft=4096, hop=2048), dict(n_fft=2048, hop=1024),
               dict(n_fft=2048, hop=512, xfade_ms=500.0)):
        pipe = E.GatePipeline(ss, gate_ui=50, **kw)
        pipe.run()
        assert not pipe.gated_used, kw


def test_gated_full_size_c2():
    """BASELINE C2 (60 min stereo 44.1 kHz, 2048/512): the bench's fused pass
    equals the two-pass chain bit for bit."""
    torch, E = _engine()
    sr = 44100
    n = 3600 * sr
    ss = E.StreamSet.synthetic(1, n, 2, sr, seed0=1000)
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=512)
    assert pipe.gated_used and pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)


def test_gated_full_size_c4():
    """BASELINE C4 as benched per GPU (64 x 5 min stereo 48 kHz, seeds as
    bench.py): the fused pass equals the two-pass chain bit for bit on every
    stream (r, states, chunk peaks, output)."""
    torch, E = _engine()
    sr = 48000
    n = 300 * sr
    ss = E.StreamSet.synthetic(64, n, 2, sr, seed0=1000)
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=512)
    assert pipe.gated_used and pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)


def test_gated_level_sweeps_through_thresholds():
    """Levels that sweep through the hysteresis band with short plateaus at
    each threshold (quiet -> up through both thresholds -> loud -> down, three
    times): the plateau frames sit within 0.1 % of a threshold, where the
    approximate look-back declines and the exact walk takes over; every run
    still resolves, and the fused pass equals the two-pass chain bit for bit."""
    torch, E = _engine()
    sr, hop = 44100, 512
    probe = E.GatePipeline(E.StreamSet.synthetic(1, sr, 2, sr, seed0=1), gate_ui=50,
                           n_fft=2048, hop=hop)
    ton, toff = probe.Ton, probe.Toff   # level thresholds (dB) of this gate setting
    del probe
    segs = []
    for _ in range(3):
        # plateaus at each threshold (0.25 s, fewer than up-delay + 1 frames)
        for secs, d0, d1 in ((1.0, -60, -60), (1.0, -47, toff), (0.25, toff, toff),
                             (0.5, toff, ton), (0.25, ton, ton), (1.0, ton, -33),
                             (3.0, -20, -20), (2.0, -35, -45)):
            m = int(secs * sr)
            segs.append(np.linspace(d0, d1, m))
    db = np.concatenate(segs)
    t = np.arange(len(db)) / sr
    s = (np.sqrt(2.0) * 10.0 ** (db / 20.0) * np.sin(2 * np.pi * 1000.0 * t)).astype(np.float32)
    x = np.stack([s, s], 1)
    ss = E.StreamSet.from_arrays([x, synth_stream(12, len(s), 2, sr)], sr)
    pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=hop)
    assert pipe.gated_used and pipe.gate_fallbacks == 0
    _assert_same(torch, pipe, ref)


@pytest.mark.parametrize("opts", [
    # 8 x 5 min 48 kHz on 64 run slots: 56 interior slots want ~4000-frame runs;
    # more than 4096 frames per slot would break the chain, so the plan cuts
    # two rounds of runs
    dict(SLOTS=64),
    # an explicit 8192-frame request is capped at 4096 all the same
    dict(SLOTS=64, RUN_FRAMES=8192),
    # the same with a single run slot per stream's worth: many rounds
    dict(SLOTS=16),
])
def test_gated_hovering_long_runs(opts):
    """A batch whose frames exceed slots x 4096 (SURVEY C4's 512 streams on one
    GPU are 14.4 M frames on 2048 slots; TOMATIS_DEV_SLOTS reproduces the ratio
    on 8 streams) with one stream hovering at the threshold for all 5 minutes:
    runs stay within the chained look-back (tm_kernels.hip build_runs), the pass
    takes the fused gate with no two-pass fallback, bit-identical to the
    two-pass chain (src/process_tomatis.py:373-385 has no look-back horizon)."""
    torch, E = _engine()
    sr = 48000
    n = 300 * sr
    with _dev_opts(**opts):
        ss = E.StreamSet.synthetic(8, n, 2, sr, seed0=1000)
        o = ss.offs[3]
        ss.x[o:o + 2 * n] = torch.from_numpy(_hover(n, sr).reshape(-1)).to(ss.x.device)
        pipe, ref = _pair(E, ss, gate_ui=50, n_fft=2048, hop=512)
        assert pipe.gated_used and pipe.gate_fallbacks == 0, opts
        _assert_same(torch, pipe, ref)
        # pipelined passes of the same long-run plan: no fallback either
        pp = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512, pipelined=True)
        pp.run()
        pp.run()
        res = pp.result()
        assert pp.gate_fallbacks == 0
        assert torch.equal(res.y, ref[0]) and torch.equal(res.chunk_peaks, ref[3])
