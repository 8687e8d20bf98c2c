"""GPU: the two-round fused limiter (TOMATIS_OPT_LIMITER_ROUNDS, DESIGN.md §6
"Limiter rounds") against the one-round layout and the oracle.

Round 1 leaves its output unscaled; k_r2_plan lists, per round-2 run, the
round-1 hop blocks of chunks that round 1 completed; round 2 scales them inside
its frame loop (LDS-DMA staging) and the rest in its tail.  Every frame is
computed by the same instructions in either layout (3 warm-up frames rebuild
the OLA accumulator exactly), and a chunk's scale is the same float32
limit / peak, so the two layouts must agree bit for bit -- on streams where
every chunk is limited, none is, or some are, and on stream batches, mono,
hop 256 (hop 1024 stays one round) and time shards.  One configuration is also checked against the
oracle (reference: src/process_tomatis.py:331-357, the per-chunk limiter).
"""
import numpy as np
import pytest

from oracle import tomatis_oracle as orc
from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu
LIM = 0.999


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine
    return torch, engine


def _scaled(E, torch, n_streams, n, ch, sr, gains, seed0):
    ss = E.StreamSet.synthetic(n_streams, n, ch, sr, seed0=seed0)
    for i, g in enumerate(gains):
        if g != 1.0:
            o = ss.offs[i]
            ss.x[o:o + n * ch] *= g
    return ss


def _both(E, torch, ss, **kw):
    pipe = E.GatePipeline(ss, gate_ui=50, **kw)
    pipe.plan.set_limiter_rounds(2)
    rounds = pipe.plan.limiter_rounds
    pipe.run()
    y2 = pipe.y.clone()
    pk2 = pipe.peaks.clone()
    assert pipe.plan.error_bits() == 0
    pipe.plan.set_limiter_rounds(1)
    assert pipe.plan.limiter_rounds == 1
    pipe.run()
    assert pipe.plan.error_bits() == 0
    pipe.plan.set_limiter_rounds(0)
    return rounds, y2, pk2, pipe


@pytest.mark.parametrize("case", [
    # (streams, seconds, ch, sr, n_fft, hop, per-stream input gains)
    ("c2_like", 1, 720, 2, 44100, 2048, 512, [1.0]),
    ("quiet", 1, 300, 2, 44100, 2048, 512, [0.05]),
    ("batch_mixed", 6, 90, 2, 48000, 2048, 512, [1.0, 0.05, 0.3, 1.0, 0.15, 0.6]),
    ("mono_hop256", 2, 150, 1, 44100, 2048, 256, [1.0, 0.2]),
    ("hop1024", 1, 240, 2, 44100, 2048, 1024, [1.0]),
])
def test_two_rounds_bit_identical(case):
    torch, E = _engine()
    _, ns, secs, ch, sr, n_fft, hop, gains = case
    n = sr * secs + 77
    ss = _scaled(E, torch, ns, n, ch, sr, gains, seed0=400)
    rounds, y2, pk2, pipe = _both(E, torch, ss, n_fft=n_fft, hop=hop)
    # hop <= 512 only: round 2's per-sequence LDS slot of a hop block beside the
    # single-exchange FFT's exchange rows (tm_kernels.hip build_runs)
    expect = 2 if hop <= 512 else 1
    assert rounds == expect, "an eligible standard-mode plan takes two rounds when asked"
    assert torch.equal(pipe.peaks, pk2)
    assert torch.equal(pipe.y, y2), "two-round output differs from one round"
    # the limiter property on every stream: chunks over the limit end at it
    res = pipe.result()
    for i in range(ns):
        y = res.output(i)
        for (a, b), pk in zip(res.chunk_ranges(i), res.stream_peaks(i)):
            if b > a and pk > LIM:
                m = float(np.max(np.abs(y[a:b])))
                assert abs(m - LIM) <= 2e-6, (i, a, b, m)


def test_two_rounds_vs_oracle():
    torch, E = _engine()
    sr, n = 44100, 44100 * 150 + 333
    x = synth_stream(21, n, 2, sr)
    ss = E.StreamSet.from_arrays([x], sr)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    pipe.plan.set_limiter_rounds(2)
    assert pipe.plan.limiter_rounds == 2
    res = pipe.run()
    assert pipe.plan.error_bits() == 0
    ref = orc.process_standard(x, sr, gate_ui=50, n_fft=2048, hop=512)
    assert np.array_equal(res.stream_states(0), ref["states"])
    y = res.output(0)
    m = ref["wsum"][ref["pad"]:ref["pad"] + n] >= 1e-3
    flags = res.scale_flags(0)
    ok = np.ones(n, dtype=bool)
    for (a, b), f in zip(res.chunk_ranges(0), flags):
        if f:
            ok[a:b] = False
    err = float(np.max(np.abs(y[m & ok] - ref["y"][m & ok])))
    assert err <= 1e-4, err


def test_two_rounds_fault_recovery():
    """Round 2's tail waits (chunks that straddle the rounds, its own chunks):
    a forced wait timeout still reaches finish_plan's unfused re-run."""
    torch, E = _engine()
    sr, n = 44100, 44100 * 120 + 5
    ss = E.StreamSet.synthetic(1, n, 2, sr, seed0=77)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    pipe.plan.set_limiter_rounds(2)
    assert pipe.plan.limiter_rounds == 2
    pipe.run()
    y0 = pipe.y.clone()
    pipe.plan.set_limiter_spin(0)
    try:
        with pytest.warns(RuntimeWarning, match="fused limiter wait timed out"):
            pipe.run()
    finally:
        pipe.plan.set_limiter_spin(1 << 18)
    assert torch.equal(pipe.y, y0)


def test_two_rounds_timeshard_edges():
    """Time shards leave their edge chunks to the peak exchange: the round-2
    plan stops at them and the tails skip them.  Shards (two rounds each, a
    process-wide dev override) vs the unsharded stream in one round:
    bit-identical."""
    torch, E = _engine()
    from tomatis_audio_processor_amd import timeshard as TS
    sr, n = 44100, 44100 * 240 + 11
    x = synth_stream(5, n, 2, sr)
    params = dict(gate_ui=50, n_fft=2048, hop=512)
    pipe = E.GatePipeline(E.StreamSet.from_arrays([x], sr), **params)
    pipe.plan.set_limiter_rounds(1)
    res = pipe.run()
    from tomatis_audio_processor_amd._lib import dev_options
    with dev_options(LIMITER_ROUNDS=2):
        y, st, pk = TS.run_emulated(x, sr, 3, **params)
    assert np.array_equal(st, res.stream_states(0))
    assert pk.tobytes() == res.stream_peaks(0).tobytes()
    assert y.tobytes() == res.output(0).tobytes()
