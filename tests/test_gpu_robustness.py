"""GPU: the product paths read the device error word and recover / fail loudly,
and the batch sizes bench.py times (C3, C4 per GPU) are checked, not only
timed.

* Fault injection: ``TOMATIS_OPT_LIMITER_SPIN = 0`` makes every fused-limiter
  wave give up at once (TOMATIS_ERR_LIMITER_WAIT, its samples left unscaled).
  ``engine.finish_plan`` must see the bit, warn, re-run the transform with the
  separate limiter launch and return output bit-identical to an undisturbed
  run -- for the standard, adaptive (AdaptiveGroups) and time-shard paths.
* C3 exactly as benched: 64 x 5 min stereo 44.1 kHz, AdaptiveGroups(2),
  2048/512 -- 4 streams against ``orc.process_adaptive`` (threshold, states,
  alpha bit-exact; samples <= 1e-4 where sum w^2 >= 1e-3), the global-limiter
  property on all 64 (reference: src/process_tomatis_adaptive.py:340-345).
* C4 per-GPU batch: 64 x 5 min stereo 48 kHz, standard, 2048/512 -- 4 streams
  against ``orc.process_standard``, the per-chunk limiter property on all 64
  (src/process_tomatis.py:331-357: every chunk over 0.999 is scaled to it).
"""
import numpy as np
import pytest

from oracle import tomatis_oracle as orc
from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu
TOL = 1e-4
TAU = 1e-3
LIM = 0.999


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine
    return torch, engine


def test_fused_limiter_timeout_recovery_standard():
    torch, E = _engine()
    sr, n = 44100, 44100 * 40 + 123
    ss = E.StreamSet.synthetic(2, n, 2, sr, seed0=31)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    pipe.run()
    y0 = pipe.y.clone()
    assert pipe.plan.error_bits() == 0
    pipe.plan.set_limiter_spin(0)
    try:
        with pytest.warns(RuntimeWarning, match="fused limiter wait timed out"):
            pipe.run()
    finally:
        pipe.plan.set_limiter_spin(1 << 18)
    assert torch.equal(pipe.y, y0)
    assert pipe.plan.error_bits() == 0
    # the injected fault really leaves chunks unscaled when nobody checks
    pipe.plan.set_limiter_spin(0)
    try:
        pipe.run(check_device=False)
        bits = pipe.plan.error_bits()
    finally:
        pipe.plan.set_limiter_spin(1 << 18)
    assert bits == 1
    assert not torch.equal(pipe.y, y0)
    pipe.run()
    assert torch.equal(pipe.y, y0)


def test_fused_limiter_timeout_recovery_adaptive_groups():
    torch, E = _engine()
    sr = 44100
    ss = E.StreamSet.synthetic(6, sr * 20, 2, sr, seed0=90)
    pipe = E.AdaptiveGroups(ss, groups=2, n_fft=2048, hop=512)
    pipe.run()
    y0 = pipe.y.clone()
    for p in pipe.pipes:
        p.plan.set_limiter_spin(0)
    try:
        with pytest.warns(RuntimeWarning, match="fused limiter"):
            pipe.run()
    finally:
        for p in pipe.pipes:
            p.plan.set_limiter_spin(1 << 18)
    assert torch.equal(pipe.y, y0)


def test_fused_limiter_timeout_recovery_timeshard():
    torch, E = _engine()
    from tomatis_audio_processor_amd import timeshard
    sr, n = 44100, 44100 * 60
    x = synth_stream(5, n, 2, sr)
    params = dict(gate_ui=50, n_fft=2048, hop=512)
    ref = E.GatePipeline(E.StreamSet.from_arrays([x], sr), **params).run().output(0)
    st = timeshard.RankStep(x, sr, n, 0, 1, ch=2, **params)
    st.rn.pipe.plan.set_limiter_spin(0)
    try:
        with pytest.warns(RuntimeWarning, match="fused limiter"):
            res = st.run()
    finally:
        st.rn.pipe.plan.set_limiter_spin(1 << 18)
    assert np.array_equal(res.output(0), ref)


def test_pair_barrier_bit_raises():
    """A set TOMATIS_ERR_PAIR_BARRIER bit is never recovered: finish_plan raises."""
    torch, E = _engine()

    class FakePlan:
        def __init__(self):
            self.bits = 2

        def error_bits(self, reset=True):
            b, self.bits = self.bits, 0
            return b

    with pytest.raises(E.DeviceCheckError):
        E.finish_plan(FakePlan(), lambda: None, "test")


def test_c3_batch_as_benched():
    """bench.py --workload c3's one-file-job leg (``one_file_job``: unpipelined
    passes, the global limiter inside each pass): 64 x 5 min, AdaptiveGroups(2),
    seeds 1000..  The pipelined mode of the headline: test_gpu_as_benched.py."""
    torch, E = _engine()
    sr, n, S = 44100, 300 * 44100, 64
    n_fft, hop = 2048, 512
    ss = E.StreamSet.synthetic(S, n, 2, sr, seed0=1000)
    pipe = E.AdaptiveGroups(ss, groups=2, n_fft=n_fft, hop=hop)
    res = pipe.run()
    torch.cuda.synchronize()
    thr = res.extra["thresholds"].cpu().numpy()
    y_all = res.y[:S * n * 2].view(S, n, 2)
    # the global limiter on every stream (one chunk each)
    pk_out = y_all.abs().amax(dim=(1, 2)).cpu().numpy()
    for i in range(S):
        peak = float(res.stream_peaks(i)[0])
        assert pk_out[i] <= LIM * (1 + 2e-7), (i, pk_out[i])
        if peak > LIM:
            assert pk_out[i] >= LIM * (1 - 1e-6), (i, pk_out[i], peak)
    # 4 streams (first/last of each group) against the oracle
    for i in (0, 31, 32, 63):
        x = synth_stream(1000 + i, n, 2, sr)
        ref = orc.process_adaptive(x, sr, n_fft=n_fft, hop=hop)
        assert float(thr[i]) == ref["threshold"], f"stream {i}"
        np.testing.assert_array_equal(res.stream_states(i), ref["states"])
        assert np.array_equal(res.stream_alpha(i).view(np.uint64), ref["alpha"].view(np.uint64))
        y = res.output(i)
        m = ref["wsum"] >= TAU
        gs = (float(np.float32(LIM) / np.float32(res.stream_peaks(i)[0]))
              if res.stream_peaks(i)[0] > LIM else 1.0)
        rs = ref["scale"] or 1.0
        if not res.scale_flags(i)[0]:
            assert abs(gs / rs - 1) <= 5e-5
            assert np.abs(y[m] - ref["y"][m]).max() <= TOL, f"stream {i}"
        else:
            assert np.abs(y[m] / gs - ref["y"][m] / rs).max() * min(gs, rs) <= TOL


def test_c4_batch_per_gpu():
    """bench.py --workload c4's one-file-job leg (one GPU's share of C4,
    unpipelined: the fused limiter tail): 64 x 5 min 48 kHz.  The pipelined
    mode of the headline: test_gpu_as_benched.py."""
    torch, E = _engine()
    sr, n, S = 48000, 300 * 48000, 64
    ss = E.StreamSet.synthetic(S, n, 2, sr, seed0=1000)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    res = pipe.run()
    torch.cuda.synchronize()
    # per-chunk limiter property on every stream: chunk maxima on the device
    y_all = res.y[:S * n * 2].view(S, n, 2)
    ranges = res.chunk_ranges(0)
    assert all(res.chunk_ranges(i) == ranges for i in range(S))
    cmax = torch.stack([y_all[:, a:b].abs().amax(dim=(1, 2)) for a, b in ranges], 1).cpu().numpy()
    for i in range(S):
        peaks = res.stream_peaks(i)
        for c in range(len(ranges)):
            assert cmax[i, c] <= LIM * (1 + 2e-7), (i, c, cmax[i, c])
            if peaks[c] > LIM:
                assert cmax[i, c] >= LIM * (1 - 1e-6), (i, c)
    for i in (0, 21, 42, 63):
        x = synth_stream(1000 + i, n, 2, sr)
        ref = orc.process_standard(x, sr, gate_ui=50, n_fft=2048, hop=512)
        np.testing.assert_array_equal(res.stream_states(i), ref["states"])
        y = res.output(i)
        m = ref["wsum"][ref["pad"]:ref["pad"] + n] >= TAU
        flags = res.scale_flags(i)
        peaks = res.stream_peaks(i)
        for c, (a, b) in enumerate(ranges):
            if flags[c]:
                continue
            gs = float(np.float32(LIM) / np.float32(peaks[c])) if peaks[c] > LIM else 1.0
            rs = ref["scales"][c] or 1.0
            assert abs(gs / rs - 1) <= 5e-5, (i, c)
            assert np.abs(y[a:b][m[a:b]] - ref["y"][a:b][m[a:b]]).max() <= TOL, (i, c)


def test_c5_batch_per_gpu():
    """bench.py --workload c5, one pass + flush (one GPU's share of C5): 16 x
    5 min stereo 96 kHz, xfade 500 ms (4096/1024) -> layer-2b residual EQ
    (bench.ChainC5).  Stage 1: the per-chunk limiter property on all 16 streams;
    4 streams vs orc.process_standard(xfade_ms=500) -- states and alpha bit-exact,
    chunk scales within 5e-5, samples <= 1e-4 where sum w^2 >= 1e-3 (reference:
    src/process_tomatis_xfade.py:206-219,251-312).  Stage 2 on the same 4:
    orc.apply_residual_eq on the GPU's own stage-1 floats, samples <= 1e-4
    (src/layer2b_apply_residual_eq.py:120-160)."""
    torch, E = _engine()
    import bench
    S, secs, sr, ch, _, n_fft, hop, _ = bench.WORKLOADS["c5"]
    n = secs * sr
    ss = E.StreamSet.synthetic(S, n, ch, sr, seed0=1000)
    chain = bench.ChainC5(E, ss, sr, n_fft, hop)
    res2 = chain.run()
    if res2 is None:  # pipelined stage 1 (as benched): flush runs its stage 2
        res2 = chain.flush()
    torch.cuda.synchronize()
    res1 = chain.s1.result()
    y_all = res1.y[:S * n * ch].view(S, n, ch)
    ranges = res1.chunk_ranges(0)
    assert all(res1.chunk_ranges(i) == ranges for i in range(S))
    cmax = torch.stack([y_all[:, a:b].abs().amax(dim=(1, 2)) for a, b in ranges], 1).cpu().numpy()
    for i in range(S):
        peaks = res1.stream_peaks(i)
        for c in range(len(ranges)):
            assert cmax[i, c] <= LIM * (1 + 2e-7), (i, c, cmax[i, c])
            if peaks[c] > LIM:
                assert cmax[i, c] >= LIM * (1 - 1e-6), (i, c)
    rf = np.geomspace(20.0, sr / 2, 400)
    rd = 4.0 * np.sin(np.log2(rf / 20.0) * 1.7) * np.exp(-rf / 12000.0)
    for i in (0, 5, 10, 15):
        x = synth_stream(1000 + i, n, ch, sr)
        ref = orc.process_standard(x, sr, gate_ui=50, gate_offset=-90, n_fft=n_fft, hop=hop,
                                   xfade_ms=500.0)
        np.testing.assert_array_equal(res1.stream_states(i), ref["states"])
        np.testing.assert_array_equal(res1.stream_alpha(i), ref["alpha"])
        y1 = res1.output(i)
        m = ref["wsum"][ref["pad"]:ref["pad"] + n] >= TAU
        flags = res1.scale_flags(i)
        peaks = res1.stream_peaks(i)
        for c, (a, b) in enumerate(ranges):
            if flags[c]:
                continue
            gs = float(np.float32(LIM) / np.float32(peaks[c])) if peaks[c] > LIM else 1.0
            rs = ref["scales"][c] or 1.0
            assert abs(gs / rs - 1) <= 5e-5, (i, c)
            assert np.abs(y1[a:b][m[a:b]] - ref["y"][a:b][m[a:b]]).max() <= TOL, (i, c)
        y2 = res2.output(i)
        r2 = orc.apply_residual_eq(y1, sr, rf, rd, n_fft=n_fft, hop=hop)
        assert y2.shape == r2["y"].shape
        m2 = r2["wsum"] >= TAU
        assert np.abs(y2[m2] - r2["y"][m2]).max() <= TOL, i
