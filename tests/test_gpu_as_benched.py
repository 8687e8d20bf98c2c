"""GPU: the pipelines bench.py times, at the sizes it times them, in the mode it
times them (batch pipelines: pass k+1's transform applies pass k's limiter in
its frame loops -- the k_stft_ola PR instantiation that earns the headline).

For C2 (one 60-min stream), C4 (64 x 5 min, one GPU's share), C3 (64 x 5 min
adaptive, AdaptiveGroups(2)) and C5 (16 x 5 min 96 kHz xfade -> layer-2b):
three pipelined passes over three distinct inputs (bench.py's seeds), then
flush().  Every pass's final output and chunk peaks (and per-pass states / r /
alpha) must equal an unpipelined pass over the same input bit for bit; the
middle pass -- limited inside the next pass's frame loop, not by a tail or a
flush -- is checked against the oracle directly: states (and alpha) bit-exact,
chunk scales within 5e-5, samples within 1e-4 where sum w^2 >= 1e-3
(src/process_tomatis.py:331-357,394-426; src/process_tomatis_adaptive.py:
298-345; src/process_tomatis_xfade.py:251-312; src/layer2b_apply_residual_eq.py:
120-160).
"""
import numpy as np
import pytest

from oracle import tomatis_oracle as orc
from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu
TOL = 1e-4
TAU = 1e-3
LIM = 0.999
PASSES = 3


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine
    return torch, engine


def _seed0(j):
    """bench.py's input j (rank 0): streams seed0 + i"""
    return 1000 + 7919 * j


def _inputs(E, S, n, ch, sr):
    return [E.StreamSet.synthetic(S, n, ch, sr, seed0=_seed0(j)).x for j in range(PASSES)]


def _set(pipe, x):
    for q in getattr(pipe, "pipes", None) or [getattr(pipe, "s1", pipe)]:
        q.ss.x = x


def _check_chunks(res, i, ref, y, n):
    """scales within 5e-5 and samples within 1e-4 per unflagged chunk"""
    m = ref["wsum"][ref["pad"]:ref["pad"] + n] >= TAU
    flags = res.scale_flags(i)
    peaks = res.stream_peaks(i)
    for c, (a, b) in enumerate(res.chunk_ranges(i)):
        if flags[c]:
            continue
        gs = float(np.float32(LIM) / np.float32(peaks[c])) if peaks[c] > LIM else 1.0
        rs = ref["scales"][c] or 1.0
        assert abs(gs / rs - 1) <= 5e-5, (i, c)
        assert np.abs(y[a:b][m[a:b]] - ref["y"][a:b][m[a:b]]).max() <= TOL, (i, c)


def _result_of(E, pipe, y, peaks, r, states, alpha):
    """a GatePipeline's Result over the given per-pass arrays (a pass that is
    final but no longer the pipeline's current one)"""
    st = pipe.streams
    return E.Result(y=y, out_offs=pipe.out_offs, out_lens=[s.out_len for s in st], ch=pipe.ss.ch,
                    frame_base=[s.frame_base for s in st], n_frames=[s.n_frames for s in st],
                    first_start=[s.first_start for s in st], hop=pipe.hop, states=states, r=r,
                    alpha=alpha, chunk_peaks=peaks, chunk_base=[s.chunk_base for s in st],
                    n_chunks=[s.n_chunks for s in st],
                    extra=dict(bounds=pipe.bounds, n_fft=pipe.n_fft, norm="eps", limit=LIM,
                               limiter_applied=True, out_begin=[s.out_begin for s in st]))


def _gate_passes(torch, E, ss, xs, kw, check_mid):
    """unpipelined references, then the pipelined passes as bench.py's timed
    loop runs them: back to back with no host synchronisation.  Each pass's
    arrays are copied on the stream once final (its output after the next
    pass, its r / states after its own) and compared at the end;
    check_mid(res) on the middle pass."""
    ref = E.GatePipeline(ss, **kw)
    refs = []
    for x in xs:
        _set(ref, x)
        ref.run()
        refs.append((ref.y.clone(), ref.peaks.clone(), ref.r.clone(), ref.states.clone(),
                     ref.alpha.clone() if ref.alpha is not None else None))
    del ref
    pipe = E.GatePipeline(ss, pipelined=True, **kw)
    F = pipe.plan.total_frames
    got, cur = [], None
    for k, x in enumerate(xs):
        _set(pipe, x)
        assert pipe.run(check_device=False) is None and pipe.pending and pipe.pipelined
        if cur is not None:    # pass k-1 was limited inside pass k's transform
            got.append((cur[0].clone(), cur[1].clone()) + cur[2:])
        cur = (pipe.y, pipe.peaks, pipe.r.clone(), pipe.states.clone(),
               pipe.alpha.clone() if pipe.alpha is not None else None)
    res = pipe.result()
    got.append((res.y, res.chunk_peaks) + cur[2:])
    assert pipe.finish() == 0 and not pipe.pending
    assert pipe.gate_fallbacks == 0
    for k, (y, pk, r, st, al) in enumerate(got):
        ry, rpk, rr, rst, ral = refs[k]
        assert torch.equal(st[:F], rst[:F]), f"pass {k}: states differ"
        assert torch.equal(r[:F].view(torch.int32), rr[:F].view(torch.int32)), f"pass {k}: r differs"
        if al is not None:
            assert torch.equal(al[:F], ral[:F]), f"pass {k}: alpha differs"
        assert torch.equal(pk, rpk), f"pass {k}: chunk peaks differ"
        assert torch.equal(y, ry), f"pass {k}: output differs"
    check_mid(_result_of(E, pipe, *got[1]))
    return pipe


def test_c2_pipelined_as_benched():
    """bench.py (default, C2): GatePipeline(pipelined=True) over the full
    60-min stream, three distinct inputs; pass 1 vs the oracle."""
    torch, E = _engine()
    import bench
    S, secs, sr, ch, _, n_fft, hop, _ = bench.WORKLOADS["c2"]
    n = secs * sr
    xs = _inputs(E, S, n, ch, sr)
    ss = E.StreamSet(x=xs[0], offs=[0], lens=[n], ch=ch, sr=sr)
    kw = dict(gate_ui=50, n_fft=n_fft, hop=hop)

    def mid(res):
        ref = orc.process_standard(synth_stream(_seed0(1), n, ch, sr), sr, **kw)
        np.testing.assert_array_equal(res.stream_states(0), ref["states"])
        _check_chunks(res, 0, ref, res.output(0), n)

    pipe = _gate_passes(torch, E, ss, xs, kw, mid)
    assert pipe.gated_used


def test_c4_pipelined_as_benched():
    """bench.py --workload c4: 64 x 5 min 48 kHz per GPU, pipelined; pass 1's
    streams 0, 21, 42, 63 vs the oracle, the per-chunk limiter property on all."""
    torch, E = _engine()
    import bench
    S, secs, sr, ch, _, n_fft, hop, _ = bench.WORKLOADS["c4"]
    n = secs * sr
    xs = _inputs(E, S, n, ch, sr)
    ss = E.StreamSet(x=xs[0], offs=[i * n * ch for i in range(S)], lens=[n] * S, ch=ch, sr=sr)
    kw = dict(gate_ui=50, n_fft=n_fft, hop=hop)

    def mid(res):
        y_all = res.y[:S * n * ch].view(S, n, ch)
        ranges = res.chunk_ranges(0)
        cmax = torch.stack([y_all[:, a:b].abs().amax(dim=(1, 2)) for a, b in ranges], 1).cpu().numpy()
        for i in range(S):
            peaks = res.stream_peaks(i)
            for c in range(len(ranges)):
                assert cmax[i, c] <= LIM * (1 + 2e-7), (i, c, cmax[i, c])
                if peaks[c] > LIM:
                    assert cmax[i, c] >= LIM * (1 - 1e-6), (i, c)
        for i in (0, 21, 42, 63):
            ref = orc.process_standard(synth_stream(_seed0(1) + i, n, ch, sr), sr, **kw)
            np.testing.assert_array_equal(res.stream_states(i), ref["states"])
            _check_chunks(res, i, ref, res.output(i), n)

    _gate_passes(torch, E, ss, xs, kw, mid)


def _result_nf(p):
    """a pipeline's Result without flushing (its arrays as they stand)"""
    pend = p.pending
    p.pending = False
    try:
        return p.result()
    finally:
        p.pending = pend


def test_c3_pipelined_as_benched():
    """bench.py --workload c3: AdaptiveGroups(2, pipelined=True), 64 x 5 min;
    every pass bit-identical to unpipelined; pass 1's streams 0, 31, 32, 63 vs
    orc.process_adaptive (threshold, states, alpha bit-exact; global scale)."""
    torch, E = _engine()
    import bench
    S, secs, sr, ch, _, n_fft, hop, _ = bench.WORKLOADS["c3"]
    n = secs * sr
    xs = _inputs(E, S, n, ch, sr)
    ss = E.StreamSet(x=xs[0], offs=[i * n * ch for i in range(S)], lens=[n] * S, ch=ch, sr=sr)
    ref = E.AdaptiveGroups(ss, groups=2, n_fft=n_fft, hop=hop)
    refs = []
    for x in xs:
        _set(ref, x)
        r = ref.run()
        refs.append((r.y.clone(), r.chunk_peaks.clone(), r.states.clone(), r.alpha.clone(),
                     r.extra["thresholds"].clone()))
    del ref, r
    pipe = E.AdaptiveGroups(ss, groups=2, n_fft=n_fft, hop=hop, pipelined=True)
    held = None
    for k, x in enumerate(xs):
        _set(pipe, x)
        assert pipe.run() is None and pipe.pending and pipe.pipelined
        if held is not None:
            y, pk, st, al, thr = held
            torch.cuda.synchronize()
            assert torch.equal(thr, refs[k - 1][4]), f"pass {k - 1}: thresholds differ"
            assert torch.equal(st, refs[k - 1][2]) and torch.equal(al, refs[k - 1][3])
            assert torch.equal(pk, refs[k - 1][1]), f"pass {k - 1}: peaks differ"
            assert torch.equal(y, refs[k - 1][0]), f"pass {k - 1}: output differs"
            if k - 1 == 1:  # res_nf: pass 1's merged Result (its buffer final now)
                thr_h = thr.cpu().numpy()
                for i in (0, 31, 32, 63):
                    rr = orc.process_adaptive(synth_stream(_seed0(1) + i, n, ch, sr), sr,
                                              n_fft=n_fft, hop=hop)
                    assert float(thr_h[i]) == rr["threshold"], f"stream {i}"
                    np.testing.assert_array_equal(res_nf.stream_states(i), rr["states"])
                    assert np.array_equal(res_nf.stream_alpha(i).view(np.uint64),
                                          rr["alpha"].view(np.uint64))
                    yi = res_nf.output(i)
                    m = rr["wsum"] >= TAU
                    p0 = res_nf.stream_peaks(i)[0]
                    gs = float(np.float32(LIM) / np.float32(p0)) if p0 > LIM else 1.0
                    rs = rr["scale"] or 1.0
                    if not res_nf.scale_flags(i)[0]:
                        assert abs(gs / rs - 1) <= 5e-5, f"stream {i}"
                        assert np.abs(yi[m] - rr["y"][m]).max() <= TOL, f"stream {i}"
                    else:  # an ill-conditioned global peak (conditioning.py): shapes
                        assert np.abs(yi[m] / gs - rr["y"][m] / rs).max() * min(gs, rs) <= TOL
        res_nf = E.merge_results([_result_nf(p) for p in pipe.pipes])
        held = (res_nf.y, res_nf.chunk_peaks.clone(), res_nf.states.clone(), res_nf.alpha.clone(),
                res_nf.extra["thresholds"].clone())
    res = pipe.result()
    assert not pipe.pending
    assert torch.equal(res.chunk_peaks, refs[-1][1]) and torch.equal(res.y, refs[-1][0])


def test_c5_pipelined_as_benched():
    """bench.py --workload c5: ChainC5(pipelined=True), 16 x 5 min 96 kHz,
    three passes: stage 1 (xfade 4096/1024, pipelined through VGPR partner
    blocks) and stage 2 (layer-2b) of every pass bit-identical to the
    unpipelined chain; pass 1's stage 1 vs the oracle on 4 streams."""
    torch, E = _engine()
    import bench
    S, secs, sr, ch, _, n_fft, hop, _ = bench.WORKLOADS["c5"]
    n = secs * sr
    xs = _inputs(E, S, n, ch, sr)
    ss = E.StreamSet(x=xs[0], offs=[i * n * ch for i in range(S)], lens=[n] * S, ch=ch, sr=sr)
    ref = bench.ChainC5(E, ss, sr, n_fft, hop, pipelined=False)
    refs = []
    for x in xs:
        _set(ref, x)
        r2 = ref.run()
        assert r2 is not None
        refs.append((ref.s1.y.clone(), ref.s1.peaks.clone(), ref.s1.states.clone(),
                     ref.s1.alpha.clone(), r2.y.clone()))
    del ref, r2
    chain = bench.ChainC5(E, ss, sr, n_fft, hop, pipelined=True)
    assert chain.pipelined
    F = chain.s1.plan.total_frames
    held = None
    for k, x in enumerate(xs):
        _set(chain, x)
        out2 = chain.run()
        assert out2 is None and chain.s1.pending
        if held is not None:
            y1, pk, st, al = held
            assert torch.equal(st[:F], refs[k - 1][2][:F]) and torch.equal(al[:F], refs[k - 1][3][:F])
            assert torch.equal(pk, refs[k - 1][1]), f"pass {k - 1}: stage-1 peaks differ"
            assert torch.equal(y1, refs[k - 1][0]), f"pass {k - 1}: stage-1 output differs"
            y2 = chain.s2[y1.data_ptr()].y
            assert torch.equal(y2, refs[k - 1][4]), f"pass {k - 1}: stage-2 output differs"
            if k - 1 == 1:
                res1 = _result_of(E, chain.s1, y1, pk, chain.s1.r, st, al)
                for i in (0, 5, 10, 15):
                    rr = orc.process_standard(synth_stream(_seed0(1) + i, n, ch, sr), sr, gate_ui=50,
                                              gate_offset=-90, n_fft=n_fft, hop=hop, xfade_ms=500.0)
                    np.testing.assert_array_equal(res1.stream_states(i), rr["states"])
                    np.testing.assert_array_equal(res1.stream_alpha(i), rr["alpha"])
                    _check_chunks(res1, i, rr, res1.output(i), n)
        held = (chain.s1.y, chain.s1.peaks, chain.s1.states.clone(), chain.s1.alpha.clone())
    last2 = chain.flush()
    torch.cuda.synchronize()
    assert torch.equal(chain.s1.y, refs[-1][0]) and torch.equal(last2.y, refs[-1][4])
