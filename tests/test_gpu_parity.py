"""GPU parity: the HIP path (through the C ABI) vs the oracle and the reference goldens.

Contract: gate states, frame r / levels and chunk layout
bit-exact; samples within 1e-4 where the OLA window sum is >= 1e-3 (elsewhere
the reference itself is ill-conditioned, F7; those samples are only reported).
"""
import numpy as np
import pytest

from tests.golden_util import (CASES, BY_NAME, load_fixture, case_input, run_oracle,
                               parse_eq_csv, parse_diff_csv)

pytestmark = pytest.mark.gpu
TOL = 1e-4
TAU = 1e-3


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine
    return torch, engine


def run_gpu(case, fx, x):
    torch, E = _engine()
    p = dict(case["params"])
    sr, mode = case["sr"], case["mode"]
    ss = E.StreamSet.from_arrays([x], sr)
    if mode == "standard":
        pipe = E.GatePipeline(ss, **p)
    elif mode == "xfade":
        pipe = E.GatePipeline(ss, **{**p, "xfade_ms": p.get("xfade_ms", 0.0)})
    elif mode == "adaptive":
        pipe = E.AdaptivePipeline(ss, **p)
    elif mode == "layer2":
        from tomatis_audio_processor_amd import dsp
        fr, db = parse_eq_csv(str(fx["eq_csv"]))
        n_fft, hop = p.get("n_fft", 4096), p.get("hop", 2048)
        gain = dsp.build_gain_per_bin(sr, n_fft, fr, db)
        pipe = E.StaticEqPipeline(ss, gain, n_fft=n_fft, hop=hop, pad=p.get("pad", True),
                                  global_gain_db=p.get("global_gain_db", 0.0))
    else:
        from tomatis_audio_processor_amd import dsp
        rf, rd = parse_diff_csv(str(fx["diff_csv"]))
        safe = mode == "layer2b_safe"
        n_fft, hop = p.get("n_fft", 4096), p.get("hop", 2048)
        res_s = dsp.smooth_on_logfreq(rf, rd, win=61 if safe else 41)
        freqs = np.fft.rfftfreq(n_fft, 1.0 / sr)
        if safe:
            lin, _ = dsp.build_eq_from_residual_safe(freqs, rf, res_s)
        else:
            lin, _ = dsp.build_eq_from_residual(freqs, rf, res_s)
        pipe = E.StaticEqPipeline(ss, lin, n_fft=n_fft, hop=hop, pad=False)
    res = pipe.run()
    torch.cuda.synchronize()
    return pipe, res


def _mask_for(case, ref):
    mode = case["mode"]
    N = case["N"]
    if mode in ("standard", "xfade"):
        pad = ref["pad"]
        return ref["wsum"][pad:pad + N] >= TAU
    if mode == "adaptive":
        return ref["wsum"] >= TAU
    return ref["wsum"] >= TAU


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_case_parity(case):
    fx = load_fixture(case["name"])
    x = case_input(case)
    ref = run_oracle(case, fx, x)
    pipe, res = run_gpu(case, fx, x)
    mode = case["mode"]
    y = res.output(0)
    yr = np.asarray(ref["y"], np.float64)
    assert y.shape == yr.shape
    if mode in ("standard", "xfade"):
        # frame r bit-exact, states bit-exact
        r = res.stream_r(0)
        np.testing.assert_array_equal(r.view(np.uint32), ref["r"].view(np.uint32))
        np.testing.assert_array_equal(res.stream_states(0), ref["states"])
        if mode == "xfade":
            np.testing.assert_array_equal(res.stream_alpha(0), ref["alpha"])
    if mode == "adaptive":
        np.testing.assert_array_equal(res.stream_states(0), ref["states"])
        np.testing.assert_array_equal(res.stream_alpha(0), ref["alpha"])
        assert float(res.extra["thresholds"].cpu().numpy()[0]) == ref["threshold"]
    m = _mask_for(case, ref)
    assert m.shape[0] == y.shape[0]
    if not len(y):
        return
    if mode in ("standard", "xfade", "adaptive"):
        _check_chunks(res, ref, y, yr, m, mode)
    else:
        err = np.abs(y[m] - yr[m])
        assert float(err.max(initial=0.0)) <= TOL, f"max err {err.max()}"
    if mode == "layer2" and ref.get("y_gp") is not None:
        _check_gain_protect(res, ref, fx, m)


def _scale_of(peak, limit=0.999):
    return float(np.float32(limit) / np.float32(peak)) if peak > limit else 1.0


def _check_chunks(res, ref, y, yr, m, mode):
    """Per limiter chunk: an unflagged chunk (scale determined by well-conditioned
    samples, conditioning.py) matches the oracle sample by sample; a flagged one
    matches before the limiter, and every chunk whose scale differs from the
    oracle's must be flagged (no missed ill-conditioned scale)."""
    from tomatis_audio_processor_amd import conditioning
    flags = res.scale_flags(0)
    ranges = res.chunk_ranges(0)
    peaks = res.stream_peaks(0)
    ref_scales = ref["scales"] if mode != "adaptive" else [ref["scale"] or 1.0]
    assert len(ranges) == len(ref_scales) == len(flags)
    for c, (a, b) in enumerate(ranges):
        if b <= a:
            continue
        gs, rs = _scale_of(peaks[c]), float(ref_scales[c] or 1.0)
        mm = m[a:b]
        if abs(gs / rs - 1.0) > conditioning.ETA:
            assert flags[c], f"chunk {c}: scale {gs} vs oracle {rs} but not flagged"
        if not flags[c]:
            err = np.abs(y[a:b][mm] - yr[a:b][mm])
        else:
            err = np.abs(y[a:b][mm] / gs - yr[a:b][mm] / rs) * min(gs, rs)
        assert float(err.max(initial=0.0)) <= TOL, f"chunk {c} (flag {flags[c]}): {err.max()}"


def _check_gain_protect(res, ref, fx, m):
    """layer-2 gain protect (src/layer2_apply_eq.py:220-233): when the scale is
    determined (unflagged) the GPU's _gp output matches the reference's _gp
    samples (fixture gp_sub, and the oracle's y_gp, which reproduces gp_sha);
    when flagged it is at least the main output times the GPU's own scale."""
    from tomatis_audio_processor_amd import engine
    import torch
    peak = float(res.stream_peaks(0)[0])
    flag = res.scale_flags(0, limit=0.99)[0]
    scale = 0.99 / max(peak, 1e-12)
    n = res.out_lens[0] * res.ch
    ygp = engine.scale_copy(res.y[:n], scale).cpu().numpy().reshape(-1, res.ch)
    y = res.output(0)
    np.testing.assert_array_equal(ygp, (y * np.float32(scale)).astype(np.float32))
    if not flag:
        assert abs(scale / ref["scale"] - 1.0) <= 5e-5
        step = max(1, len(ref["y_gp"]) // 1500)
        np.testing.assert_array_equal(ref["y_gp"][::step], fx["gp_sub"])
        err = np.abs(ygp[m] - ref["y_gp"][m])
        assert float(err.max(initial=0.0)) <= TOL
        sub_m = m[::step]
        err = np.abs(ygp[::step][sub_m] - fx["gp_sub"][sub_m])
        assert float(err.max(initial=0.0)) <= TOL
    else:
        # the reference's peak_seen is an ill-conditioned head/tail sample
        w = ref["wsum"]
        p = np.abs(ref["y"]).max(axis=1)
        assert p[w < TAU].max() >= p[w >= TAU].max() * (1 - 1e-4)


def test_ill_tail_chunk_is_flagged():
    """Golden std_48k_st_tail_ill: the reference's last-chunk limiter scale is set
    by a tail sample with sum w^2 < 1e-3 (process_tomatis.py:447-453): the flag
    fires on that chunk and not on the first."""
    c = BY_NAME["std_48k_st_tail_ill"]
    fx = load_fixture(c["name"])
    x = case_input(c)
    pipe, res = run_gpu(c, fx, x)
    assert res.scale_flags(0) == [False, True]


def test_silent_edges_gain_protect_unflagged():
    c = BY_NAME["l2_48k_st_pad_gp_silent_edges"]
    fx = load_fixture(c["name"])
    pipe, res = run_gpu(c, fx, case_input(c))
    assert res.scale_flags(0, limit=0.99) == [False]
    assert BY_NAME["l2_48k_st_pad_gp"]["name"]
    pipe2, res2 = run_gpu(BY_NAME["l2_48k_st_pad_gp"], load_fixture("l2_48k_st_pad_gp"),
                          case_input(BY_NAME["l2_48k_st_pad_gp"]))
    assert res2.scale_flags(0, limit=0.99) == [True]


def test_synth_kernel_matches_numpy():
    torch, E = _engine()
    from tomatis_audio_processor_amd.synth import synth_stream
    ss = E.StreamSet.synthetic(2, 50000, 2, 44100, seed0=5)
    torch.cuda.synchronize()
    got = ss.x.cpu().numpy().reshape(2, 50000, 2)
    for i in range(2):
        np.testing.assert_array_equal(got[i], synth_stream(5 + i, 50000, 2, 44100))


def test_gate_api_functions():
    """compute_frame_levels / simulate_gate / find_optimal_threshold on the GPU
    match the oracle's restatement of the reference functions."""
    torch, E = _engine()
    from oracle import tomatis_oracle as orc
    c = BY_NAME["adapt_44k_st_2048_512"]
    x = case_input(c)
    ref = orc.process_adaptive(x, c["sr"], n_fft=2048, hop=512)
    # the reference computes levels on the attenuated signal (adaptive.py:215-219)
    xa = x * (10 ** (np.asarray(-ref["atten_db"]) / 20.0))
    lv, valid, times = E.compute_frame_levels(xa, c["sr"], 2048, 512)
    np.testing.assert_array_equal(lv, ref["levels"])
    T = E.find_optimal_threshold(lv, valid, 3.0, ref["min_hold_frames"], 0.5)
    assert T == ref["threshold"]
    st = E.simulate_gate(lv, T, 3.0, ref["min_hold_frames"])
    assert st == ["C1" if s == 1 else "C2" for s in ref["states"]]


@pytest.mark.parametrize("gate_path", ["runscan", "tf", "fused"])
@pytest.mark.parametrize("up_delay_ms", [0.0, 30.0, 250.0])
def test_gate_paths_multistream(gate_path, up_delay_ms, monkeypatch):
    """Every gate implementation -- the two-pass chain's closed-form run scan
    and transfer-function scan (tomatis_gate_std, fused_levels=False: they also
    serve every gate-carry fallback, non-exclusive predicates and xfade) and the
    in-kernel automaton (tomatis_stft_ola_gated) -- against the reference
    automaton over the GPU's own frame r, on 3 streams of different lengths
    whose level toggles around the thresholds every few frames."""
    torch, E = _engine()
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd._lib import dev_options
    sr, rng = 44100, np.random.default_rng(int(up_delay_ms) + 7)
    xs = []
    for n in (sr * 20 + 77, sr * 9, sr * 31 + 1000):
        steps = np.repeat(10 ** (rng.uniform(-75, -5, n // 700 + 1) / 20), 700)[:n]
        xs.append((rng.standard_normal((n, 2)) * steps[:, None]).astype(np.float32))
    ss = E.StreamSet.from_arrays(xs, sr)
    with dev_options(GATE_TF=1 if gate_path == "tf" else -1):
        pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512, up_delay_ms=up_delay_ms,
                              fused_levels=gate_path == "fused")
        res = pipe.run()
        torch.cuda.synchronize()
    assert pipe.gated_used == (gate_path == "fused")
    for i in range(3):
        r = res.stream_r(i)
        starts = res.first_start[i] + 512 * np.arange(len(r), dtype=np.int64)
        ref = orc.gate_standard(orc.r_to_level(r), starts, pipe.Ton, pipe.Toff,
                                pipe.up_delay_samples)
        st = res.stream_states(i)
        assert 0 < np.count_nonzero(st == 2) < len(st)
        np.testing.assert_array_equal(st, ref)


def test_fused_limiter_matches_two_pass(monkeypatch):
    """tomatis_stft_ola_limited (limiter inside the transform kernel) is bit-identical
    to tomatis_stft_ola + tomatis_apply_limiter on 4 streams with many chunks, loud
    enough that most chunks are limited."""
    torch, E = _engine()
    sr = 48000
    rng = np.random.default_rng(11)
    xs = [(rng.standard_normal((n, 2)) * 0.3).astype(np.float32)
          for n in (sr * 40 + 5, sr * 13, sr * 27 + 999, sr * 6)]
    outs = []
    from tomatis_audio_processor_amd._lib import dev_options
    for fuse in (0, 1):
        with dev_options(FUSE_LIMITER=fuse):
            ss = E.StreamSet.from_arrays(xs, sr)
            pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
            res = pipe.run()
        torch.cuda.synchronize()
        pipe.plan.check_device()
        outs.append((res.y.cpu().numpy().copy(), res.chunk_peaks.cpu().numpy().copy()))
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert np.count_nonzero(outs[0][1].view(np.float32) > 0.999) > 10
    np.testing.assert_array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))


@pytest.mark.parametrize("xfade_ms", [0.0, 500.0, 5000.0])
def test_adaptive_alpha_long_streams(xfade_ms):
    """Chunk-parallel adaptive alpha (k_minhold) == the sequential reference scan
    (process_tomatis_adaptive.py:253-265) bit-for-bit on streams long enough for
    many 256-frame chunks; 5000 ms makes most chunks sync-free (carry chain)."""
    torch, E = _engine()
    from oracle import tomatis_oracle as orc
    ss = E.StreamSet.synthetic(3, 44100 * 95 + 777, 2, 44100, seed0=71)
    pipe = E.AdaptivePipeline(ss, n_fft=2048, hop=512, xfade_ms=xfade_ms)
    res = pipe.run()
    torch.cuda.synchronize()
    pipe.plan.check_device()  # fused global limiter finished within its wait bound
    for i in range(3):
        st = res.stream_states(i)
        assert len(st) > 8 * 256
        ref = orc.alpha_scan_adaptive(st, pipe.xf)
        got = res.stream_alpha(i)
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
        a, F = res.frame_base[i], res.n_frames[i]
        rows = pipe.rows[a:a + F].cpu().numpy().astype(np.int64)
        assert np.array_equal(rows, 2 + np.rint(ref * max(pipe.xf, 1)).astype(np.int64))


@pytest.mark.parametrize("min_hold_ms,hop,secs", [(0.0, 512, 40), (250.0, 512, 770),
                                                  (3000.0, 128, 150)])
def test_minhold_bisect_table_paths(min_hold_ms, hop, secs):
    """k_minhold (per-threshold 2-bit symbols, segment transfer tables) against the
    reference automaton and bisection (process_tomatis_adaptive.py:87-154) on the
    GPU's own levels: min-hold 0; a stream of > 65536 frames (symbols outside
    LDS); a 1034-frame min-hold (transfer tables outside LDS)."""
    torch, E = _engine()
    from oracle import tomatis_oracle as orc
    sr, rng = 44100, np.random.default_rng(secs)
    n = sr * secs
    steps = np.repeat(10 ** (rng.uniform(-75, -5, n // 5000 + 1) / 20), 5000)[:n]
    x = (rng.standard_normal((n, 2)) * steps[:, None] * 0.3).astype(np.float32)
    ss = E.StreamSet.from_arrays([x, x[: n // 3]], sr)
    pipe = E.AdaptivePipeline(ss, n_fft=2048, hop=hop, min_hold_ms=min_hold_ms)
    res = pipe.run()
    torch.cuda.synchronize()
    lv_all = res.extra["levels"].cpu().numpy()
    T_all = res.extra["thresholds"].cpu().numpy()
    for i in range(2):
        a, F = res.frame_base[i], res.n_frames[i]
        lv = lv_all[a:a + F]
        T = orc.optimal_threshold(lv, lv > -70, 3.0, pipe.mh, 0.5)
        assert T_all[i] == T, (i, T_all[i], T)
        st = res.stream_states(i)
        ref = orc.gate_minhold(lv, T, 3.0, pipe.mh)
        assert 0 < np.count_nonzero(ref == 2) < F
        np.testing.assert_array_equal(st, ref)
