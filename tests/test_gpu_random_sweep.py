"""GPU parity over a seeded random sweep of configurations, each against the
oracle (the same checks as test_gpu_parity.test_case_parity: frame r, gate
states, alpha and adaptive thresholds bit-exact; per limiter chunk, samples
within 1e-4 where sum w^2 >= 1e-3, or the chunk flagged by conditioning.py).

The goldens pin the oracle to the reference on 29 fixed cases; this sweep
widens the GPU side: random modes (standard, cross-fade, adaptive), n_fft /
hop (the fused 2048 kernel with hop 256 / 512, the two-wave 4096 kernel, the
LDS / Bluestein any-size path), channels, rates, lengths (down to shorter than
a frame), input levels and gate / cross-fade parameters
(src/process_tomatis.py:160-478, src/process_tomatis_xfade.py:55-359,
src/process_tomatis_adaptive.py:201-345).  The configurations are drawn once
from a fixed seed, so every run checks the same ones.
"""
import numpy as np
import pytest

from tests.golden_util import run_oracle
from tests.test_gpu_parity import _check_chunks, _mask_for, run_gpu
from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu

SHAPES = [(2048, 512), (2048, 256), (4096, 1024), (4096, 2048), (1024, 256), (3000, 750),
          (512, 128)]


def _configs(n=40, seed=20261018):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        mode = ["standard", "standard", "xfade", "adaptive"][rng.integers(4)]
        n_fft, hop = SHAPES[rng.integers(len(SHAPES))]
        sr = int([44100, 48000, 96000][rng.integers(3)])
        ch = int(rng.integers(1, 3))
        secs = float(rng.choice([0.02, 0.3, 2.0, 6.0, 12.0]))
        N = max(64, int(secs * sr) + int(rng.integers(0, 997)))
        gain = float(10.0 ** (rng.uniform(-3.0, 0.3)))
        if mode == "standard":
            params = dict(gate_ui=int(rng.integers(20, 80)), n_fft=n_fft, hop=hop,
                          up_delay_ms=float(rng.choice([0.0, 100.0, 250.0, 600.0])),
                          gate_mode=str(rng.choice(["log_percent", "linear"])))
        elif mode == "xfade":
            params = dict(gate_ui=int(rng.integers(20, 80)), gate_offset=-90, n_fft=n_fft,
                          hop=hop, xfade_ms=float(rng.choice([0.0, 200.0, 500.0, 1500.0])),
                          up_delay_ms=float(rng.choice([0.0, 250.0])))
        else:
            params = dict(n_fft=n_fft, hop=hop, xfade_ms=float(rng.choice([0.0, 500.0])),
                          min_hold_ms=float(rng.choice([0.0, 250.0, 1000.0])),
                          target_c2=float(rng.choice([0.3, 0.5, 0.7])))
        out.append(dict(name=f"r{i:02d}_{mode}_{n_fft}_{hop}_{ch}ch_{sr}", mode=mode, sr=sr,
                        ch=ch, N=N, seed=3000 + i, gain=gain, params=params))
    return out


CONFIGS = _configs()


@pytest.mark.parametrize("case", CONFIGS, ids=[c["name"] for c in CONFIGS])
def test_random_config_vs_oracle(case):
    x = (synth_stream(case["seed"], case["N"], case["ch"], case["sr"]) *
         np.float32(case["gain"])).astype(np.float32)
    ref = run_oracle(case, None, x)
    pipe, res = run_gpu(case, None, x)
    mode = case["mode"]
    y = res.output(0)
    yr = np.asarray(ref["y"], np.float64)
    assert y.shape == yr.shape
    if mode in ("standard", "xfade"):
        np.testing.assert_array_equal(res.stream_r(0).view(np.uint32), ref["r"].view(np.uint32))
        np.testing.assert_array_equal(res.stream_states(0), ref["states"])
        if mode == "xfade":
            np.testing.assert_array_equal(res.stream_alpha(0), ref["alpha"])
    else:
        np.testing.assert_array_equal(res.stream_states(0), ref["states"])
        np.testing.assert_array_equal(res.stream_alpha(0), ref["alpha"])
        np.testing.assert_array_equal(np.float64(res.extra["thresholds"].cpu().numpy()[0]),
                                      np.float64(ref["threshold"]))  # (NaN == NaN: no frames)
    if not len(y):
        return
    _check_chunks(res, ref, y, yr, _mask_for(case, ref), mode)


def _check_chunks_i(res, i, ref, y, yr, m, mode):
    """test_gpu_parity._check_chunks for stream i of a batch"""
    from tomatis_audio_processor_amd import conditioning
    flags, ranges, peaks = res.scale_flags(i), res.chunk_ranges(i), res.stream_peaks(i)
    ref_scales = ref["scales"] if mode != "adaptive" else [ref["scale"] or 1.0]
    assert len(ranges) == len(ref_scales) == len(flags)
    for c, (a, b) in enumerate(ranges):
        if b <= a:
            continue
        gs = float(np.float32(0.999) / np.float32(peaks[c])) if peaks[c] > 0.999 else 1.0
        rs = float(ref_scales[c] or 1.0)
        mm = m[a:b]
        if abs(gs / rs - 1.0) > conditioning.ETA:
            assert flags[c], f"stream {i} chunk {c}: scale {gs} vs oracle {rs} but not flagged"
        if not flags[c]:
            err = np.abs(y[a:b][mm] - yr[a:b][mm])
        else:
            err = np.abs(y[a:b][mm] / gs - yr[a:b][mm] / rs) * min(gs, rs)
        assert float(err.max(initial=0.0)) <= 1e-4, f"stream {i} chunk {c}: {err.max()}"


def _batches(n=16, seed=77031):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        mode = ["standard", "xfade", "adaptive"][rng.integers(3)]
        n_fft, hop = SHAPES[rng.integers(len(SHAPES))]
        ch = int(rng.choice([1, 2, 2, 3]))
        if ch > 2 and (n_fft, hop) in ((2048, 512), (2048, 256), (4096, 1024), (4096, 2048)):
            n_fft, hop = 3000, 750          # > 2 channels: the any-size path
        sr = int([44100, 48000, 96000][rng.integers(3)])
        ns = int(rng.integers(1, 6))
        lens = [max(16, int(float(rng.choice([0.01, 0.2, 1.5, 4.0, 9.0])) * sr)
                    + int(rng.integers(0, 1500))) for _ in range(ns)]
        gains = [float(10.0 ** rng.uniform(-3.0, 0.3)) for _ in range(ns)]
        if mode == "adaptive":
            params = dict(n_fft=n_fft, hop=hop, xfade_ms=float(rng.choice([0.0, 500.0])),
                          min_hold_ms=float(rng.choice([0.0, 250.0])))
        elif mode == "xfade":
            params = dict(gate_ui=int(rng.integers(30, 70)), gate_offset=-90, n_fft=n_fft, hop=hop,
                          xfade_ms=float(rng.choice([0.0, 500.0])))
        else:
            params = dict(gate_ui=int(rng.integers(30, 70)), n_fft=n_fft, hop=hop)
        out.append(dict(name=f"b{i:02d}_{mode}_{n_fft}_{hop}_{ch}ch_{ns}x", mode=mode, sr=sr,
                        ch=ch, lens=lens, gains=gains, seed=5000 + 10 * i, params=params))
    return out


BATCHES = _batches()


@pytest.mark.parametrize("case", BATCHES, ids=[c["name"] for c in BATCHES])
def test_random_batch_vs_oracle(case):
    """A batch of 1-5 streams of ragged lengths (one launch, per-stream gate,
    thresholds and limiter chunks) against the oracle run on each stream alone."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine as E
    mode, sr, ch = case["mode"], case["sr"], case["ch"]
    xs = [(synth_stream(case["seed"] + j, n, ch, sr) * np.float32(g)).astype(np.float32)
          for j, (n, g) in enumerate(zip(case["lens"], case["gains"]))]
    ss = E.StreamSet.from_arrays(xs, sr)
    p = dict(case["params"])
    if mode == "adaptive":
        pipe = E.AdaptivePipeline(ss, **p)
    else:
        pipe = E.GatePipeline(ss, **p)
    res = pipe.run()
    torch.cuda.synchronize()
    for j, x in enumerate(xs):
        c1 = dict(mode=mode, sr=sr, ch=ch, N=len(x), params=p)
        ref = run_oracle(c1, None, x)
        y = res.output(j)
        yr = np.asarray(ref["y"], np.float64)
        assert y.shape == yr.shape, (j, y.shape, yr.shape)
        if mode in ("standard", "xfade"):
            np.testing.assert_array_equal(res.stream_r(j).view(np.uint32), ref["r"].view(np.uint32))
            np.testing.assert_array_equal(res.stream_states(j), ref["states"])
            if mode == "xfade":
                np.testing.assert_array_equal(res.stream_alpha(j), ref["alpha"])
        else:
            np.testing.assert_array_equal(res.stream_states(j), ref["states"])
            np.testing.assert_array_equal(res.stream_alpha(j), ref["alpha"])
            np.testing.assert_array_equal(np.float64(res.extra["thresholds"].cpu().numpy()[j]),
                                          np.float64(ref["threshold"]))
        if len(y):
            _check_chunks_i(res, j, ref, y, yr, _mask_for(c1, ref), mode)


def _eq_cases(n=12, seed=99177):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        n_fft, hop = SHAPES[rng.integers(len(SHAPES))]
        sr = int([44100, 48000, 96000][rng.integers(3)])
        ch = int(rng.choice([1, 2]))
        N = max(32, int(float(rng.choice([0.05, 1.0, 5.0])) * sr) + int(rng.integers(0, 999)))
        k = int(rng.integers(3, 30))
        fr = np.sort(rng.uniform(20.0, sr / 2, k)).astype(np.float32)
        db = rng.uniform(-12.0, 12.0, k).astype(np.float32)
        out.append(dict(name=f"eq{i:02d}_{n_fft}_{hop}_{ch}ch_{sr}", sr=sr, ch=ch, N=N,
                        seed=7000 + i, n_fft=n_fft, hop=hop, pad=bool(rng.integers(2)),
                        gdb=float(rng.choice([0.0, -3.0, 4.5])), fr=fr, db=db,
                        gain=float(10.0 ** rng.uniform(-2.0, 0.0))))
    return out


EQS = _eq_cases()


@pytest.mark.parametrize("case", EQS, ids=[c["name"] for c in EQS])
def test_random_static_eq_vs_oracle(case):
    """layer2_apply_eq's static-EQ STFT (src/layer2_apply_eq.py:66-233; pad /
    no pad as layer-2b) with a random EQ curve, against the oracle: samples
    within 1e-4 where sum w^2 >= 1e-3."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd import dsp, engine as E
    sr, ch, n_fft, hop = case["sr"], case["ch"], case["n_fft"], case["hop"]
    x = (synth_stream(case["seed"], case["N"], ch, sr) * np.float32(case["gain"])).astype(np.float32)
    ref = orc.apply_eq_stft(x, sr, case["fr"], case["db"], n_fft=n_fft, hop=hop, pad=case["pad"],
                            global_gain_db=case["gdb"])
    gain = dsp.build_gain_per_bin(sr, n_fft, case["fr"], case["db"])
    np.testing.assert_array_equal(gain, ref["gain"])
    pipe = E.StaticEqPipeline(E.StreamSet.from_arrays([x], sr), gain, n_fft=n_fft, hop=hop,
                              pad=case["pad"], global_gain_db=case["gdb"])
    res = pipe.run()
    torch.cuda.synchronize()
    y, yr = res.output(0), np.asarray(ref["y"], np.float64)
    assert y.shape == yr.shape
    m = ref["wsum"] >= 1e-3
    err = np.abs(y[m] - yr[m])
    assert float(err.max(initial=0.0)) <= 1e-4, float(err.max())
