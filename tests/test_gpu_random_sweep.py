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
