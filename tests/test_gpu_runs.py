"""GPU: the fused kernel's work decomposition does not change a single bit.

The host cuts every stream into interior runs (fast loop) and edge runs
(generic loop) and sizes runs to the device's resident slots
(tm_kernels.hip plan_build); the limiter is fused in-kernel or run as a second
launch.  Every output hop block is the same frame-ordered float32 sum whatever
the cut, so outputs, chunk peaks and states must be bitwise identical across:
run lengths (TOMATIS_DEV_RUN_FRAMES), the interior loop on/off
(TOMATIS_DEV_FAST_LOOP), and the fused/unfused limiter (TOMATIS_DEV_FUSE_LIMITER),
for the two-pass chain (tomatis_levels -> tomatis_gate_std -> transform) and,
at n_fft 2048 / hop 512, the in-kernel gate (tomatis_stft_ola_gated) as well,
which must also agree with each other.  One small case is also
checked against the oracle.  Streams of unequal, odd lengths make frame_base
odd for some streams (the gain-row ids are read as aligned 32-bit words).
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


def _dev(env):
    from tomatis_audio_processor_amd._lib import dev_options
    return dev_options(**{k.replace("TOMATIS_", ""): int(v) for k, v in env.items()})


def _run(E, torch, xs, sr, env, fused=False, **params):
    with _dev(env):
        ss = E.StreamSet.from_arrays(xs, sr)
        pipe = E.GatePipeline(ss, fused_levels=fused, **params)
        res = pipe.run()
        assert pipe.gated_used == (fused and params["n_fft"] == 2048 and params["hop"] == 512)
        torch.cuda.synchronize()
        pipe.plan.check_device()
        outs = [res.output(i) for i in range(len(xs))]
        sts = [res.stream_states(i) for i in range(len(xs))]
        pks = [res.stream_peaks(i) for i in range(len(xs))]
        return outs, sts, pks


@pytest.mark.parametrize("n_fft,hop,sr", [(2048, 512, 44100), (4096, 1024, 96000),
                                          (4096, 2048, 48000)])
def test_decomposition_bit_identical(n_fft, hop, sr):
    torch, E = _engine()
    lens = [sr * 37 + 1, sr * 20 + 259, sr * 61 + 777]  # odd frame counts -> odd frame_base
    xs = [synth_stream(500 + i, n, 2, sr) for i, n in enumerate(lens)]
    params = dict(gate_ui=50, n_fft=n_fft, hop=hop)
    base = _run(E, torch, xs, sr, {}, **params)
    variants = [{"TOMATIS_RUN_FRAMES": 48}, {"TOMATIS_RUN_FRAMES": 131},
                {"TOMATIS_RUN_FRAMES": 1000}, {"TOMATIS_FAST_LOOP": 0},
                {"TOMATIS_FUSE_LIMITER": 0}, {"TOMATIS_RUN_FRAMES": 77, "TOMATIS_FUSE_LIMITER": 0}]
    runs = [(env, False) for env in variants]
    if n_fft == 2048 and hop == 512:  # the in-kernel gate takes this shape
        runs += [({}, True), ({"TOMATIS_RUN_FRAMES": 131}, True), ({"TOMATIS_RUN_FRAMES": 1000}, True),
                 ({"TOMATIS_FUSE_LIMITER": 0}, True)]
    for env, fused in runs:
        got = _run(E, torch, xs, sr, env, fused=fused, **params)
        for i in range(len(xs)):
            assert np.array_equal(got[1][i], base[1][i]), (env, i, "states")
            assert got[2][i].tobytes() == base[2][i].tobytes(), (env, i, "chunk peaks")
            assert got[0][i].tobytes() == base[0][i].tobytes(), (env, i, "samples")


def test_small_runs_vs_oracle():
    """Many interior/edge run boundaries (48-frame runs) against the oracle."""
    torch, E = _engine()
    sr, N = 48000, 48000 * 12 + 333
    x = synth_stream(9, N, 2, sr)
    outs, sts, _ = _run(E, torch, [x], sr, {"TOMATIS_RUN_FRAMES": 48},
                        gate_ui=50, n_fft=2048, hop=512)
    ref = orc.process_standard(x, sr, gate_ui=50, n_fft=2048, hop=512)
    assert np.array_equal(sts[0], ref["states"])
    m = ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3
    err = np.abs(outs[0][m] - ref["y"][m])
    assert float(err.max()) <= 1e-4


@pytest.mark.parametrize("n_fft,hop,sr,xfade_ms", [(2048, 512, 48000, 500.0), (4096, 1024, 96000, 500.0),
                                                   (2048, 512, 44100, 0.0), (4096, 2048, 48000, 30.0)])
def test_xfade_alpha_parallel_matches_sequential(n_fft, hop, sr, xfade_ms):
    """The three-pass segment-parallel alpha scan equals the sequential float64
    recurrence bit for bit (alpha, gain rows, hence samples)."""
    torch, E = _engine()
    lens = [sr * 200 + 11, sr * 45 + 777]
    xs = [synth_stream(900 + i, n, 2, sr) for i, n in enumerate(lens)]

    def run(env):
        with _dev(env):
            ss = E.StreamSet.from_arrays(xs, sr)
            pipe = E.GatePipeline(ss, gate_ui=50, gate_offset=-90, n_fft=n_fft, hop=hop,
                                  xfade_ms=xfade_ms)
            res = pipe.run()
            torch.cuda.synchronize()
            return ([res.stream_alpha(i) for i in range(len(xs))],
                    [res.output(i) for i in range(len(xs))],
                    pipe.rows[:pipe.plan.total_frames].cpu().numpy())

    a_seq, y_seq, r_seq = run({"TOMATIS_ALPHA_SEQ": 1})
    a_par, y_par, r_par = run({})
    assert np.array_equal(r_par, r_seq)
    for i in range(len(xs)):
        assert a_par[i].tobytes() == a_seq[i].tobytes()
        assert y_par[i].tobytes() == y_seq[i].tobytes()


def test_xfade_alpha_unsynced_segments():
    """States that flip faster than the cross-fade can settle (every 0.2 s
    against xf + 2 = 49 frames) leave whole alpha segments without a sync
    frame: k_alpha_chain walks them from their carry-in, in segment order.
    Equal to the sequential float64 recurrence bit for bit."""
    torch, E = _engine()
    sr, n_fft, hop = 48000, 2048, 512
    rng = np.random.default_rng(5)
    xs = []
    for n in (sr * 60 + 123, sr * 25 + 7):
        t = np.arange(n)
        env = np.where((t // int(0.2 * sr)) % 2 == 0, 10 ** (-20 / 20), 10 ** (-60 / 20))
        env[2 * n // 3:] = 10 ** (-20 / 20)  # then steady: segments sync again
        xs.append((rng.standard_normal((n, 2)) * env[:, None] * 0.5).astype(np.float32))

    def run(env):
        with _dev(env):
            ss = E.StreamSet.from_arrays(xs, sr)
            pipe = E.GatePipeline(ss, gate_ui=50, gate_offset=-90, n_fft=n_fft, hop=hop,
                                  xfade_ms=500.0, up_delay_ms=10.0)
            res = pipe.run()
            torch.cuda.synchronize()
            return ([res.stream_alpha(i) for i in range(len(xs))],
                    [res.stream_states(i) for i in range(len(xs))])

    a_seq, s_seq = run({"TOMATIS_ALPHA_SEQ": 1})
    a_par, s_par = run({})
    flips = int(np.count_nonzero(np.diff(s_seq[0].astype(np.int8))))
    assert flips > 100, flips  # the states do flip faster than the fade settles
    for i in range(len(xs)):
        assert np.array_equal(s_par[i], s_seq[i])
        assert a_par[i].tobytes() == a_seq[i].tobytes()
