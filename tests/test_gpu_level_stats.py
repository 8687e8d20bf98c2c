"""tomatis_level_stats (adaptive threshold statistics on the device) against
numpy's np.percentile(valid, 5/95) and np.median(valid), bitwise
(src/process_tomatis_adaptive.py:123-131), on crafted level arrays: ties,
all-invalid streams (median of every level), one and two valid levels, odd and
even counts, -70 exactly (invalid), and a stream without frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _numpy_stats(lv):
    valid = lv[lv > -70]
    if len(lv) == 0:
        return np.array([np.nan, np.nan, 0.0])
    if len(valid) == 0:
        return np.array([np.nan, np.nan, np.median(lv)])
    return np.array([np.percentile(valid, 5), np.percentile(valid, 95), np.median(valid)])


def test_level_stats_bitwise():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import dsp, engine
    from tomatis_audio_processor_amd._lib import check, lib, ptr, stream_handle
    n_fft, hop, sr = 2048, 512, 44100
    # lengths giving a spread of frame counts, incl. a stream too short for a frame
    lens = [40000, 40512, 300000, 2047, 1000000, 60000, 61000, 90000, 44100 * 30]
    rng = np.random.default_rng(7)
    arrays = [rng.standard_normal((n, 2)).astype(np.float32) * 0.1 for n in lens]
    ss = engine.StreamSet.from_arrays(arrays, sr)
    pipe = engine.AdaptivePipeline(ss, n_fft=n_fft, hop=hop)
    sts = pipe.plan.streams
    Ft = pipe.plan.total_frames
    lv = np.empty(Ft, np.float64)
    for i in range(len(lens)):
        a, F = sts[i].frame_base, sts[i].n_frames
        assert F == dsp.adaptive_frames(lens[i], n_fft, hop)[1]
        v = rng.normal(-40, 15, F)
        if i == 0:
            v = np.round(v * 2) / 2                   # heavy ties
        elif i == 1:
            v = rng.uniform(-120, -70, F)             # no valid level (-70 is invalid)
            v[::7] = -70.0
        elif i == 2:
            v[:] = -90.0
            v[F // 3] = -12.5                         # one valid level
        elif i == 4:
            v[:] = -80.0
            v[5], v[F - 1] = 3.0, -69.999             # two valid levels
        elif i == 5:
            v[v < -55] = -70.0
        elif i == 6:
            v = np.full(F, -33.25)                    # all equal
        elif i == 7:
            v = -v                                    # mixed signs, -0.0 impossible
        lv[a:a + F] = v
    pipe.levels[:Ft].copy_(torch.from_numpy(lv))
    check(lib().tomatis_level_stats(pipe.plan.h, ptr(pipe.levels), ptr(pipe._tlh),
                                    stream_handle()), "level_stats")
    got = pipe._tlh.cpu().numpy().reshape(-1, 3)
    for i in range(len(lens)):
        a, F = sts[i].frame_base, sts[i].n_frames
        want = _numpy_stats(lv[a:a + F])
        assert np.array_equal(got[i].view(np.uint64), want.view(np.uint64)) or (
            np.array_equal(np.isnan(got[i]), np.isnan(want))
            and np.array_equal(got[i][~np.isnan(want)].view(np.uint64),
                               want[~np.isnan(want)].view(np.uint64))), (i, F, got[i], want)
        assert np.array_equal(dsp.level_stats(lv[a:a + F][lv[a:a + F] > -70]), want) \
            if (lv[a:a + F] > -70).any() else True


def test_minhold_speculative_equals_serial_and_oracle():
    """tomatis_minhold_bisect's speculative rounds (7 tree midpoints per launch,
    TOMATIS_OPT_MINHOLD_SERIAL = 0) against the serial 30-step loop (= 1):
    thresholds, states, rows and alpha bit-identical, and the thresholds equal
    the oracle's find_optimal_threshold (src/process_tomatis_adaptive.py:
    133-154) — on streams that exit early, run all 30 steps, have no valid
    level, no frames, or a constant level."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd import engine
    from tomatis_audio_processor_amd._lib import OPT_MINHOLD_SERIAL, check, lib, ptr, stream_handle
    n_fft, hop, sr = 2048, 512, 44100
    lens = [44100 * 60, 2047, 44100 * 20, 300000, 44100 * 45, 90000, 44100 * 120]
    rng = np.random.default_rng(11)
    arrays = [np.zeros((n, 2), np.float32) for n in lens]
    ss = engine.StreamSet.from_arrays(arrays, sr)
    pipe = engine.AdaptivePipeline(ss, n_fft=n_fft, hop=hop)
    sts = pipe.plan.streams
    Ft = pipe.plan.total_frames
    lv = np.empty(Ft, np.float64)
    for i in range(len(lens)):
        a, F = sts[i].frame_base, sts[i].n_frames
        # alternating loud / quiet blocks (the gate's real input) + noise
        blk = rng.integers(20, 400, size=F // 20 + 2)
        v = np.repeat(np.where(np.arange(len(blk)) % 2 == 0, -25.0, -55.0), blk)[:F]
        v = v + rng.normal(0, 4, F)
        if i == 2:
            v = rng.uniform(-120, -71, F)             # no valid level
        elif i == 3:
            v = np.full(F, -33.25)                    # constant: c2 jumps 0 <-> 1
        elif i == 5:
            v = np.round(v)                           # ties
        lv[a:a + F] = v
    pipe.levels[:Ft].copy_(torch.from_numpy(lv))
    L, hs = lib(), stream_handle()
    check(L.tomatis_level_stats(pipe.plan.h, ptr(pipe.levels), ptr(pipe._tlh), hs), "stats")
    outs = []
    for serial in (1, 0):
        pipe.plan.set_option(OPT_MINHOLD_SERIAL, serial)
        pipe.states.zero_()
        pipe.rows.zero_()
        pipe.alpha.zero_()
        check(L.tomatis_minhold_bisect(pipe.plan.h, ptr(pipe.levels), ptr(pipe._tlh),
                                       pipe.target_c2, pipe.hyst_db, ptr(pipe.t_out),
                                       ptr(pipe.states), ptr(pipe.rows), ptr(pipe.alpha), hs),
              "minhold_bisect")
        torch.cuda.synchronize()
        outs.append([t.cpu().numpy().copy() for t in (pipe.t_out, pipe.states, pipe.rows,
                                                       pipe.alpha)])
    for a, b in zip(*outs):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
    t = outs[1][0]
    mh = pipe.mh
    for i in range(len(lens)):
        a, F = sts[i].frame_base, sts[i].n_frames
        if F == 0:
            continue
        x = lv[a:a + F]
        want = orc.optimal_threshold(x, x > -70, pipe.hyst_db, mh, pipe.target_c2)
        assert float(t[i]) == float(want), (i, t[i], want)
