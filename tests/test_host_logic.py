"""Host-side logic of the product vs the oracle (no GPU needed)."""
import os

import numpy as np
import pytest

from oracle import tomatis_oracle as orc
from tomatis_audio_processor_amd import audio_io, dsp, sharding
from tomatis_audio_processor_amd.synth import synth_stream


@pytest.mark.parametrize("n_fft,hop", [(2048, 512), (4096, 2048), (4096, 1024), (2048, 300),
                                       (2048, 2048), (4096, 4096)])
def test_flush_bounds_match_reference_rule(n_fft, hop):
    rng = np.random.default_rng(n_fft + hop)
    for N in list(rng.integers(1, 2_000_000, 40)) + [n_fft, n_fft + 1, 240000, 1234567]:
        assert dsp.std_flush_bounds(int(N), n_fft, hop) == orc.std_chunk_bounds(int(N), n_fft, hop)


@pytest.mark.parametrize("n_fft,hop", [(2048, 512), (4096, 2048), (4096, 1024), (2048, 300)])
def test_schedules(n_fft, hop):
    for N in [1, 100, n_fft - 1, n_fft, n_fft + 1, 48000, 441000, 12345]:
        pad, pe, F, s0 = dsp.std_schedule(N, n_fft, hop)
        opad, ope, oF, ostarts = orc._std_schedule(N, n_fft, hop)
        assert (pad, pe, F) == (opad, ope, oF)
        k0, Fa, sa = dsp.adaptive_frames(N, n_fft, hop)
        xp = N + 2 * (n_fft // 2)
        n_all = (xp - n_fft) // hop + 1 if xp >= n_fft else 0
        valid = [k for k in range(n_all) if 0 <= k * hop - n_fft // 2 < N]
        assert Fa == len(valid)
        if valid:
            assert (k0, sa) == (valid[0], valid[0] * hop - n_fft // 2)


def test_tables_bit_identical_to_oracle():
    for sr in (44100, 48000, 96000):
        for n_fft in (2048, 4096):
            f = np.fft.rfftfreq(n_fft, d=1.0 / sr)
            for lo, hi in [(15.0, -15.0), (-15.0, 15.0), (6.0, 0.0), (-3.0, -3.0)]:
                a = dsp.build_tilt_gain_db(f, 1000.0, 12.0, lo, hi)
                b = orc.tilt_gain_db(f, 1000.0, 12.0, lo, hi)
                assert a.tobytes() == b.tobytes()
                assert dsp.db_to_lin(a).tobytes() == orc.db_to_lin_f32(b).tobytes()
    assert dsp.hann(2048).tobytes() == orc.hann_sym(2048)[0].tobytes()


@pytest.mark.parametrize("Ton,Toff", [(-38.5, -41.5), (-40.0, -40.0), (-61.08, -64.08),
                                      (-5.0, -8.0), (-119.9, -122.9)])
def test_gate_bits_exact(Ton, Toff):
    on, oe, off, fe = dsp.gate_bits(Ton, Toff)
    rng = np.random.default_rng(7)
    lo = np.float32(1e-6).view(np.uint32)
    b = np.concatenate([rng.integers(int(lo), 0x3F800000, 300000),
                        np.arange(max(0, on - 20000), on + 20000),
                        np.arange(max(0, off - 20000), off + 20000)]).astype(np.uint32)
    lv = orc.r_to_level(b.view(np.float32))
    assert np.array_equal((b >= on) ^ np.isin(b, oe), lv >= Ton)
    assert np.array_equal((b <= off) ^ np.isin(b, fe), lv <= Toff)


def test_wav_roundtrip(tmp_path):
    x = synth_stream(3, 4800, 2, 48000)
    p = str(tmp_path / "a.wav")
    audio_io.write(p, x, 48000, "WAV", "PCM_24")
    y, sr = audio_io.read(p)
    assert sr == 48000 and y.shape == x.shape
    assert np.max(np.abs(y - x)) <= 1.0 / 8388607
    assert audio_io.info(p) == (48000, 2, 4800)
    q = str(tmp_path / "b.wav")
    audio_io.write(q, x, 44100, "WAV", "FLOAT")
    z, _ = audio_io.read(q)
    assert np.array_equal(z, x)


def test_flac_fallback_to_wav(tmp_path, monkeypatch):
    if audio_io.have_soundfile():
        pytest.skip("libsndfile present: FLAC is written directly")

    def fail(*a, **k):
        raise audio_io.AudioFormatError("encoder unavailable")
    monkeypatch.setattr(audio_io, "_write_flac", fail)  # reference branch :242-251
    x = synth_stream(4, 1000, 2, 48000)
    out = str(tmp_path / "o.flac")
    path, is_flac = audio_io.write_with_fallback(out, x, 48000, log=lambda m: None)
    assert not is_flac and path == out.replace(".flac", ".wav") and os.path.exists(path)


def test_guard_messages():
    from tomatis_audio_processor_amd.process_tomatis import check_format
    with pytest.raises(ValueError, match="期望 48kHz，实际 44100 Hz"):
        check_format(44100, 2, False)
    with pytest.raises(ValueError, match="期望双声道，实际 1 声道"):
        check_format(48000, 1, False)
    check_format(44100, 1, True)


def test_cli_flags_and_defaults():
    """Flags/defaults of src/process_tomatis.py:488-515, _xfade.py:368-391,
    _adaptive.py:378-399, layer2_apply_eq.py:241-248, layer2b*.py:58-70."""
    from tomatis_audio_processor_amd import (process_tomatis as std, process_tomatis_xfade as xf,
                                             process_tomatis_adaptive as ad,
                                             layer2b_apply_residual_eq as l2b)
    a = std.build_parser().parse_args(["-i", "a", "-o", "b"])
    assert (a.gate_ui, a.gate_mode, a.dynamic_range, a.gate_scale, a.gate_offset, a.hyst_db,
            a.up_delay_ms, a.fc, a.slope, a.c1_low, a.c1_high, a.c2_low, a.c2_high, a.n_fft,
            a.hop, a.state_csv, a.output_gain_db) == (50, "log_percent", 80.0, 1.0, -100, 3.0,
                                                      250.0, 1000.0, 12.0, 15.0, -15.0, -15.0,
                                                      15.0, 4096, 2048, None, 0.0)
    b = xf.build_parser().parse_args(["-i", "a", "-o", "b"])
    assert (b.xfade_ms, b.gate_offset, b.n_fft, b.hop) == (0.0, -100, 4096, 2048)
    assert not hasattr(b, "gate_mode")
    c = ad.build_parser().parse_args(["-i", "a", "-o", "b"])
    assert (c.target_c2, c.hyst_db, c.min_hold_ms, c.xfade_ms, c.headroom_margin, c.n_fft,
            c.hop) == (0.5, 3.0, 250.0, 500.0, 2.0, 4096, 2048)
    d = l2b.build_parser().parse_args(["--in_audio", "a", "--out_audio", "b"])
    assert (d.smooth_win, d.clamp_hi, d.mid_start, d.mid_clamp_hi, d.hf_start,
            d.hf_clamp_hi, d.diff_csv) == (41, 6.0, 3000.0, 2.0, 8000.0, 0.0, "diff_spectrum.csv")
    e = l2b.build_parser(safe=True).parse_args(["--in_audio", "a", "--out_audio", "b"])
    assert (e.smooth_win, e.clamp_hi, e.hf_start) == (61, 1.0, 3000.0)


def test_eq_helpers_match_oracle():
    from tests.golden_util import load_fixture, parse_eq_csv, parse_diff_csv
    fx = load_fixture("l2_48k_st_pad_gp")
    fr, db = parse_eq_csv(str(fx["eq_csv"]))
    assert dsp.build_gain_per_bin(48000, 2048, fr, db).tobytes() == \
        orc.eq_gain_per_bin(48000, 2048, fr, db).tobytes()
    fx = load_fixture("l2b_96k_st_4096_1024")
    rf, rd = parse_diff_csv(str(fx["diff_csv"]))
    s1 = dsp.smooth_on_logfreq(rf, rd, 41)
    assert s1.tobytes() == orc.smooth_on_logfreq(rf, rd, 41).tobytes()
    f = np.fft.rfftfreq(4096, 1 / 96000)
    assert dsp.build_eq_from_residual(f, rf, s1)[0].tobytes() == \
        orc.eq_from_residual(f, rf, s1)[0].tobytes()
    assert dsp.build_eq_from_residual_safe(f, rf, s1)[0].tobytes() == \
        orc.eq_from_residual(f, rf, s1, clamp_lo=-1.0, clamp_hi=1.0, hf_start=3000.0,
                             safe=True)[0].tobytes()


def test_lpt_partition():
    costs = [5, 5, 5, 5, 9, 1, 1, 3]
    parts = sharding.lpt_partition(costs, 3)
    assert sorted(sum(parts, [])) == list(range(len(costs)))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)
    eq = sharding.lpt_partition([10] * 512, 8)
    assert [len(p) for p in eq] == [64] * 8


def test_alpha_lattice_endpoints():
    from tomatis_audio_processor_amd.engine import _alpha_lattice
    for xf in (1, 3, 22, 47):
        lat = _alpha_lattice(xf)
        assert len(lat) == xf + 1 and lat[0] == 0.0 and lat[-1] == 1.0
        a = 0.0
        for m in range(1, xf):
            a = a + 1.0 / xf
            assert lat[m] == a


def test_level_stats_bit_identical_to_numpy():
    """dsp.level_stats (one partition) == np.percentile 5/95 + np.median, bitwise."""
    from tomatis_audio_processor_amd import dsp
    rng = np.random.default_rng(3)
    for t in range(3000):
        n = int(rng.integers(1, 300)) if t % 2 else int(rng.integers(1, 20000))
        v = rng.standard_normal(n) * 20 - 40
        if t % 3 == 0:
            v = np.round(v, 1)  # ties
        got = np.array(dsp.level_stats(v))
        ref = np.array([np.percentile(v, 5), np.percentile(v, 95), np.median(v)])
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (n, got, ref)


def test_batch_output_names_unique():
    """Inputs with the same file name in different directories get distinct
    outputs (no silent overwrite across or within ranks)."""
    from tomatis_audio_processor_amd.batch import output_names
    names = output_names(["a/x.wav", "b/x.wav", "c/y.flac", "x.flac"], "wav")
    assert names == ["x_0_tomatis.wav", "x_1_tomatis.wav", "y_tomatis.wav", "x_3_tomatis.wav"]
    assert len(set(names)) == len(names)


def test_level_nonmonotone_steps_are_isolated():
    """Exhaustive over every finite float32 r >= 2^-20 (r >= 1e-6 always): the
    reference's level 20*log10(f32(r)+EPS) steps down at isolated points, each
    far more than gate_bits' +-8192-ulp window from the next, so no crossing
    window can hold more than one exception (the 4-entry table never overflows)."""
    lo = int(np.float32(2.0 ** -20).view(np.uint32))
    hi = 0x7F7FFFFF
    bad = []
    step = 1 << 23
    with np.errstate(over="ignore"):
        for a in range(lo, hi, step):
            b = np.arange(a, min(a + step + 1, hi + 1), dtype=np.uint32)
            lv = (20.0 * np.log10(b.view(np.float32) + 1e-12)).astype(np.float64)
            bad.extend((b[np.nonzero(lv[1:] < lv[:-1])[0]]).tolist())
    assert 0 < len(bad) < 64
    assert np.min(np.diff(np.asarray(bad, np.int64))) > 4 * 8192


def test_analysis_n_fft_bounds_host_side():
    """analysis._check_n_fft (tm_analysis.hip's limits): powers of two in
    [16, 16384], other lengths in [16, 8192] (Bluestein over >= 2n - 1 points
    in LDS); refused before any device call."""
    from tomatis_audio_processor_amd import analysis
    for ok in (16, 17, 100, 1000, 3000, 4096, 8191, 8192, 16384):
        analysis._check_n_fft(ok)
    for bad in (1, 8, 15, 8193, 9000, 12000, 16383, 32768):
        with pytest.raises(ValueError, match="n_fft"):
            analysis._check_n_fft(bad)


def test_levels_threaded_inside_host_pool_no_deadlock(monkeypatch):
    """host_levels runs on _host_pool(); its float64 branch splits the
    log10 chain into slices.  With one pool worker the slices must not queue
    behind their own caller (they run on a separate executor)."""
    import concurrent.futures as cf
    from tomatis_audio_processor_amd import dsp, engine
    monkeypatch.setenv("TOMATIS_LOG10_THREADS", "4")
    monkeypatch.setattr(engine, "_POOL", cf.ThreadPoolExecutor(max_workers=1))
    r = np.random.default_rng(3).random(1 << 17) * 0.5
    out = np.empty(len(r), np.float64)
    fut = engine._host_pool().submit(engine._levels_threaded, r, out)
    fut.result(timeout=60)
    assert np.array_equal(out, dsp.r_to_level(r))


def test_split_batches():
    """batch.py cuts a rank's files into consecutive batches within the input
    budget; an oversize file is a batch of its own; every id once, in order."""
    from tomatis_audio_processor_amd.batch import split_batches
    sizes = {0: 5, 1: 3, 2: 9, 3: 20, 4: 1, 5: 1, 6: 7}
    b = split_batches(list(range(7)), sizes, 10)
    assert b == [[0, 1], [2], [3], [4, 5, 6]]
    assert [i for x in b for i in x] == list(range(7))
    assert split_batches([], sizes, 10) == []
    assert split_batches([3], sizes, 1) == [[3]]
    assert split_batches([4, 5], sizes, 100) == [[4, 5]]
