"""GPU gate calibration against the reference golden:
levels bit-exact, band tilts within float32 FFT rounding, simulate_state and
the whole calibrate_to_baseline_v2 result (the `best` grid point, gate_offset,
delay) identical to the reference's JSON."""
import json
import os

import numpy as np
import pytest

from tests.golden.calib_case import CASE, make_inputs
from tests.test_calibration import fixture

pytestmark = pytest.mark.gpu


def _cal():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import calibrate_to_baseline_v2 as cal
    return cal


def _inputs(fx):
    from tests.golden_util import sha
    xo, xb = make_inputs()
    assert [sha(xo), sha(xb)] == [str(s) for s in fx["in_sha"]], "input generator drifted"
    return xo, xb


def test_levels_tilts_and_states():
    cal = _cal()
    fx = fixture()
    xo, xb = _inputs(fx)
    d = int(fx["delay"])
    sr, n_fft, hop = CASE["sr"], CASE["n_fft"], CASE["hop"]
    bs, os_ = max(0, -d), max(0, d)
    avail = min(len(xb) - bs, len(xo) - os_, int(CASE["max_minutes"] * 60 * sr))
    ol = cal.frame_levels(xo[os_:os_ + avail], n_fft, hop)
    bl = cal.frame_levels(xb[bs:bs + avail], n_fft, hop)
    np.testing.assert_array_equal(ol.view(np.uint32), fx["orig_level"].view(np.uint32))
    np.testing.assert_array_equal(bl.view(np.uint32), fx["base_level"].view(np.uint32))
    ti = cal.band_tilts(xb[bs:bs + avail], sr, n_fft, hop)
    assert np.abs(ti - fx["tilts"]).max() < 1e-3
    idx = np.flatnonzero(fx["music_mask"])
    fs = (np.arange(len(ol)) * hop).astype(np.int64)[idx]
    for (g, T, hy, up), ref in zip(fx["sim_params"], fx["sim_states"]):
        got = cal.simulate_state((fx["orig_level"] + np.float32(g))[idx], fs, sr, T, hy, up)
        np.testing.assert_array_equal(got, ref)


def test_calibrate_matches_reference_json(tmp_path):
    cal = _cal()
    from tomatis_audio_processor_amd import audio_io
    fx = fixture()
    xo, xb = _inputs(fx)
    po, pb = str(tmp_path / "orig.wav"), str(tmp_path / "base.wav")
    audio_io.write(po, xo, CASE["sr"], "WAV", "FLOAT")
    audio_io.write(pb, xb, CASE["sr"], "WAV", "FLOAT")
    out_json = str(tmp_path / "cal.json")
    cal.main(["--orig", po, "--base", pb, "--out_json", out_json] + CASE["argv"])
    got = json.load(open(out_json, encoding="utf-8"))
    ref = json.loads(str(fx["json"]))
    for k in ("orig", "base"):
        got.pop(k)
        ref.pop(k)
    assert got == ref
