"""Gate calibration: host pieces against the reference
golden (tests/golden/calib_v2.npz, made by tools/make_calib_goldens.py by
running src/calibrate_to_baseline_v2.py itself)."""
import json
import os

import numpy as np
import pytest

from tests.golden_util import GOLDEN_DIR
from tomatis_audio_processor_amd import calibrate_to_baseline_v2 as cal


def fixture():
    with np.load(os.path.join(GOLDEN_DIR, "calib_v2.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_debounce_matches_reference():
    fx = fixture()
    np.testing.assert_array_equal(cal.debounce_state(fx["deb_in"], 3), fx["deb_out"])
    np.testing.assert_array_equal(cal.debounce_state(fx["base_state_raw"], 3), fx["base_state"])


@pytest.mark.parametrize("seq", [[1], [2, 1, 1, 1], [1, 2, 2, 1, 1, 1, 2], [2, 2, 1, 2, 2, 2, 1, 1]])
def test_debounce_edge_runs(seq):
    """Short leading / trailing / whole-sequence runs, against the reference's
    sequential rule restated literally."""
    def literal(state, min_run=3):
        s = np.array(state).copy()
        n, i = len(s), 0
        while i < n:
            j = i + 1
            while j < n and s[j] == s[i]:
                j += 1
            if j - i < min_run:
                s[i:j] = s[i - 1] if i > 0 else s[j] if j < n else s[i]
            i = j
        return s
    np.testing.assert_array_equal(cal.debounce_state(np.array(seq), 3), literal(seq))


def test_kmeans_state_split_matches_reference():
    from scipy.signal import medfilt
    fx = fixture()
    ts = medfilt(fx["tilts"], kernel_size=5).astype(np.float32)
    mm = fx["music_mask"]
    lab, _, _ = cal.kmeans2_1d(ts[mm])
    st = np.ones(len(ts), np.int32)
    st[mm] = np.where(lab == 1, 2, 1)
    m1 = float(np.mean(ts[mm][lab == 1]))
    m0 = float(np.mean(ts[mm][lab == 0]))
    if m0 > m1:
        st[mm] = np.where(lab == 0, 2, 1)
    np.testing.assert_array_equal(st, fx["base_state_raw"])


def test_golden_json_is_self_consistent():
    js = json.loads(str(fixture()["json"]))
    assert js["T_raw_dbfs"] == js["T_adj_dbfs"] - js["gain_db_base_minus_orig"]
    assert js["gate_offset"] == js["T_raw_dbfs"] - js["gate_scale"] * js["gate_ui"]
