"""Pin the oracle: it must reproduce the reference's golden vectors bit-exactly.

Fixtures were produced by running the reference itself (tools/make_goldens.py).
"""
import numpy as np
import pytest

from tests.golden_util import (CASES, load_fixture, case_input, run_oracle, sha,
                               std_chunk_lens)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference(case):
    fx = load_fixture(case["name"])
    x = case_input(case)
    assert sha(x) == str(fx["in_sha"]), "synthetic input generator drifted"
    res = run_oracle(case, fx, x)
    y = res["y"]
    assert tuple(y.shape) == tuple(fx["out_shape"])
    assert str(y.dtype) == str(fx["out_dtype"])
    step = int(fx["out_step"])
    np.testing.assert_array_equal(y[::step], fx["out_sub"])
    assert sha(y) == str(fx["out_sha"]), "oracle output not bit-exact with reference"
    mode = case["mode"]
    if mode in ("standard", "xfade"):
        N = case["N"]
        lens = std_chunk_lens(res["bounds"], N)
        np.testing.assert_array_equal(lens, fx["chunk_lens"])
        m = (res["starts"] >= 0) & (res["starts"] < N)
        np.testing.assert_array_equal(np.nonzero(m)[0], fx["csv_frame_idx"])
        np.testing.assert_array_equal(res["states"][m], fx["csv_state"])
        if mode == "standard":
            np.testing.assert_array_equal(res["levels"][m], fx["csv_level"])
        else:
            np.testing.assert_array_equal(
                np.array([f"{v:.2f}" for v in res["levels"][m]]), fx["csv_level_2f"])
            np.testing.assert_array_equal(
                np.array([f"{v:.3f}" for v in res["alpha"][m]]), fx["csv_alpha_3f"])
    elif mode == "adaptive":
        np.testing.assert_array_equal(res["states"], fx["csv_state"])
        np.testing.assert_array_equal(
            np.array([f"{v:.4f}" for v in res["levels"]]), fx["csv_level_4f"])
        np.testing.assert_array_equal(
            np.array([f"{v:.4f}" for v in res["alpha"]]), fx["csv_alpha_4f"])
    elif mode == "layer2" and "gp_sha" in fx:
        assert res["y_gp"] is not None
        assert sha(res["y_gp"]) == str(fx["gp_sha"])
