"""Helpers shared by the oracle-vs-golden and GPU parity tests."""
from __future__ import annotations

import csv
import hashlib
import io
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from tomatis_audio_processor_amd.synth import synth_stream  # noqa: E402
from tests.golden.cases import CASES, BY_NAME  # noqa: E402

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load_fixture(name: str) -> dict:
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as z:
        fx = {k: z[k] for k in z.files}
    fx["meta"] = json.loads(str(fx["meta"]))
    return fx


def case_input(c: dict) -> np.ndarray:
    x = synth_stream(c["seed"], c["N"], c["ch"], c["sr"])
    if c.get("in_scale") is not None:
        x = (x * np.float32(c["in_scale"])).astype(np.float32)
    if c.get("silence"):
        k = int(c["silence"])
        x[:k] = 0.0
        x[len(x) - k:] = 0.0
    return x


def parse_eq_csv(text: str):
    """Same parsing as src/layer2_apply_eq.py:11-46 (float32, sorted)."""
    rd = csv.DictReader(io.StringIO(text))
    cols = [c.lower().strip() for c in rd.fieldnames]
    f_col = next(c for c in ["freq_hz", "freq", "hz", "f"] if c in cols)
    d_col = next(c for c in ["delta_db_smooth", "delta_db", "db", "gain_db",
                             "delta", "gain"] if c in cols)
    fr, db = [], []
    for row in rd:
        fr.append(float(row[f_col]))
        db.append(float(row[d_col]))
    fr = np.array(fr, np.float32)
    db = np.array(db, np.float32)
    idx = np.argsort(fr)
    return fr[idx], db[idx]


def parse_diff_csv(text: str):
    """Same parsing as src/layer2b_apply_residual_eq.py:72-76 (pandas, float32)."""
    import pandas as pd
    d = pd.read_csv(io.StringIO(text))
    col = ("delta_db_base_minus_cand" if "delta_db_base_minus_cand" in d.columns
           else "delta_db")
    return d["freq_hz"].to_numpy(np.float32), d[col].to_numpy(np.float32)


def run_oracle(c: dict, fx: dict | None = None, x: np.ndarray | None = None) -> dict:
    """Run the oracle processor matching case ``c``."""
    from oracle import tomatis_oracle as orc
    if x is None:
        x = case_input(c)
    p = dict(c["params"])
    mode = c["mode"]
    if mode == "standard":
        if "hysteresis_db" in p:
            p["hysteresis_db"] = p.pop("hysteresis_db")
        return orc.process_standard(x, c["sr"], **p)
    if mode == "xfade":
        p.setdefault("xfade_ms", 0.0)
        return orc.process_standard(x, c["sr"], **p)
    if mode == "adaptive":
        return orc.process_adaptive(x, c["sr"], **p)
    if mode == "layer2":
        fr, db = parse_eq_csv(str(fx["eq_csv"]))
        return orc.apply_eq_stft(x, c["sr"], fr, db, **p)
    if mode in ("layer2b", "layer2b_safe"):
        rf, rd = parse_diff_csv(str(fx["diff_csv"]))
        safe = mode == "layer2b_safe"
        q = dict(smooth_win=61 if safe else 41, clamp_hi=1.0 if safe else 6.0,
                 hf_start=3000.0 if safe else 8000.0)
        q.update(p)
        return orc.apply_residual_eq(x, c["sr"], rf, rd, safe=safe, **q)
    raise ValueError(mode)


def std_chunk_lens(bounds, N):
    out = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        s, e = max(0, int(a)), min(N, int(b))
        if e > s:
            out.append(e - s)
    return np.array(out, np.int64)


def csv_frame_mask(starts, N):
    return (starts >= 0) & (starts < N)


__all__ = ["CASES", "BY_NAME", "sha", "load_fixture", "case_input", "run_oracle",
           "parse_eq_csv", "parse_diff_csv", "std_chunk_lens", "csv_frame_mask"]
