#!/usr/bin/env python3
"""Generate the golden parity fixtures under ``tests/golden/`` by running the
REFERENCE (``/root/reference/src``) on seeded synthetic inputs.

Build-container only (``/root/reference`` does not exist on the GPU box).  The
reference modules import ``soundfile`` at top level; it is not installed here,
so ``tools/_sf_stub`` provides an in-memory stand-in that serves the input
arrays and captures written float chunks before PCM quantisation.  Nothing of
the reference is copied: fixtures hold only parameters, seeds, hashes of the
reference's float outputs, decimated output samples, chunk lengths and the
reference's own state-CSV columns.

Usage:  python tools/make_goldens.py [--only NAME]
"""
from __future__ import annotations

import argparse
import csv
import hashlib
import importlib
import io
import json
import os
import sys
import tempfile
import contextlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF_SRC = "/root/reference/src"
OUT_DIR = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, os.path.join(HERE, "_sf_stub"))
sys.path.insert(0, REPO)
import soundfile as sfstub  # noqa: E402  (the stand-in)
from tomatis_audio_processor_amd.synth import synth_stream  # noqa: E402
from tests.golden.cases import CASES, eq_csv_rows, diff_csv_rows  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load_ref(modname):
    if REF_SRC not in sys.path:
        sys.path.insert(1, REF_SRC)
    return importlib.import_module(modname)


def case_input(c):
    x = synth_stream(c["seed"], c["N"], c["ch"], c["sr"])
    if c.get("in_scale") is not None:
        x = (x * np.float32(c["in_scale"])).astype(np.float32)
    if c.get("silence"):
        k = int(c["silence"])
        x[:k] = 0.0
        x[len(x) - k:] = 0.0
    return x


def read_csv(path):
    with open(path, newline="", encoding="utf-8") as f:
        rows = list(csv.reader(f))
    return rows[0], rows[1:]


def run_case(c, tmp):
    sfstub.GUARD_BYPASS = bool(c.get("bypass", False))
    sfstub.STORE.clear()
    sfstub.WRITES.clear()
    x = case_input(c)
    inp = os.path.join(tmp, "in.flac")
    out = os.path.join(tmp, "out.flac")
    sfstub.STORE[inp] = (x, c["sr"])
    p = dict(c["params"])
    res = {}
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        if c["mode"] in ("standard", "xfade"):
            mod = load_ref("process_tomatis" if c["mode"] == "standard"
                           else "process_tomatis_xfade")
            st_csv = os.path.join(tmp, "state.csv")
            mod.process(inp, out, state_csv_path=st_csv, **p)
            chunks = sfstub.WRITES[out]
            y = np.concatenate(chunks) if chunks else np.zeros((0, c["ch"]), np.float32)
            res["chunk_lens"] = np.array([len(q) for q in chunks], np.int64)
            hdr, rows = read_csv(st_csv)
            res["csv_frame_idx"] = np.array([int(r[0]) for r in rows], np.int64)
            res["csv_state"] = np.array([1 if r[3] == "C1" else 2 for r in rows], np.uint8)
            if c["mode"] == "standard":
                # level written with repr(): the exact float value
                res["csv_level"] = np.array([float(r[2]) for r in rows], np.float64)
            else:
                res["csv_level_2f"] = np.array([r[2] for r in rows])
                res["csv_alpha_3f"] = np.array([r[4] for r in rows])
        elif c["mode"] == "adaptive":
            mod = load_ref("process_tomatis_adaptive")
            st_csv = os.path.join(tmp, "state.csv")
            mod.process(inp, out, state_csv_path=st_csv, **p)
            y = np.asarray(sfstub.WRITES[out][0])
            hdr, rows = read_csv(st_csv)
            res["csv_state"] = np.array([1 if r[3] == "C1" else 2 for r in rows], np.uint8)
            res["csv_level_4f"] = np.array([r[2] for r in rows])
            res["csv_alpha_4f"] = np.array([r[4] for r in rows])
            res["csv_time_6f"] = np.array([r[1] for r in rows])
        elif c["mode"] == "layer2":
            mod = load_ref("layer2_apply_eq")
            eq = os.path.join(tmp, "eq.csv")
            text = eq_csv_rows(c)
            res["eq_csv"] = np.array(text)
            with open(eq, "w", newline="") as f:
                f.write(text)
            mod.apply_eq_stft(inp, out, eq, **p)
            chunks = sfstub.WRITES[out]
            y = np.concatenate(chunks)
            gp = out.replace(".flac", "_gp.flac")
            if gp in sfstub.WRITES:
                ygp = np.concatenate(sfstub.WRITES[gp])
                res["gp_sha"] = np.array(sha(ygp))
                res["gp_sub"] = ygp[::max(1, len(ygp) // 1500)]
        elif c["mode"] in ("layer2b", "layer2b_safe"):
            modname = ("layer2b_apply_residual_eq" if c["mode"] == "layer2b"
                       else "layer2b_apply_residual_eq_safe")
            mod = load_ref(modname)
            dcsv = os.path.join(tmp, "diff_spectrum.csv")
            text = diff_csv_rows(c)
            res["diff_csv"] = np.array(text)
            with open(dcsv, "w", newline="") as f:
                f.write(text)
            argv = ["x", "--in_audio", inp, "--out_audio", out, "--diff_csv", dcsv]
            for k, v in p.items():
                argv += [f"--{k}", str(v)]
            old = sys.argv
            sys.argv = argv
            try:
                mod.main()
            finally:
                sys.argv = old
            chunks = sfstub.WRITES.get(out, [])
            y = np.concatenate(chunks) if chunks else np.zeros((0, c["ch"]), np.float32)
        else:
            raise ValueError(c["mode"])
    res["out_sha"] = np.array(sha(y))
    res["out_dtype"] = np.array(str(y.dtype))
    res["out_shape"] = np.array(y.shape, np.int64)
    step = max(1, len(y) // 2000)
    res["out_step"] = np.array(step, np.int64)
    res["out_sub"] = y[::step]
    res["in_sha"] = np.array(sha(x))
    res["meta"] = np.array(json.dumps(c))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    os.makedirs(OUT_DIR, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        for c in CASES:
            if a.only and c["name"] != a.only:
                continue
            res = run_case(c, tmp)
            np.savez_compressed(os.path.join(OUT_DIR, c["name"] + ".npz"), **res)
            print(f"{c['name']:32s} out={tuple(res['out_shape'])} {res['out_dtype']}"
                  f" chunks={res.get('chunk_lens', [])}")


if __name__ == "__main__":
    main()
