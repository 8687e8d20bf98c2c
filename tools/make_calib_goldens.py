#!/usr/bin/env python3
"""Golden fixture for the gate calibration made by running
the REFERENCE src/calibrate_to_baseline_v2.py in the build container.

Inputs (regenerated identically by the tests): orig = synth stream (seed 61,
60 s stereo 48 kHz); base = the oracle's standard processing of orig with a
known gate (linear mapping, offset -92, hysteresis 2 dB, up-delay 100 ms,
4096/2048), attenuated 2.5 dB and delayed 1234 samples.  The reference's main()
runs on them through the in-memory soundfile stand-in; its JSON and, from its
own functions, the per-frame levels, band tilts, debounced base states and a
few simulate_state sequences are stored.  Nothing of the reference is copied.

Usage: python tools/make_calib_goldens.py
"""
import contextlib
import hashlib
import importlib
import io
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "_sf_stub"))
sys.path.insert(0, REPO)
import soundfile as sfstub  # noqa: E402
from tests.golden.calib_case import CASE, make_inputs  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    sys.path.insert(1, "/root/reference/src")
    ref = importlib.import_module("calibrate_to_baseline_v2")
    from scipy.signal import medfilt
    xo, xb = make_inputs()
    sr = CASE["sr"]
    sfstub.GUARD_BYPASS = False
    sfstub.STORE.clear()
    sfstub.STORE["orig.wav"] = (xo, sr)
    sfstub.STORE["base.wav"] = (xb, sr)
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        out_json = os.path.join(tmp, "cal.json")
        argv = ["calibrate_to_baseline_v2.py", "--orig", "orig.wav", "--base", "base.wav",
                "--out_json", out_json] + CASE["argv"]
        old = sys.argv
        sys.argv = argv
        buf = io.StringIO()
        try:
            with contextlib.redirect_stdout(buf):
                ref.main()
        finally:
            sys.argv = old
        res["json"] = np.array(open(out_json, encoding="utf-8").read())
        res["stdout"] = np.array(buf.getvalue())
    js = json.loads(str(res["json"]))
    delay = js["delay_samples_orig_minus_base"]
    # the per-frame arrays main() builds, from the reference's own functions
    n_fft, hop = CASE["n_fft"], CASE["hop"]
    bs, os_ = max(0, -delay), max(0, delay)
    avail = min(len(xb) - bs, len(xo) - os_, int(CASE["max_minutes"] * 60 * sr))
    xbs, xos = xb[bs:bs + avail], xo[os_:os_ + avail]
    F = 1 + (avail - n_fft) // hop
    ol = np.zeros(F, np.float32)
    bl = np.zeros(F, np.float32)
    ti = np.zeros(F, np.float32)
    for i in range(F):
        st = i * hop
        ol[i] = ref.rms_dbfs_from_mono(ref.power_mono(xos[st:st + n_fft]))
        bl[i] = ref.rms_dbfs_from_mono(ref.power_mono(xbs[st:st + n_fft]))
        ti[i] = ref.stft_band_tilt(xbs[st:st + n_fft], sr, n_fft)
    mm = bl > -65.0
    ts = medfilt(ti, kernel_size=5).astype(np.float32)
    lab, _, _ = ref.kmeans2_1d(ts[mm])
    bstate = np.ones(F, np.int32)
    bstate[mm] = np.where(lab == 1, 2, 1).astype(np.int32)
    m1 = float(np.mean(ts[mm][lab == 1])) if np.any(lab == 1) else -1e9
    m0 = float(np.mean(ts[mm][lab == 0])) if np.any(lab == 0) else -1e9
    if m0 > m1:
        bstate[mm] = np.where(lab == 0, 2, 1).astype(np.int32)
    res["base_state_raw"] = bstate.copy()
    res["base_state"] = ref.debounce_state(bstate, min_run=3)
    res.update(orig_level=ol, base_level=bl, tilts=ti, music_mask=mm, delay=np.array(delay),
               in_sha=np.array([sha(xo), sha(xb)]))
    # simulate_state on the fitted frames for a few parameter sets
    idx = np.flatnonzero(mm)
    fs = (np.arange(F) * hop).astype(np.int64)[idx]
    rng = np.random.default_rng(5)
    sims = []
    params = []
    for _ in range(6):
        g = np.float32(rng.uniform(-3, 3))
        T = float(np.float32(rng.uniform(-70, -20)))
        hy = float(rng.choice([0, 1, 2, 3, 4, 6]))
        up = float(rng.choice([0, 50, 100, 150, 200, 250]))
        sims.append(ref.simulate_state((ol + g)[idx], fs, sr, T, hy, up))
        params.append([float(g), T, hy, up])
    res["sim_params"] = np.array(params)
    res["sim_states"] = np.stack(sims).astype(np.int8)
    # debounce on a random jittery sequence
    seq = np.where(rng.random(400) < 0.5, 1, 2).astype(np.int32)
    seq[100:160] = 2
    res["deb_in"] = seq
    res["deb_out"] = ref.debounce_state(seq, min_run=3)
    out = os.path.join(REPO, "tests", "golden", "calib_v2.npz")
    np.savez_compressed(out, **res)
    print(str(res["json"]))


if __name__ == "__main__":
    main()
