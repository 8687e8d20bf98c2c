"""Host-side DSP set-up helpers, under the reference's names (layer L2 of SURVEY §1).

These are the once-per-file table builders and scalar mappings of the
reference; they stay on the host in numpy exactly as the reference computes
them (bit-identical tables).  The per-frame work they feed runs in the HIP
library (``engine.py``).

Reference (file:line):
  rms_dbfs                      src/process_tomatis.py:43-52
  gate_ui_to_dbfs               src/process_tomatis.py:54-80
  gate_ui_to_dbfs_log_percent   src/process_tomatis.py:82-103
  db_to_lin                     src/process_tomatis.py:105-107
  build_tilt_gain_db            src/process_tomatis.py:109-158
  load_eq_csv                   src/layer2_apply_eq.py:11-46
  build_gain_per_bin            src/layer2_apply_eq.py:48-64
  smooth_on_logfreq             src/layer2b_apply_residual_eq.py:12-35
  build_eq_from_residual        src/layer2b_apply_residual_eq.py:37-55
  build_eq_from_residual_safe   src/layer2b_apply_residual_eq_safe.py:37-49
The r -> level -> gate-predicate reduction (``gate_bits``) is this build's own:
it turns the reference's float comparisons ``level >= Ton`` / ``level <= Toff``
into exact integer comparisons on the bit pattern of the float32 frame RMS.
"""
from __future__ import annotations

import csv

import numpy as np

EPS = 1e-12
PEAK_LIMIT = 0.999


# ---------------------------------------------------------------------------
# scalar mappings and tables
# ---------------------------------------------------------------------------

def gate_ui_to_dbfs(gate_ui: float, gate_scale: float = 1.0, gate_offset: float = -100.0) -> float:
    """T_dBFS = gate_scale * gate_ui + gate_offset (linear mapping)."""
    return gate_scale * gate_ui + gate_offset


def gate_ui_to_dbfs_log_percent(gate_ui: float, dynamic_range: float = 80.0) -> float:
    """T_dBFS = -DR + DR * gate_ui / 100 (log-percent mapping, CLI default)."""
    return -dynamic_range + dynamic_range * gate_ui / 100.0


def db_to_lin(db):
    """dB -> linear gain as float32."""
    return (10.0 ** (np.asarray(db) / 20.0)).astype(np.float32)


def build_tilt_gain_db(freqs, fc, slope_db_per_oct, low_gain_db, high_gain_db):
    """Tilt curve pivoting at fc: ramp at ``slope`` dB/oct to a plateau per side."""
    f = np.maximum(freqs, 1.0)
    octs = np.log2(f / fc).astype(np.float32)
    g = np.zeros_like(octs, dtype=np.float32)
    lo = np.sign(low_gain_db) * np.minimum(slope_db_per_oct * np.maximum(0.0, -octs),
                                           abs(low_gain_db))
    hi = np.sign(high_gain_db) * np.minimum(slope_db_per_oct * np.maximum(0.0, octs),
                                            abs(high_gain_db))
    g[octs < 0] = lo[octs < 0]
    g[octs > 0] = hi[octs > 0]
    return g


def hann(n_fft: int) -> np.ndarray:
    """Symmetric Hann window as float32 (np.hanning), as the reference uses."""
    return np.hanning(n_fft).astype(np.float32)


def rms_dbfs(x_mono) -> float:
    """RMS level of one mono frame in dBFS.

    Kept for API parity (validators call it per frame).  Bulk per-frame levels
    are computed on the GPU by ``engine.frame_r`` + ``r_to_level``.
    """
    x_mono = np.asarray(x_mono)
    r = np.sqrt(np.mean(x_mono * x_mono) + EPS)
    return float(20.0 * np.log10(r + EPS))


def r_to_level(r: np.ndarray) -> np.ndarray:
    """Per-frame dBFS from the GPU frame RMS ``r`` (float32 or float64), as float64.

    Same numpy ufuncs as the reference's scalar ``float(20*log10(r+EPS))``
    (array and scalar paths are bit-identical on this numpy)."""
    return (20.0 * np.log10(np.asarray(r) + EPS)).astype(np.float64)


# ---------------------------------------------------------------------------
# exact gate predicates on float32 r bit patterns
# ---------------------------------------------------------------------------

_POS_INF_BITS = 0x7F800000
_WINDOW = 1 << 13


def _level_of_bits(bits: np.ndarray) -> np.ndarray:
    r = np.asarray(bits, dtype=np.uint32).view(np.float32)
    return r_to_level(r)


def _first_true(pred, lo: int, hi: int) -> int:
    """Smallest b in [lo, hi] with pred(b) (pred assumed monotone); hi+1 if none."""
    if not pred(np.array([hi], np.uint32))[0]:
        return hi + 1
    while lo < hi:
        mid = (lo + hi) // 2
        if pred(np.array([mid], np.uint32))[0]:
            hi = mid
        else:
            lo = mid + 1
    return lo


def gate_bits(Ton: float, Toff: float):
    """Exact integer form of ``level(r) >= Ton`` and ``level(r) <= Toff``.

    Returns ``(on_bits, on_exc, off_bits, off_exc)`` such that for every
    non-NaN float32 ``r >= 0`` with bit pattern ``b``:
      level(r) >= Ton  <=>  (b >= on_bits)  XOR  (b in on_exc)
      level(r) <= Toff <=>  (b <= off_bits) XOR  (b in off_exc)
    numpy's float32 log10 is not correctly rounded and (very rarely) not
    monotone, so a window of +-8192 ulps around each crossing is evaluated
    exhaustively and any out-of-order patterns become exceptions.
    """
    def p_on(b):
        return _level_of_bits(b) >= Ton

    def p_off(b):
        return _level_of_bits(b) <= Toff

    # --- on ---
    c = _first_true(p_on, 0, _POS_INF_BITS)
    lo, hi = max(0, c - _WINDOW), min(_POS_INF_BITS, c + _WINDOW)
    w = np.arange(lo, hi + 1, dtype=np.int64)
    pw = p_on(w.astype(np.uint32))
    # on_bits: first index after the last False in the window
    falses = np.nonzero(~pw)[0]
    on_bits = int(w[falses[-1]] + 1) if len(falses) else lo
    on_exc = [int(b) for b in w[(w < on_bits) & pw]]
    # --- off: last b with level <= Toff  <=> first b with level > Toff, minus 1
    c2 = _first_true(lambda b: ~p_off(b), 0, _POS_INF_BITS)
    lo2, hi2 = max(0, c2 - _WINDOW), min(_POS_INF_BITS, c2 + _WINDOW)
    w2 = np.arange(lo2, hi2 + 1, dtype=np.int64)
    pw2 = p_off(w2.astype(np.uint32))
    trues = np.nonzero(pw2)[0]
    off_bits = int(w2[trues[-1]]) if len(trues) else lo2 - 1
    # everything <= off_bits in the window must be true; record the falses
    off_exc = [int(b) for b in w2[(w2 <= off_bits) & ~pw2]]
    if off_bits < 0:  # never true: b <= 0 with b == 0 flipped off by an exception
        off_bits, off_exc = 0, [0]
    # Unreachable for any finite threshold: every r is >= 1e-6 (the +EPS under the
    # square root), and over all finite float32 r >= 2^-20 numpy's level has 35
    # non-monotone steps, each >= 2^23 ulps from the next, so a +-8192-ulp
    # window holds at most one (tests/test_host_logic.py scans all 1.3e9
    # patterns).  Kept as a guard for a numpy whose log10 behaves otherwise.
    if len(on_exc) > 4 or len(off_exc) > 4:
        raise RuntimeError("gate threshold crossing too irregular for the exception table")
    return on_bits, on_exc, off_bits, off_exc


# ---------------------------------------------------------------------------
# layer-2 / layer-2b EQ curves
# ---------------------------------------------------------------------------

def load_eq_csv(eq_csv_path):
    """(freq_hz, gain_db) float32 columns of an EQ CSV, sorted by frequency.

    Column aliases as the reference: freq_hz/freq/hz/f and
    delta_db_smooth/delta_db/db/gain_db/delta/gain.
    """
    with open(eq_csv_path, "r", encoding="utf-8") as f:
        rd = csv.DictReader(f)
        cols = [c.lower().strip() for c in rd.fieldnames]
        f_col = next((c for c in ["freq_hz", "freq", "hz", "f"] if c in cols), None)
        d_col = next((c for c in ["delta_db_smooth", "delta_db", "db", "gain_db", "delta",
                                  "gain"] if c in cols), None)
        if f_col is None or d_col is None:
            raise ValueError(f"EQ CSV 列名不符合预期。发现列: {rd.fieldnames}")
        print(f"[EQ_LOAD] Using columns: freq='{f_col}', gain='{d_col}'")
        fr, db = [], []
        for row in rd:
            fr.append(float(row[f_col]))
            db.append(float(row[d_col]))
    fr = np.array(fr, np.float32)
    db = np.array(db, np.float32)
    order = np.argsort(fr)
    return fr[order], db[order]


def build_gain_per_bin(sr, n_fft, eq_freqs, eq_db):
    """Interpolate an EQ curve on log10(f) to rfft bins (edge-clamped), float32 linear."""
    fb = np.fft.rfftfreq(n_fft, 1.0 / sr).astype(np.float32)
    xb = np.log10(np.maximum(fb, 1.0))
    xk = np.log10(np.maximum(eq_freqs, 1.0))
    yb = np.interp(xb, xk, eq_db, left=eq_db[0], right=eq_db[-1]).astype(np.float32)
    return (10.0 ** (yb / 20.0)).astype(np.float32)


def smooth_on_logfreq(freq, db, win=21):
    """Moving average of a residual curve on a uniform log-frequency grid."""
    lf = np.log10(np.maximum(freq, 1.0))
    order = np.argsort(lf)
    lfs, dbs = lf[order], db[order]
    n = len(dbs)
    grid = np.linspace(lfs.min(), lfs.max(), n)
    on_grid = np.interp(grid, lfs, dbs)
    win = max(3, win | 1)
    half = win // 2
    padded = np.pad(on_grid, (half, half), mode="edge")
    box = np.ones(win, dtype=np.float32) / win
    smooth = np.convolve(padded, box, mode="valid")
    back = np.interp(lfs, grid, smooth)
    out = np.empty_like(back)
    out[order] = back
    return out


def build_eq_from_residual(freqs_rfft, res_freq, res_db, clamp_lo=-6.0, clamp_hi=6.0,
                           mid_start=3000.0, mid_clamp_hi=2.0, hf_start=8000.0,
                           hf_clamp_hi=0.0):
    """Residual -> per-bin EQ with global, 3-8 kHz and >=8 kHz clamps."""
    db = np.interp(freqs_rfft, res_freq, res_db, left=res_db[0], right=res_db[-1])
    db = np.clip(db, clamp_lo, clamp_hi)
    mid = (freqs_rfft >= mid_start) & (freqs_rfft < hf_start)
    db[mid] = np.clip(db[mid], clamp_lo, mid_clamp_hi)
    hf = freqs_rfft >= hf_start
    db[hf] = np.clip(db[hf], clamp_lo, hf_clamp_hi)
    return (10.0 ** (db / 20.0)).astype(np.float32), db.astype(np.float32)


def build_eq_from_residual_safe(freqs_rfft, res_freq, res_db, clamp_lo=-1.0, clamp_hi=1.0,
                                hf_start=3000.0):
    """'Safe' variant: +-1 dB clamp and 0 dB at and above ``hf_start``."""
    db = np.interp(freqs_rfft, res_freq, res_db, left=res_db[0], right=res_db[-1])
    db = np.clip(db, clamp_lo, clamp_hi)
    db[freqs_rfft >= hf_start] = 0.0
    return (10.0 ** (db / 20.0)).astype(np.float32), db.astype(np.float32)


def read_diff_csv(path_or_buf):
    """``diff_spectrum.csv`` columns as float32 (pandas, as the reference)."""
    import pandas as pd
    d = pd.read_csv(path_or_buf)
    col = "delta_db_base_minus_cand" if "delta_db_base_minus_cand" in d.columns else "delta_db"
    return d["freq_hz"].to_numpy(np.float32), d[col].to_numpy(np.float32)


# ---------------------------------------------------------------------------
# schedules (pure integer arithmetic of the reference loops)
# ---------------------------------------------------------------------------

def std_schedule(N: int, n_fft: int, hop: int):
    """Frame schedule of process_tomatis.py:270-272 (pad, pad_end, F, first start)."""
    pad = n_fft // 2
    pad_end = (hop - ((N - n_fft) % hop)) % hop
    total = pad + N + pad_end
    F = (total - n_fft) // hop + 1 if total >= n_fft else 0
    return pad, pad_end, F, -pad


def std_flush_bounds(N: int, n_fft: int, hop: int, flush: int = 48000 * 5):
    """Limiter chunk boundaries of process_tomatis.py:419-426 (absolute positions)."""
    pad, _, F, s0 = std_schedule(N, n_fft, hop)
    base = s0
    bounds = [base]
    # flush after frame k when (s_{k+1} - base) - n_fft >= flush; closed form:
    if F:
        # first flush: smallest k with s0 + (k+1)*hop - n_fft - s0 >= flush
        k1 = max(0, -(-(flush + n_fft) // hop) - 1)
        if k1 <= F - 1:
            b = s0 + (k1 + 1) * hop - n_fft
            step = -(-flush // hop)  # frames between flushes
            k = k1
            while k <= F - 1:
                bounds.append(b)
                k += step
                b += step * hop
        end = s0 + (F - 1) * hop + n_fft
        if end > bounds[-1]:
            bounds.append(end)
    return bounds


def adaptive_frames(N: int, n_fft: int, hop: int):
    """Frames of process_tomatis_adaptive.py:70-77,298-300: (first k, count, first start)."""
    pad = n_fft // 2
    total = N + 2 * pad
    n_all = (total - n_fft) // hop + 1 if total >= n_fft else 0
    k = np.arange(n_all, dtype=np.int64)
    orig = k * hop - pad
    ok = np.nonzero((orig >= 0) & (orig < N))[0]
    if len(ok) == 0:
        return 0, 0, 0
    return int(ok[0]), int(len(ok)), int(orig[ok[0]])


def level_stats(valid: np.ndarray):
    """``(np.percentile(v, 5), np.percentile(v, 95), np.median(v))`` of a
    float64 array with one ``np.partition`` (numpy 2.x 'linear' rule and
    median rule restated; src/process_tomatis_adaptive.py:129-131 calls the
    three separately, each partitioning again).  Bit-identical: checked
    against the numpy calls in tests/test_host_logic.py."""
    v = np.asarray(valid, np.float64)
    n = v.size
    q = np.array([5.0, 95.0]) / 100
    vi = (n - 1) * q
    prev = np.floor(vi)
    above = vi >= n - 1
    pi = np.where(above, n - 1, prev).astype(np.intp)
    ni = np.where(above, n - 1, prev + 1).astype(np.intp)
    gamma = np.where(above, 0.0, vi - prev)
    h = n // 2
    mk = [h - 1, h] if n % 2 == 0 else [h]
    kth = np.unique(np.concatenate([pi, ni, mk, [0, n - 1]]))
    part = np.partition(v, kth)
    a, b = part[pi], part[ni]
    d = b - a
    lerp = a + d * gamma
    lerp = np.where(gamma >= 0.5, b - d * (1 - gamma), lerp)
    if n % 2:
        med = part[h] + 0.0
    else:
        med = (0.0 + part[h - 1] + part[h]) / 2.0
    return float(lerp[0]), float(lerp[1]), float(med)
