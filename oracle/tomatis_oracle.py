"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement (numpy) of the reference hot path of
xyjk0511/tomatis-audio-processor.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline.  The product (``tomatis_audio_processor_amd``)
never imports it: the product path is the HIP library and fails loudly without
it.

Pinning: every processor below is checked against golden vectors produced by
running the reference itself in the build container (``tests/golden/``,
generator ``tools/make_goldens.py``).  The restatement reuses the same numpy
primitives in the same order, so it is *bit-exact* with the reference on this
numpy (2.2.6): states, frame r / levels, chunk boundaries and the float output
hashes must match exactly (``tests/test_oracle_golden.py``).

What is restated (reference file:line, relative to the reference root):
  * frame schedule / padding      src/process_tomatis.py:270-272,310-316,365-367,441-449
  * power-mono RMS level          src/process_tomatis.py:43-52,369-371
  * gate threshold mappings       src/process_tomatis.py:54-103,277-285
  * standard gate automaton       src/process_tomatis.py:373-385
  * tilt gains / window           src/process_tomatis.py:105-158,256-267
  * spectral filter per frame     src/process_tomatis.py:394-398
  * OLA / normalise / limiter     src/process_tomatis.py:322-357,400-426,451-453
  * xfade alpha + mixed gain      src/process_tomatis_xfade.py:153-155,251-274
  * adaptive processor            src/process_tomatis_adaptive.py:57-154,157-351
  * layer-2 static EQ             src/layer2_apply_eq.py:11-64,66-233
  * layer-2b residual EQ          src/layer2b_apply_residual_eq.py:12-55,57-160
                                  src/layer2b_apply_residual_eq_safe.py:37-49
Vectorisation notes (each verified bit-identical to the per-frame loop on this
numpy): batched ``np.fft.rfft/irfft`` along the last axis equals per-frame
calls; ``np.mean`` along a contiguous last axis uses the same pairwise
summation as the per-frame call; ``np.log10`` on arrays equals the scalar call.
The OLA itself is kept as a frame-ordered loop (float32 sum order matters).
"""
from __future__ import annotations


import numpy as np
from numpy.lib.stride_tricks import as_strided

EPS = 1e-12
PEAK_LIMIT = 0.999
FLUSH_STD = 48000 * 5          # hard-coded flush size, process_tomatis.py:420


# ----------------------------------------------------------------------------
# L2 helpers
# ----------------------------------------------------------------------------

def gate_ui_to_dbfs(gate_ui, gate_scale=1.0, gate_offset=-100.0):
    """process_tomatis.py:54-80 (linear mapping)."""
    return gate_scale * gate_ui + gate_offset


def gate_ui_to_dbfs_log_percent(gate_ui, dynamic_range=80.0):
    """process_tomatis.py:82-103 (log-percent mapping, the CLI default)."""
    return -dynamic_range + dynamic_range * gate_ui / 100.0


def db_to_lin_f32(db):
    """process_tomatis.py:105-107 / process_tomatis_xfade.py:33-35."""
    return (10.0 ** (np.asarray(db) / 20.0)).astype(np.float32)


def tilt_gain_db(freqs, fc, slope, low_db, high_db):
    """process_tomatis.py:109-158 — two-sided ramp + plateau tilt in dB (f32)."""
    f = np.maximum(freqs, 1.0)
    oct_ = np.log2(f / fc).astype(np.float32)
    out = np.zeros_like(oct_, dtype=np.float32)
    below = slope * np.maximum(0.0, -oct_)
    above = slope * np.maximum(0.0, oct_)
    lo = np.sign(low_db) * np.minimum(below, abs(low_db))
    hi = np.sign(high_db) * np.minimum(above, abs(high_db))
    out[oct_ < 0] = lo[oct_ < 0]
    out[oct_ > 0] = hi[oct_ > 0]
    return out


def hann_sym(n_fft):
    """process_tomatis.py:266-267 — symmetric np.hanning window and its square."""
    w = np.hanning(n_fft).astype(np.float32)
    return w, (w * w).astype(np.float32)


# ----------------------------------------------------------------------------
# Framing and levels
# ----------------------------------------------------------------------------

def frame_view(xpad, n_fft, hop, n_frames, first=0):
    """Strided [F, n_fft, ch] view of ``xpad`` (frames at first + k*hop)."""
    s0, s1 = xpad.strides
    base = xpad[first:]
    return as_strided(base, shape=(n_frames, n_fft, xpad.shape[1]),
                      strides=(hop * s0, s0, s1), writeable=False)


def frame_r(frames, block=256):
    """Per-frame RMS ``r`` (process_tomatis.py:51,369-371).

    ``mono = sqrt(mean(frame**2, axis=1))``; ``r = sqrt(mean(mono*mono)+EPS)``
    in the frame dtype (float32, or float64 in the adaptive quiet case).
    """
    F = frames.shape[0]
    out = np.empty(F, dtype=frames.dtype)
    for a in range(0, F, block):
        fr = np.ascontiguousarray(frames[a:a + block])
        mono = np.sqrt(np.mean(fr ** 2, axis=2))
        out[a:a + block] = np.sqrt(np.mean(mono * mono, axis=1) + EPS)
    return out


def r_to_level(r):
    """``float(20*log10(r+EPS))`` per frame (process_tomatis.py:52), as f64."""
    return (20.0 * np.log10(r + EPS)).astype(np.float64)


# ----------------------------------------------------------------------------
# Gate automata
# ----------------------------------------------------------------------------

def gate_standard(levels, starts, Ton, Toff, up_delay_samples):
    """process_tomatis.py:373-385 — hysteresis + up-delay; returns u8 states (1/2)."""
    st = np.empty(len(levels), dtype=np.uint8)
    state, pending = 1, None
    for k, (lv, s) in enumerate(zip(levels.tolist(), starts.tolist())):
        if state == 1:
            if lv >= Ton:
                if pending is None:
                    pending = s + up_delay_samples
            else:
                pending = None
            if pending is not None and s >= pending:
                state, pending = 2, None
        else:
            if lv <= Toff:
                state, pending = 1, None
        st[k] = state
    return st


def gate_minhold(levels, threshold, hyst_db=3.0, min_hold_frames=6):
    """process_tomatis_adaptive.py:87-121 — min-hold automaton; u8 states (1/2)."""
    Ton = threshold + hyst_db / 2
    Toff = threshold - hyst_db / 2
    st = np.empty(len(levels), dtype=np.uint8)
    state, since = 1, min_hold_frames
    for k, lv in enumerate(levels):          # numpy float64 scalars, as reference
        since += 1
        if since >= min_hold_frames:
            if state == 1:
                if lv >= Ton:
                    state, since = 2, 0
            else:
                if lv <= Toff:
                    state, since = 1, 0
        st[k] = state
    return st


def optimal_threshold(levels, valid_mask, hyst_db=3.0, min_hold_frames=6,
                      target_c2=0.5):
    """process_tomatis_adaptive.py:124-154 — bisection on [p5, p95]."""
    valid = levels[valid_mask]
    if len(valid) == 0:
        return np.median(levels)
    T_low = np.percentile(valid, 5)
    T_high = np.percentile(valid, 95)
    best_T = np.median(valid)
    best_diff = 1.0
    for _ in range(30):
        T_mid = (T_low + T_high) / 2
        st = gate_minhold(levels, T_mid, hyst_db, min_hold_frames)
        c2 = int(np.count_nonzero(st == 2)) / len(st)
        diff = abs(c2 - target_c2)
        if diff < best_diff:
            best_diff, best_T = diff, T_mid
        if diff < 0.01:
            break
        if c2 < target_c2:
            T_high = T_mid
        else:
            T_low = T_mid
    return best_T


def alpha_scan_xfade(states, xfade_frames):
    """process_tomatis_xfade.py:251-262 — per-frame alpha (python float / f64)."""
    step = 1.0 / xfade_frames if xfade_frames > 0 else 1.0
    a = 0.0
    out = np.empty(len(states), dtype=np.float64)
    for k, s in enumerate(states.tolist()):
        tgt = 0.0 if s == 1 else 1.0
        if xfade_frames > 0:
            d = tgt - a
            if abs(d) <= step:
                a = tgt
            else:
                a += step * np.sign(d)
        else:
            a = tgt
        out[k] = a
    return out


def alpha_scan_adaptive(states, xfade_frames):
    """process_tomatis_adaptive.py:253-265 — alpha[0] = target[0], then ±step."""
    tgt = np.where(states == 2, 1.0, 0.0)
    a = np.zeros_like(tgt)
    if len(a) == 0:
        return a
    a[0] = tgt[0]
    step = 1.0 / xfade_frames if xfade_frames > 0 else 1.0
    for i in range(1, len(a)):
        d = tgt[i] - a[i - 1]
        if abs(d) <= step:
            a[i] = tgt[i]
        else:
            a[i] = a[i - 1] + step * np.sign(d)
    return a


# ----------------------------------------------------------------------------
# Spectral filter + OLA
# ----------------------------------------------------------------------------

def spectral_filter(frames, win, gains):
    """process_tomatis.py:394-398 — per channel rfft * gain -> irfft * win.

    ``frames`` [F, n_fft, ch]; ``gains`` [F, n_bins] float32.  Returns
    [F, n_fft, ch] in the frame dtype.
    """
    F, n_fft, ch = frames.shape
    y = np.empty(frames.shape, dtype=frames.dtype)
    for c in range(ch):
        X = np.fft.rfft(frames[:, :, c] * win, axis=1)
        X *= gains
        yc = np.fft.irfft(X, n=n_fft, axis=1)
        if frames.dtype == np.float32:
            yc = yc.astype(np.float32)
        y[:, :, c] = yc * win
    return y


def ola(y, starts, n_fft, win2, length, origin, clip_lo=None, clip_hi=None):
    """Frame-ordered overlap-add (process_tomatis.py:400-406).

    Accumulates ``y[k]`` at absolute start ``starts[k]`` into a buffer whose
    index 0 is absolute position ``origin``.  With ``clip_lo/clip_hi`` only the
    part inside ``[clip_lo, clip_hi)`` is added (adaptive mode,
    process_tomatis_adaptive.py:316-323).
    """
    ch = y.shape[2]
    out = np.zeros((length, ch), dtype=y.dtype)
    w = np.zeros(length, dtype=np.float32)
    for k in range(y.shape[0]):
        s = int(starts[k])
        a, b = s, s + n_fft
        if clip_lo is not None:
            a = max(a, clip_lo)
            b = min(b, clip_hi)
        if b <= a:
            continue
        out[a - origin:b - origin] += y[k, a - s:b - s]
        w[a - origin:b - origin] += win2[a - s:b - s]
    return out, w


# ----------------------------------------------------------------------------
# Processors
# ----------------------------------------------------------------------------

def _std_schedule(N, n_fft, hop):
    pad = n_fft // 2
    pad_end = (hop - ((N - n_fft) % hop)) % hop
    total = pad + N + pad_end
    F = (total - n_fft) // hop + 1 if total >= n_fft else 0
    starts = -pad + hop * np.arange(F, dtype=np.int64)
    return pad, pad_end, F, starts


def std_chunk_bounds(N, n_fft, hop, flush=FLUSH_STD):
    """Flush schedule of process_tomatis.py:419-426,451-453 in absolute coords.

    Returns the list of chunk boundaries [B0=-pad, B1, ..., end] where ``end``
    is the end of the last frame.  Simulated with the reference's own integer
    arithmetic (it depends only on the frame index, not on read blocks).
    """
    pad, _, F, starts = _std_schedule(N, n_fft, hop)
    out_base = -pad
    bounds = [out_base]
    for k in range(F):
        nxt = int(starts[k]) + hop
        safe = (nxt - out_base) - n_fft
        if safe >= flush:
            out_base += safe
            bounds.append(out_base)
    end = int(starts[F - 1]) + n_fft if F else out_base
    if end > bounds[-1]:
        bounds.append(end)
    return bounds


def _write_chunks(yfull, origin, bounds, N, out_gain_db=0.0):
    """write_clamped per chunk (process_tomatis.py:331-357)."""
    ch = yfull.shape[1]
    out = np.zeros((N, ch), dtype=np.float32)
    scales = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        s, e = max(0, a), min(N, b)
        if e <= s:
            scales.append(None)
            continue
        chunk = yfull[s - origin:e - origin]
        if out_gain_db != 0.0:
            chunk = chunk * (10.0 ** (out_gain_db / 20.0))
        peak = np.max(np.abs(chunk))
        if peak > PEAK_LIMIT:
            sc = PEAK_LIMIT / peak
            chunk = chunk * sc
            scales.append(float(sc))
        else:
            scales.append(1.0)
        out[s:e] = chunk
    return out, scales


def process_standard(x, sr, gate_ui=50, gate_mode="log_percent",
                     dynamic_range=80.0, gate_scale=1.0, gate_offset=-100,
                     hysteresis_db=3.0, fc=1000.0, slope=12.0,
                     c1_low=15.0, c1_high=-15.0, c2_low=-15.0, c2_high=15.0,
                     up_delay_ms=250.0, n_fft=4096, hop=2048,
                     output_gain_db=0.0, xfade_ms=None):
    """Standard (``xfade_ms is None``) or xfade processor on an in-memory array.

    Standard: src/process_tomatis.py:160-478.  Xfade: src/process_tomatis_xfade.py:55-359
    (linear gate mapping only, no output gain).  Returns a dict with the float32
    output as written (before PCM quantisation), states, r, levels, alpha, chunk
    bounds and limiter scales.
    """
    x = np.asarray(x, dtype=np.float32)
    if x.ndim == 1:
        x = x[:, None]
    N, ch = x.shape
    freqs = np.fft.rfftfreq(n_fft, d=1.0 / sr)
    g1_db = tilt_gain_db(freqs, fc, slope, c1_low, c1_high)
    g2_db = tilt_gain_db(freqs, fc, slope, c2_low, c2_high)
    g1, g2 = db_to_lin_f32(g1_db), db_to_lin_f32(g2_db)
    win, win2 = hann_sym(n_fft)
    pad, pad_end, F, starts = _std_schedule(N, n_fft, hop)
    if xfade_ms is not None or gate_mode != "log_percent":
        T = gate_ui_to_dbfs(gate_ui, gate_scale, gate_offset)
    else:
        T = gate_ui_to_dbfs_log_percent(gate_ui, dynamic_range)
    Ton, Toff = T + hysteresis_db / 2.0, T - hysteresis_db / 2.0
    D = int(sr * up_delay_ms / 1000.0)

    xpad = np.concatenate([np.zeros((pad, ch), np.float32), x,
                           np.zeros((pad_end, ch), np.float32)])
    frames = frame_view(xpad, n_fft, hop, F)
    r = frame_r(frames)
    levels = r_to_level(r)
    states = gate_standard(levels, starts, Ton, Toff, D)

    alpha = None
    if xfade_ms is None:
        gains = np.where((states == 1)[:, None], g1[None, :], g2[None, :])
    else:
        frame_ms = hop / sr * 1000.0
        xf = max(1, int(np.ceil(xfade_ms / frame_ms))) if xfade_ms > 0 else 0
        alpha = alpha_scan_xfade(states, xf)
        gains = np.empty((F, len(g1)), dtype=np.float32)
        for k in range(F):
            a = alpha[k]
            if xfade_ms > 0 and 0 < a < 1:
                gains[k] = db_to_lin_f32((1 - a) * g1_db + a * g2_db)
            else:
                gains[k] = g1 if a < 0.5 else g2
    y = spectral_filter(frames, win, gains)
    length = int(starts[-1]) + n_fft + pad if F else 0
    out, w = ola(y, starts, n_fft, win2, length, origin=-pad)
    yfull = out / (w[:, None] + EPS)
    bounds = std_chunk_bounds(N, n_fft, hop)
    gain_db = output_gain_db if xfade_ms is None else 0.0
    yout, scales = _write_chunks(yfull, -pad, bounds, N, gain_db)
    return dict(y=yout, states=states, r=r, levels=levels, alpha=alpha,
                starts=starts, bounds=np.asarray(bounds, np.int64),
                scales=scales, wsum=w, g1=g1, g2=g2, Ton=Ton, Toff=Toff,
                up_delay_samples=D, pad=pad, pad_end=pad_end)


def process_adaptive(x, sr, fc=1000.0, slope=12.0, c1_low=15.0, c1_high=-15.0,
                     c2_low=-15.0, c2_high=15.0, target_c2=0.5, hyst_db=3.0,
                     min_hold_ms=250.0, xfade_ms=500.0, headroom_margin=2.0,
                     n_fft=4096, hop=2048):
    """src/process_tomatis_adaptive.py:157-351 on an in-memory float32 array.

    Keeps the reference's NEP-50 dtype behaviour: loud input runs
    in float32, input with peak <= -(max_gain+margin) dBFS runs in float64.
    """
    x = np.asarray(x, dtype=np.float32)
    if x.ndim == 1:
        x = x.reshape(-1, 1)
    N, ch = x.shape
    frame_ms = hop / sr * 1000
    mh = int(np.ceil(min_hold_ms / frame_ms))
    xf = int(np.ceil(xfade_ms / frame_ms))
    peak = np.max(np.abs(x))
    peak_db = 20 * np.log10(peak + EPS)
    max_gain = max(abs(c1_low), abs(c2_high))
    atten_db = max(0, peak_db + max_gain + headroom_margin)
    atten_lin = 10 ** (np.asarray(-atten_db) / 20.0)
    xa = x * atten_lin

    pad = n_fft // 2
    xpad = np.vstack([np.zeros((pad, ch), dtype=xa.dtype), xa,
                      np.zeros((pad, ch), dtype=xa.dtype)])
    n_all = (len(xpad) - n_fft) // hop + 1 if len(xpad) >= n_fft else 0
    orig = np.arange(n_all, dtype=np.int64) * hop - pad
    valid_frames = np.nonzero((orig >= 0) & (orig < N))[0]
    first = int(valid_frames[0]) if len(valid_frames) else 0
    Fv = len(valid_frames)
    frames = frame_view(xpad, n_fft, hop, Fv, first=first * hop)
    r = frame_r(frames)
    levels = r_to_level(r)
    valid = levels > -70
    T = optimal_threshold(levels, valid, hyst_db, mh, target_c2)
    states = gate_minhold(levels, T, hyst_db, mh)
    alpha = alpha_scan_adaptive(states, xf)

    freqs = np.fft.rfftfreq(n_fft, 1 / sr)
    c1_db = tilt_gain_db(freqs, fc, slope, c1_low, c1_high)
    c2_db = tilt_gain_db(freqs, fc, slope, c2_low, c2_high)
    win = np.hanning(n_fft).astype(np.float32)
    gains = np.empty((Fv, len(c1_db)), dtype=np.float32)
    for k in range(Fv):
        a = alpha[k]
        gains[k] = (10 ** (np.asarray((1 - a) * c1_db + a * c2_db) / 20.0)
                    ).astype(np.float32)
    y = spectral_filter(frames, win, gains)
    starts = orig[valid_frames]
    win2 = win ** 2
    out, norm = ola(y, starts, n_fft, win2, N, origin=0, clip_lo=0, clip_hi=N)
    norm = np.maximum(norm, 1e-8)
    for c in range(ch):
        out[:, c] /= norm
    if atten_db > 0:
        out *= 10 ** (np.asarray(atten_db) / 20.0)
    scale = None
    opk = np.max(np.abs(out)) if out.size else 0.0
    if opk > PEAK_LIMIT:
        scale = PEAK_LIMIT / opk
        out *= scale
    return dict(y=out, states=states, r=r, levels=levels, alpha=alpha,
                threshold=float(T), atten_db=atten_db, starts=starts,
                min_hold_frames=mh, xfade_frames=xf, scale=scale, wsum=norm)


# --- layer 2 -----------------------------------------------------------------

def eq_gain_per_bin(sr, n_fft, eq_freqs, eq_db):
    """src/layer2_apply_eq.py:48-64 — log-f interpolation of an EQ curve."""
    fb = np.fft.rfftfreq(n_fft, 1.0 / sr).astype(np.float32)
    fs = np.maximum(fb, 1.0)
    xk = np.log10(np.maximum(eq_freqs, 1.0))
    xb = np.log10(fs)
    yb = np.interp(xb, xk, eq_db, left=eq_db[0], right=eq_db[-1]).astype(np.float32)
    return (10.0 ** (yb / 20.0)).astype(np.float32)


def _static_stft(xpad, n_fft, hop, F, gain):
    win, win2 = hann_sym(n_fft)
    frames = frame_view(xpad, n_fft, hop, F)
    y = spectral_filter(frames, win, np.broadcast_to(gain, (F, len(gain))))
    starts = hop * np.arange(F, dtype=np.int64)
    length = int(starts[-1]) + n_fft if F else 0
    out, w = ola(y, starts, n_fft, win2, length, origin=0)
    return out, w


def _normalise(out, w):
    """``out/(w+EPS)`` (src/layer2_apply_eq.py:177,212).  The layer-2 flushes
    divide elementwise with no limiter, so chunking never changes a value."""
    return out / (w[:, None] + EPS)


def apply_eq_stft(x, sr, eq_freqs, eq_db, n_fft=4096, hop=2048, pad=True,
                  global_gain_db=0.0, auto_gain_protect=True, peak_target=0.99):
    """src/layer2_apply_eq.py:66-233 on an in-memory array.

    Returns the main output (float32, padded coordinates, head pad kept) and,
    when gain protection triggers, the ``_gp`` output (scale applied to the
    float output; the reference applies it to the PCM_24 re-read — a <=1 LSB
    difference noted in DESIGN.md).
    """
    x = np.asarray(x, dtype=np.float32)
    N, ch = x.shape
    gain = eq_gain_per_bin(sr, n_fft, eq_freqs, eq_db)
    g_global = 10.0 ** (global_gain_db / 20.0)
    xs = (x * g_global).astype(np.float32)
    pl = n_fft // 2 if pad else 0
    xpad = np.concatenate([np.zeros((pl, ch), np.float32), xs,
                           np.zeros((pl, ch), np.float32)])
    total = len(xpad)
    F = (total - n_fft) // hop + 1 if total >= n_fft else 0
    out, w = _static_stft(xpad, n_fft, hop, F, gain)
    y = _normalise(out, w)
    peak_seen = float(np.max(np.abs(y))) if y.size else 0.0
    y_gp, scale = None, None
    if auto_gain_protect and peak_seen > peak_target:
        scale = peak_target / max(peak_seen, EPS)
        y_gp = (y * scale).astype(np.float32)
    return dict(y=y, y_gp=y_gp, scale=scale, peak_seen=peak_seen, gain=gain,
                wsum=w, frames=F)


def smooth_on_logfreq(freq, db, win=21):
    """src/layer2b_apply_residual_eq.py:12-35."""
    lf = np.log10(np.maximum(freq, 1.0))
    order = np.argsort(lf)
    lf2, db2 = lf[order], db[order]
    n = len(db2)
    grid = np.linspace(lf2.min(), lf2.max(), n)
    dbg = np.interp(grid, lf2, db2)
    win = max(3, win | 1)
    p = win // 2
    xp = np.pad(dbg, (p, p), mode="edge")
    kern = np.ones(win, dtype=np.float32) / win
    sm = np.convolve(xp, kern, mode="valid")
    back = np.interp(lf2, grid, sm)
    out = np.empty_like(back)
    out[order] = back
    return out


def eq_from_residual(freqs_rfft, res_freq, res_db, clamp_lo=-6.0, clamp_hi=6.0,
                     mid_start=3000.0, mid_clamp_hi=2.0, hf_start=8000.0,
                     hf_clamp_hi=0.0, safe=False):
    """src/layer2b_apply_residual_eq.py:37-55 (and _safe.py:37-49 with safe=True)."""
    db = np.interp(freqs_rfft, res_freq, res_db, left=res_db[0], right=res_db[-1])
    db = np.clip(db, clamp_lo, clamp_hi)
    if safe:
        db[freqs_rfft >= hf_start] = 0.0
    else:
        mid = (freqs_rfft >= mid_start) & (freqs_rfft < hf_start)
        db[mid] = np.clip(db[mid], clamp_lo, mid_clamp_hi)
        hf = freqs_rfft >= hf_start
        db[hf] = np.clip(db[hf], clamp_lo, hf_clamp_hi)
    return (10.0 ** (db / 20.0)).astype(np.float32), db.astype(np.float32)


def apply_residual_eq(x, sr, res_freq, res_db, n_fft=4096, hop=2048,
                      smooth_win=41, clamp_hi=6.0, mid_start=3000.0,
                      mid_clamp_hi=2.0, hf_start=8000.0, hf_clamp_hi=0.0,
                      safe=False):
    """src/layer2b_apply_residual_eq.py:57-160 (no pad, tail dropped)."""
    x = np.asarray(x, dtype=np.float32)
    N, ch = x.shape
    res_s = smooth_on_logfreq(res_freq, res_db, win=smooth_win)
    freqs = np.fft.rfftfreq(n_fft, 1.0 / sr)
    if safe:
        lin, _ = eq_from_residual(freqs, res_freq, res_s, clamp_lo=-1.0,
                                  clamp_hi=clamp_hi, hf_start=hf_start, safe=True)
    else:
        lin, _ = eq_from_residual(freqs, res_freq, res_s, clamp_lo=-6.0,
                                  clamp_hi=clamp_hi, mid_start=mid_start,
                                  mid_clamp_hi=mid_clamp_hi, hf_start=hf_start,
                                  hf_clamp_hi=hf_clamp_hi)
    F = (N - n_fft) // hop + 1 if N >= n_fft else 0
    out, w = _static_stft(x, n_fft, hop, F, lin)
    y = _normalise(out, w)
    return dict(y=y, gain=lin, wsum=w, frames=F)


def frames_count_standard(N, n_fft, hop):
    return _std_schedule(N, n_fft, hop)[2]


def ceil_div(a, b):
    return -(-a // b)


__all__ = [n for n in dir() if not n.startswith("_")] + ["_std_schedule"]


# ----------------------------------------------------------------------------
# Analysis spectra.  Same numpy primitives in the
# same order as the reference loops; batched along frames where numpy is
# order-identical (rfft / mean along the last axis, elementwise ops).
# ----------------------------------------------------------------------------

def power_mono(x_lr):
    """compare_audio.py:7-10 (identical copy used by layer2_analyze_eq.py)."""
    p = 0.5 * (x_lr[:, 0] ** 2 + x_lr[:, 1] ** 2)
    return np.sqrt(p + EPS)


def _full_frames(x, n_fft, hop, F):
    """[F, n_fft(, ch)] view of frames starting at f*hop (all inside x)."""
    if x.ndim == 1:
        s0 = x.strides[0]
        return as_strided(x, shape=(F, n_fft), strides=(hop * s0, s0), writeable=False)
    s0, s1 = x.strides
    return as_strided(x, shape=(F, n_fft, x.shape[1]), strides=(hop * s0, s0, s1),
                      writeable=False)


def stft_mag_avg(x, sr, n_fft=4096, hop=2048):
    """compare_audio.stft_mag_avg (src/compare_audio.py:12-24)."""
    win = np.hanning(n_fft).astype(np.float32)
    F = 1 + (len(x) - n_fft) // hop
    if F <= 0:
        raise ValueError("need at least one array to stack")
    fr = _full_frames(x, n_fft, hop, F) * win
    mags = np.abs(np.fft.rfft(fr, axis=-1)).astype(np.float32)
    return mags.mean(axis=0)


def analyze_frame_r(x_lr, n_fft, hop):
    """r of rms_dbfs(power_mono(frame)) per frame (layer2_analyze_eq.py:13-15,71-73)."""
    F = 1 + (len(x_lr) - n_fft) // hop
    mono = np.ascontiguousarray(_full_frames(power_mono(x_lr), n_fft, hop, F))
    return np.sqrt(np.mean(mono * mono, axis=1) + EPS)


def stft_logpower_median(x_lr, sr, n_fft, hop, music_dbfs):
    """layer2_analyze_eq.stft_logpower_median (src/layer2_analyze_eq.py:54-88)."""
    win = np.hanning(n_fft).astype(np.float32)
    freqs = np.fft.rfftfreq(n_fft, 1.0 / sr)
    F = 1 + (len(x_lr) - n_fft) // hop
    if F <= 10:
        raise ValueError("片段太短，无法做稳定频谱统计。")
    r = analyze_frame_r(x_lr, n_fft, hop)
    lv = (20.0 * np.log10(r + EPS)).astype(np.float64)
    keep = ~(lv <= music_dbfs)
    used = int(keep.sum())
    if used < 50:
        raise ValueError(f"可用音乐帧太少（{used} 帧）。把 --music_dbfs 调低一点（例如 -70）。")
    mono = _full_frames(power_mono(x_lr), n_fft, hop, F)[keep]
    X = np.fft.rfft(mono * win, axis=-1)
    P = (X.real * X.real + X.imag * X.imag).astype(np.float32)
    logs = (10.0 * np.log10(P + EPS)).astype(np.float32)
    med = np.median(logs, axis=0).astype(np.float32)
    return freqs, med, used


def find_stable_frames(states, margin=2):
    """validate_layer1.find_stable_frames (src/validate_layer1.py:245-258)."""
    n = len(states)
    c1, c2 = [], []
    for i in range(margin, n - margin):
        w = states[i - margin:i + margin + 1]
        if all(s == "C1" for s in w):
            c1.append(i)
        elif all(s == "C2" for s in w):
            c2.append(i)
    return c1, c2


def conditional_frame_r(x, n_fft, hop):
    """r of rms_dbfs(sqrt(mean(frame**2, axis=1))) per frame f (start f*hop)."""
    x = x.reshape(len(x), -1)
    F = 1 + (len(x) - n_fft) // hop
    return frame_r(_full_frames(np.ascontiguousarray(x), n_fft, hop, F))


def compute_conditional_spectrum(x, y, sr, states, n_fft, hop, level_threshold=-60):
    """validate_layer1.compute_conditional_spectrum (src/validate_layer1.py:261-389),
    the second (effective) pair of loops at :338-375 and the median at :377-387."""
    x = x.reshape(-1, 1) if x.ndim == 1 else x
    y = y.reshape(-1, 1) if y.ndim == 1 else y
    ch = x.shape[1]
    c1s, c2s = find_stable_frames(states, margin=2)
    freqs = np.fft.rfftfreq(n_fft, 1 / sr)
    nb = len(freqs)
    win = np.hanning(n_fft).astype(np.float32)
    F = max(0, 1 + (len(x) - n_fft) // hop)
    r = conditional_frame_r(x, n_fft, hop) if F > 0 else np.zeros(0, np.float32)
    lv = (20.0 * np.log10(r + EPS)).astype(np.float64)
    res = []
    for lst in (c1s, c2s):
        idx = np.asarray([i for i in lst if i * hop >= 0 and i * hop + n_fft <= len(x)],
                         np.int64)
        idx = idx[~(lv[idx] < level_threshold)] if len(idx) else idx
        if len(idx) == 0:
            res.append((np.zeros(nb), 0))
            continue
        X = np.zeros((len(idx), nb), dtype=np.float32)
        Y = np.zeros((len(idx), nb), dtype=np.float32)
        st = (idx * hop)[:, None] + np.arange(n_fft)[None, :]
        for c in range(ch):
            X += np.abs(np.fft.rfft(x[st, c] * win, axis=-1))
            Y += np.abs(np.fft.rfft(y[st, c] * win, axis=-1))
        X /= ch
        Y /= ch
        X = np.maximum(X, 1e-10)
        med = np.median(Y / X, axis=0)
        res.append((20 * np.log10(med + EPS), len(idx)))
    return freqs, res[0][0], res[1][0], res[0][1], res[1][1]
