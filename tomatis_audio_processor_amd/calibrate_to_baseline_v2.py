"""Gate calibration against a baseline recording — MI355X drop-in for
src/calibrate_to_baseline_v2.py.

Same functions, flags, defaults, printed report and output JSON as the
reference; the per-frame and per-candidate work runs in ``libtomatis_hip.so``:

  reference (file:line)                        here
  -------------------------------------------- ----------------------------------
  power_mono / rms_dbfs_from_mono :8-15,196-197 tomatis_an_frame_r (POWER_MONO r,
                                               bit-exact numpy pairwise mean) + the
                                               reference's float32 20*log10 on host
  stft_band_tilt :17-31 (per frame)            tomatis_an_band_energy (rfft of
                                               win * power_mono, band power sums)
  simulate_state :84-109 x the grid :231-265   tomatis_cal_gate_grid: one lane per
     (gain x up-delay x hysteresis x T)        (gain, up_ms, hyst, T) candidate,
                                               mismatch / switch counts
  debounce_state :111-128, kmeans2_1d :33-44,  host (once per file, O(frames),
  medfilt, the score / arg-min :258-265        same numpy/scipy calls)
  find_delay_by_corr :46-82                    host scipy (resample_poly,
                                               fftconvolve), as the reference

The argmin is taken on the host from the device's exact integer counts in the
reference's own loop order with its own float64 score, so ``best`` is the
reference's.  Band tilts come from this build's FFT (float32 rounding differs
from pocketfft's by ~1e-7 relative); they only feed the tilt clustering.
"""
from __future__ import annotations

import argparse
import json

import numpy as np

from . import audio_io
from ._lib import GATE_CAND_DTYPE, check, lib, ptr, stream_handle

EPS = 1e-12


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("gate calibration needs a ROCm GPU (MI355X); there is no CPU fallback")
    return torch


# ---------------------------------------------------------------------------
# reference-named helpers
# ---------------------------------------------------------------------------

def power_mono(x_lr: np.ndarray) -> np.ndarray:
    """calibrate_to_baseline_v2.py:8-11 (host, elementwise)."""
    p = 0.5 * (x_lr[:, 0] * x_lr[:, 0] + x_lr[:, 1] * x_lr[:, 1])
    return np.sqrt(p + EPS)


def rms_dbfs_from_mono(mono: np.ndarray) -> float:
    """calibrate_to_baseline_v2.py:13-15 (host, one frame)."""
    r = np.sqrt(np.mean(mono * mono) + EPS)
    return float(20 * np.log10(r + EPS))


def frame_levels(x_lr, n_fft: int, hop: int) -> np.ndarray:
    """float32 levels of frames f*hop (f < 1 + (n - n_fft)//hop):
    rms_dbfs_from_mono(power_mono(frame)) as main() stores them (:185,196-197).
    r on the device (numpy's pairwise order, bit-exact), the reference's float32
    ``20*log10(r + EPS)`` on the host."""
    from .analysis import AN_LEVEL_POWER_MONO, _dev, _frame_r
    xd = _dev(x_lr, ch=2)
    n = xd.shape[0]
    if n < n_fft:
        return np.zeros(0, np.float32)
    r = _frame_r(xd, n, 2, n_fft, hop, AN_LEVEL_POWER_MONO).cpu().numpy()
    return (np.float32(20) * np.log10(r + np.float32(EPS))).astype(np.float32)


def _band_bins(sr, n_fft, band):
    freqs = np.fft.rfftfreq(n_fft, 1 / sr)
    m = (freqs >= band[0]) & (freqs < band[1])
    idx = np.nonzero(m)[0]
    return (int(idx[0]), int(idx[-1]) + 1) if len(idx) else (0, 0)


def band_tilts(x_lr, sr: int, n_fft: int, hop: int, lo=(200, 1000), hi=(2000, 8000)):
    """stft_band_tilt (:17-31) of every frame f*hop, float32 as main() stores
    them (:187,198): 10*log10(Ehi/Elo + EPS) with E = float32 band power sums
    of rfft(hanning * power_mono(frame)) plus EPS."""
    from . import dsp
    from .analysis import _dev
    torch = _torch()
    xd = _dev(x_lr, ch=2)
    n = xd.shape[0]
    if n < n_fft:
        return np.zeros(0, np.float32)
    F = 1 + (n - n_fft) // hop
    lo0, lo1 = _band_bins(sr, n_fft, lo)
    hi0, hi1 = _band_bins(sr, n_fft, hi)
    win = torch.from_numpy(dsp.hann(n_fft)).cuda()
    out = torch.empty((F, 2), dtype=torch.float32, device="cuda")
    check(lib().tomatis_an_band_energy(ptr(xd), n, n_fft, hop, lo0, lo1, hi0, hi1, ptr(win),
                                       ptr(out), stream_handle()), "an_band_energy")
    e = out.cpu().numpy()
    elo = (e[:, 0] + np.float32(EPS)).astype(np.float64)   # float(np.sum(P[lo]) + EPS)
    ehi = (e[:, 1] + np.float32(EPS)).astype(np.float64)
    return (10 * np.log10(ehi / elo + EPS)).astype(np.float32)


def stft_band_tilt(frame_lr: np.ndarray, sr: int, n_fft: int, lo=(200, 1000),
                   hi=(2000, 8000)) -> float:
    """calibrate_to_baseline_v2.py:17-31 for one frame (device FFT)."""
    return float(band_tilts(np.asarray(frame_lr, np.float32)[:n_fft], sr, n_fft, n_fft,
                            lo, hi)[0])


def kmeans2_1d(x: np.ndarray, iters=25):
    """calibrate_to_baseline_v2.py:33-44 (host; same numpy operations)."""
    m1, m2 = np.percentile(x, [30, 70]).astype(float)
    for _ in range(iters):
        d1 = np.abs(x - m1)
        d2 = np.abs(x - m2)
        c1 = x[d1 <= d2]
        c2 = x[d1 > d2]
        if len(c1) > 0:
            m1 = float(np.mean(c1))
        if len(c2) > 0:
            m2 = float(np.mean(c2))
    lab = (np.abs(x - m2) < np.abs(x - m1)).astype(np.int32)
    return lab, m1, m2


def debounce_state(state: np.ndarray, min_run: int = 3) -> np.ndarray:
    """calibrate_to_baseline_v2.py:111-128: runs shorter than ``min_run`` take
    the value on their left (the right for a leading run), left to right over
    the already-debounced sequence.  Walks runs, not frames."""
    s = np.array(state, copy=True)
    n = len(s)
    if n == 0:
        return s
    cut = np.nonzero(s[1:] != s[:-1])[0] + 1
    starts = np.concatenate([[0], cut])
    ends = np.concatenate([cut, [n]])
    for i, j in zip(starts.tolist(), ends.tolist()):
        if j - i < min_run:
            left = s[i - 1] if i > 0 else (s[j] if j < n else s[i])
            s[i:j] = left
    return s


def find_delay_by_corr(orig_path, base_path, sr=48000, ds_sr=2000, chunk_sec=25):
    """calibrate_to_baseline_v2.py:46-82: delay (orig - base) in samples from the
    cross-correlation of 2 kHz power-mono envelopes (host scipy, as the reference)."""
    from scipy.signal import fftconvolve, resample_poly
    xo, sro = audio_io.read(orig_path)
    xb, srb = audio_io.read(base_path)
    assert sro == sr and srb == sr
    assert xo.shape[1] == 2 and xb.shape[1] == 2
    nbase = len(xb)
    mid = int(0.5 * nbase)
    half = int(0.5 * chunk_sec * sr)
    s = max(0, mid - half)
    e = min(nbase, mid + half)
    mb = power_mono(xb[s:e])
    mb_ds = resample_poly(mb, ds_sr, sr).astype(np.float32)
    mb_ds = mb_ds - np.mean(mb_ds)
    mo = power_mono(xo).astype(np.float32)
    mo_ds = resample_poly(mo, ds_sr, sr).astype(np.float32)
    mo_ds = mo_ds - np.mean(mo_ds)
    corr = fftconvolve(mo_ds, mb_ds[::-1], mode="valid")
    k = int(np.argmax(corr))
    base_center = (s + (e - s) // 2) / sr
    orig_center = (k + len(mb_ds) // 2) / ds_sr
    return int(round((orig_center - base_center) * sr))


def _grid(levels_rows, starts, target, cands, want_states=False):
    """Run the candidate grid on the device: (counts [n, 2] int32, states)."""
    torch = _torch()
    lv = torch.from_numpy(np.ascontiguousarray(levels_rows, np.float32)).cuda()
    st = torch.from_numpy(np.ascontiguousarray(starts, np.int64)).cuda()
    tg = (torch.from_numpy(np.ascontiguousarray(target, np.int32)).cuda()
          if target is not None else None)
    cb = torch.from_numpy(np.ascontiguousarray(cands).view(np.uint8)).cuda()
    n_fit = int(len(starts))
    out = torch.empty((max(1, len(cands)), 2), dtype=torch.int32, device="cuda")
    states = (torch.empty((max(1, len(cands)), max(1, n_fit)), dtype=torch.uint8, device="cuda")
              if want_states else None)
    check(lib().tomatis_cal_gate_grid(ptr(lv), n_fit, ptr(st), ptr(tg), ptr(cb), len(cands),
                                      ptr(out), ptr(states), stream_handle()), "cal_gate_grid")
    cnt = out.cpu().numpy()[:len(cands)]
    return cnt, (states.cpu().numpy()[:len(cands), :n_fit] if want_states else None)


def _cand(row, T, hyst, up_ms, sr):
    c = np.zeros(1, GATE_CAND_DTYPE)
    c["level_row"] = row
    # numpy compares an np.float32 level with a Python float in float32 (NEP 50)
    c["t_on"] = np.float32(float(T) + float(hyst) / 2)
    c["t_off"] = np.float32(float(T) - float(hyst) / 2)
    c["up_delay"] = int(round(sr * float(up_ms) / 1000.0))
    return c


def simulate_state(level_dbfs: np.ndarray, frame_starts: np.ndarray, sr: int, T: float,
                   hyst: float, up_delay_ms: float) -> np.ndarray:
    """calibrate_to_baseline_v2.py:84-109 on the device: int32 states (1/2)."""
    lv = np.asarray(level_dbfs, np.float32)
    _, st = _grid(lv[None, :], frame_starts, None, _cand(0, T, hyst, up_delay_ms, sr),
                  want_states=True)
    return st[0].astype(np.int32)


def search_grid(orig_level, base_state, music_mask, frame_starts, sr, *, gain_search_pm_db=3.0,
                gain_step_db=0.5, T_pm_db=10.0, T_step_db=0.25,
                delay_list_ms=(0, 50, 100, 150, 200, 250), hyst_list=(0, 1, 2, 3, 4, 6),
                base_level=None):
    """The search of calibrate_to_baseline_v2.py:227-265: every candidate on the
    device in one launch, the reference's score and first-strict-minimum on the
    host.  Returns (best dict or None, gain_db0, n_candidates)."""
    gain_db0 = float(np.median((base_level - orig_level)[music_mask]))
    gains = np.arange(gain_db0 - gain_search_pm_db, gain_db0 + gain_search_pm_db + 1e-9,
                      gain_step_db).astype(np.float32)
    idx = np.flatnonzero(music_mask)
    fs_fit = frame_starts[idx]
    s_fit = base_state[idx]
    rows, cands, meta = [], [], []
    for gain_db in gains:
        levels_adj = (orig_level + gain_db)[idx]
        c1 = levels_adj[s_fit == 1]
        c2 = levels_adj[s_fit == 2]
        if len(c1) < 10 or len(c2) < 10:
            continue
        T0 = 0.5 * (float(np.median(c1)) + float(np.median(c2)))
        Ts = np.arange(T0 - T_pm_db, T0 + T_pm_db + 1e-9, T_step_db).astype(np.float32)
        row = len(rows)
        rows.append(levels_adj)
        for up_ms in delay_list_ms:
            for hyst in hyst_list:
                for T in Ts:
                    cands.append(_cand(row, T, hyst, up_ms, sr))
                    meta.append((float(T), float(hyst), float(up_ms), float(gain_db), float(T0)))
    if not cands:
        return None, gain_db0, 0
    cnt, _ = _grid(np.stack(rows), fs_fit, s_fit, np.concatenate(cands))
    n = len(s_fit)
    best = None
    for (T, hyst, up_ms, gain_db, T0), (mis, sw) in zip(meta, cnt.tolist()):
        mismatch = float(mis / n)          # np.mean of a bool array: exact count / n
        score = mismatch + 1e-5 * sw
        if best is None or score < best["score"]:
            best = dict(score=score, mismatch=mismatch, switches=int(sw), T=T, hyst=hyst,
                        up_ms=up_ms, gain_db=gain_db, T0=T0)
    return best, gain_db0, len(cands)


def calibrate(orig, base, gate_ui=50.0, gate_scale=1.0, n_fft=4096, hop=2048, sr=48000,
              max_minutes=6.0, hyst_list=(0, 1, 2, 3, 4, 6),
              delay_list_ms=(0, 50, 100, 150, 200, 250), tilt_lo=(200, 1000),
              tilt_hi=(2000, 8000), tilt_medfilt=5, music_dbfs=-65.0, gain_search_pm_db=3.0,
              gain_step_db=0.5, T_pm_db=10.0, T_step_db=0.25, log=print):
    """main() of the reference minus argparse and the JSON file: returns the
    dict it saves (calibrate_to_baseline_v2.py:159-307)."""
    from scipy.signal import medfilt
    delay = find_delay_by_corr(orig, base, sr=sr)
    log(f"[ALIGN] estimated delay (orig - base): {delay} samples ({delay/sr*1000:.2f} ms)")
    xo_all, sro = audio_io.read(orig)
    xb_all, srb = audio_io.read(base)
    assert sro == sr and srb == sr
    assert xo_all.shape[1] == 2 and xb_all.shape[1] == 2
    base_start = max(0, -delay)
    orig_start = max(0, delay)
    max_len = int(max_minutes * 60 * sr)
    avail = min(len(xb_all) - base_start, len(xo_all) - orig_start, max_len)
    if avail <= n_fft:
        raise ValueError("重叠可用长度太短，无法校准。")
    xb = xb_all[base_start:base_start + avail]
    xo = xo_all[orig_start:orig_start + avail]
    n_frames = 1 + (avail - n_fft) // hop
    frame_starts = (np.arange(n_frames) * hop).astype(np.int64)
    orig_level = frame_levels(xo, n_fft, hop)
    base_level = frame_levels(xb, n_fft, hop)
    tilts = band_tilts(xb, sr, n_fft, hop, tuple(tilt_lo), tuple(tilt_hi))

    music_mask = base_level > music_dbfs
    music_ratio = float(np.mean(music_mask))
    log(f"[MASK] music frames ratio: {music_ratio*100:.1f}% (threshold {music_dbfs} dBFS)")
    if music_ratio < 0.2:
        log("[WARN] 可用音乐帧太少，建议把 --music_dbfs 调低一点（例如 -70）")
    k = int(tilt_medfilt)
    if k % 2 == 0:
        k += 1
    if k < 3:
        k = 3
    tilts_s = medfilt(tilts, kernel_size=k).astype(np.float32)
    lab, _, _ = kmeans2_1d(tilts_s[music_mask])
    base_state = np.ones(n_frames, np.int32)
    base_state[music_mask] = np.where(lab == 1, 2, 1).astype(np.int32)
    mean1 = float(np.mean(tilts_s[music_mask][lab == 1])) if np.any(lab == 1) else -1e9
    mean0 = float(np.mean(tilts_s[music_mask][lab == 0])) if np.any(lab == 0) else -1e9
    if mean0 > mean1:
        base_state[music_mask] = np.where(lab == 0, 2, 1).astype(np.int32)
    base_state = debounce_state(base_state, min_run=3)
    log(f"[GAIN] initial gain_db0 (base - orig): "
        f"{float(np.median((base_level - orig_level)[music_mask])):.2f} dB")
    best, gain_db0, _ = search_grid(orig_level, base_state, music_mask, frame_starts, sr,
                                    gain_search_pm_db=gain_search_pm_db,
                                    gain_step_db=gain_step_db, T_pm_db=T_pm_db,
                                    T_step_db=T_step_db, delay_list_ms=delay_list_ms,
                                    hyst_list=hyst_list, base_level=base_level)
    if best is None:
        raise RuntimeError("未找到可用最优解：请放宽 --music_dbfs 或增大 --max_minutes。")
    T_adj = best["T"]
    gain_db = best["gain_db"]
    T_raw = T_adj - gain_db
    gate_offset = T_raw - gate_scale * gate_ui
    log("\n[BEST]")
    log(best)
    log(f"\n[RECOMMEND] gain_db (diagnostic only): {gain_db:+.2f} dB (base - orig)")
    log(f"[RECOMMEND] T_adj (on leveled orig): {T_adj:.2f} dBFS")
    log(f"[RECOMMEND] T_raw (for process_tomatis): {T_raw:.2f} dBFS")
    log(f"[RECOMMEND] gate_ui={gate_ui:.1f}, gate_scale={gate_scale:.2f}, "
        f"gate_offset={gate_offset:.2f}")
    log(f"[RECOMMEND] hyst_db={best['hyst']:.1f}, up_delay_ms={best['up_ms']:.0f}")
    log(f"[RECOMMEND] mismatch={best['mismatch']*100:.2f}%, switches={best['switches']} "
        "(on music frames)")
    out = {
        "orig": orig,
        "base": base,
        "delay_samples_orig_minus_base": int(delay),
        "music_dbfs": float(music_dbfs),
        "gain_db_base_minus_orig": float(gain_db),
        "T_adj_dbfs": float(T_adj),
        "T_raw_dbfs": float(T_raw),
        "gate_ui": float(gate_ui),
        "gate_scale": float(gate_scale),
        "gate_offset": float(gate_offset),
        "hyst_db": float(best["hyst"]),
        "up_delay_ms": float(best["up_ms"]),
        "mismatch": float(best["mismatch"]),
        "switches": int(best["switches"]),
    }
    return out, dict(best=best, orig_level=orig_level, base_level=base_level, tilts=tilts,
                     base_state=base_state, music_mask=music_mask)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--orig", required=True)
    ap.add_argument("--base", required=True)
    ap.add_argument("--gate_ui", type=float, default=50.0)
    ap.add_argument("--gate_scale", type=float, default=1.0)
    ap.add_argument("--n_fft", type=int, default=4096)
    ap.add_argument("--hop", type=int, default=2048)
    ap.add_argument("--sr", type=int, default=48000)
    ap.add_argument("--max_minutes", type=float, default=6.0)
    ap.add_argument("--hyst_list", type=float, nargs="+", default=[0, 1, 2, 3, 4, 6])
    ap.add_argument("--delay_list_ms", type=float, nargs="+", default=[0, 50, 100, 150, 200, 250])
    ap.add_argument("--tilt_lo", type=int, nargs=2, default=[200, 1000])
    ap.add_argument("--tilt_hi", type=int, nargs=2, default=[2000, 8000])
    ap.add_argument("--tilt_medfilt", type=int, default=5, help="tilt 中值滤波核大小(奇数), 3/5/7")
    ap.add_argument("--music_dbfs", type=float, default=-65.0, help="只在基准音量高于此阈值的帧上拟合")
    ap.add_argument("--gain_search_pm_db", type=float, default=3.0, help="围绕初始 gain_db0 的搜索范围 ±dB")
    ap.add_argument("--gain_step_db", type=float, default=0.5)
    ap.add_argument("--T_pm_db", type=float, default=10.0, help="围绕 T0 搜索范围 ±dB")
    ap.add_argument("--T_step_db", type=float, default=0.25)
    ap.add_argument("--out_json", default="calibration_v2.json")
    a = ap.parse_args(argv)
    out, _ = calibrate(a.orig, a.base, gate_ui=a.gate_ui, gate_scale=a.gate_scale, n_fft=a.n_fft,
                       hop=a.hop, sr=a.sr, max_minutes=a.max_minutes, hyst_list=a.hyst_list,
                       delay_list_ms=a.delay_list_ms, tilt_lo=a.tilt_lo, tilt_hi=a.tilt_hi,
                       tilt_medfilt=a.tilt_medfilt, music_dbfs=a.music_dbfs,
                       gain_search_pm_db=a.gain_search_pm_db, gain_step_db=a.gain_step_db,
                       T_pm_db=a.T_pm_db, T_step_db=a.T_step_db)
    with open(a.out_json, "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=2)
    print(f"\n[SAVED] {a.out_json}")


if __name__ == "__main__":
    main()


__all__ = ["power_mono", "rms_dbfs_from_mono", "stft_band_tilt", "kmeans2_1d",
           "find_delay_by_corr", "simulate_state", "debounce_state", "frame_levels",
           "band_tilts", "search_grid", "calibrate", "main"]
