"""Analysis spectra on the device: the validators' and calibration tools' STFTs
(SURVEY.md §8 rows f3/f4), same names, arguments, return values and errors as
the reference functions:

  stft_mag_avg                  src/compare_audio.py:12-24
  power_mono                    src/compare_audio.py:7-10
  stft_logpower_median          src/layer2_analyze_eq.py:54-88
  find_stable_frames            src/validate_layer1.py:245-258 (host: list logic)
  compute_conditional_spectrum  src/validate_layer1.py:261-389

Everything per frame or per sample runs in ``libtomatis_hip.so``
(``tm_analysis.hip``): framing, power-mono premix, window, real FFT (two real
frames per complex FFT), |X| / log-power / Y-over-X ratios, the per-frame
level (bit-exact numpy pairwise order) and its gate predicate, the mean and the
median over frames.  The host keeps once-per-call set-up (window, rfftfreq,
the level threshold as r bit patterns via ``dsp.gate_bits``, the stable-frame
classes from the state list) and the bins-sized final ``20*log10`` of the
validator.  Inputs may be numpy arrays (uploaded) or resident cuda tensors.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import dsp
from ._lib import check, lib, ptr, stream_handle

EPS = 1e-12
AN_LEVEL_CHMEAN, AN_LEVEL_POWER_MONO = 0, 1
AN_SIG_RAW, AN_SIG_POWER_MONO = 0, 1
AN_MAG, AN_LOGPOW, AN_RATIO = 0, 1, 2
MIN_N_FFT = 16               # tm_analysis.hip kMinN
MAX_N_FFT = 16384            # kMaxM: one FFT in LDS
MAX_N_FFT_BLUESTEIN = 8192   # 2 n_fft - 1 <= kMaxM


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("analysis spectra need a ROCm GPU (MI355X); there is no CPU fallback")
    return torch


def _dev(a, ch=None):
    """float32 contiguous cuda tensor of shape [n] or [n, ch]."""
    torch = _torch()
    if isinstance(a, torch.Tensor):
        t = a.to(device="cuda", dtype=torch.float32).contiguous()
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float32))).cuda()
    if ch is not None and t.dim() == 1:
        t = t.reshape(-1, 1)
    return t


def _check_n_fft(n_fft):
    """Any length np.fft.rfft takes, within the LDS: powers of two in
    [16, MAX_N_FFT], other lengths in [16, MAX_N_FFT_BLUESTEIN] (Bluestein's
    chirp-z runs a power-of-two FFT of >= 2 n_fft - 1 points)."""
    pow2 = n_fft > 0 and (n_fft & (n_fft - 1)) == 0
    cap = MAX_N_FFT if pow2 else MAX_N_FFT_BLUESTEIN
    if n_fft < MIN_N_FFT or n_fft > cap:
        raise ValueError(f"n_fft={n_fft}: the analysis kernels take {MIN_N_FFT} <= n_fft <= "
                         f"{cap} ({'power of two' if pow2 else 'Bluestein'}), as tm_analysis.hip")


def _n_frames(n, n_fft, hop):
    return 1 + (n - n_fft) // hop  # Python floor division, as the reference loops


def _spectra(x, y, n, ch, n_fft, hop, kind, sig, scale=1.0):
    torch = _torch()
    F = _n_frames(n, n_fft, hop)
    nb = n_fft // 2 + 1
    win = torch.from_numpy(dsp.hann(n_fft)).cuda()
    out = torch.empty((F, nb), dtype=torch.float32, device="cuda")
    check(lib().tomatis_an_spectra(ptr(x), ptr(y), n, ch, n_fft, hop, kind, sig,
                                   C.c_float(scale), ptr(win), ptr(out), stream_handle()),
          "an_spectra")
    return out


def _frame_r(x, n, ch, n_fft, hop, mode, scale=1.0):
    torch = _torch()
    r = torch.empty(_n_frames(n, n_fft, hop), dtype=torch.float32, device="cuda")
    check(lib().tomatis_an_frame_r(ptr(x), n, ch, n_fft, hop, mode, C.c_float(scale), ptr(r),
                                   stream_handle()), "an_frame_r")
    return r


def _select(r, thr_bits, exc, keep_above, cls=None, cls_want=0):
    """Device frame mask from exact level predicates; returns (mask, count)."""
    torch = _torch()
    F = r.numel()
    mask = torch.empty(F, dtype=torch.uint8, device="cuda")
    cnt = torch.empty(1, dtype=torch.int32, device="cuda")
    ex = (C.c_uint32 * 4)(*(list(exc) + [0] * (4 - len(exc))))
    check(lib().tomatis_an_select(ptr(r), F, thr_bits, ex, len(exc), keep_above, ptr(cls),
                                  cls_want, ptr(mask), ptr(cnt), stream_handle()), "an_select")
    return mask, int(cnt.item())


def frame_median(spec, mask=None, n_sel=None):
    """np.median(spec[mask], axis=0) on the device (float32, numpy's even rule)."""
    torch = _torch()
    F, nb = spec.shape
    n_sel = F if n_sel is None else n_sel
    work = torch.empty(int(lib().tomatis_an_median_work_words(nb)), dtype=torch.int32,
                       device="cuda")
    out = torch.empty(nb, dtype=torch.float32, device="cuda")
    check(lib().tomatis_an_frame_median(ptr(spec), F, nb, ptr(mask), n_sel, ptr(work), ptr(out),
                                        stream_handle()), "an_frame_median")
    return out


def frame_mean(spec):
    """spec.mean(axis=0) on the device in numpy's axis-0 order."""
    torch = _torch()
    F, nb = spec.shape
    out = torch.empty(nb, dtype=torch.float32, device="cuda")
    check(lib().tomatis_an_frame_mean(ptr(spec), F, nb, ptr(out), stream_handle()),
          "an_frame_mean")
    return out


# ---------------------------------------------------------------------------
# reference-named functions
# ---------------------------------------------------------------------------

def power_mono(x_lr):
    """compare_audio.py:7-10 — host numpy (elementwise, used for inputs/CSV only).
    The device fuses the same formula into the spectrum and level kernels."""
    p = 0.5 * (x_lr[:, 0] ** 2 + x_lr[:, 1] ** 2)
    return np.sqrt(p + EPS)


def stft_mag_avg(x, sr, n_fft=4096, hop=2048, *, premix=None, scale=1.0, as_tensor=False):
    """compare_audio.stft_mag_avg: mean over frames of |rfft(win * x[f*hop:+n_fft])|.

    ``x`` is the mono signal (1-D), or with ``premix="power_mono"`` the stereo
    ``[n, 2]`` whose power mono the reference would pass (fused on the device).
    ``scale`` multiplies the PCM first (compare_audio.py:82-86 scales the
    candidate before power_mono)."""
    _check_n_fft(n_fft)
    if premix == "power_mono":
        xd = _dev(x, ch=2)
        if xd.shape[1] != 2:
            raise ValueError("power_mono premix needs a stereo [n, 2] input")
        sig, ch = AN_SIG_POWER_MONO, 2
    else:
        xd = _dev(x).reshape(-1)
        sig, ch = AN_SIG_RAW, 1
    n = xd.shape[0]
    if _n_frames(n, n_fft, hop) <= 0:
        raise ValueError("need at least one array to stack")  # np.stack([]) in the reference
    spec = _spectra(xd, None, n, ch, n_fft, hop, AN_MAG, sig, scale)
    m = frame_mean(spec)
    return m if as_tensor else m.cpu().numpy()


def stft_logpower_median(x_lr, sr: int, n_fft: int, hop: int, music_dbfs: float):
    """layer2_analyze_eq.stft_logpower_median -> (freqs, median_logP_dB, used_frames).

    Frames whose power-mono level is <= music_dbfs are dropped (exact, on the bit
    pattern of r); the median over the kept frames of 10 log10(|X|^2 + EPS)."""
    _check_n_fft(n_fft)
    freqs = np.fft.rfftfreq(n_fft, 1.0 / sr)
    xd = _dev(x_lr, ch=2)
    if xd.shape[1] != 2:
        raise ValueError("stft_logpower_median expects a stereo [n, 2] input")
    n = xd.shape[0]
    F = _n_frames(n, n_fft, hop)
    if F <= 10:
        raise ValueError("片段太短，无法做稳定频谱统计。")
    r = _frame_r(xd, n, 2, n_fft, hop, AN_LEVEL_POWER_MONO)
    _, _, off_bits, off_exc = dsp.gate_bits(float(music_dbfs), float(music_dbfs))
    mask, used = _select(r, off_bits, off_exc, keep_above=0)
    if used < 50:
        raise ValueError(f"可用音乐帧太少（{used} 帧）。把 --music_dbfs 调低一点（例如 -70）。")
    spec = _spectra(xd, None, n, 2, n_fft, hop, AN_LOGPOW, AN_SIG_POWER_MONO)
    med = frame_median(spec, mask, used)
    return freqs, med.cpu().numpy(), used


def _stable_classes(states, margin=2):
    """int8 per state index: 1 = stable C1, 2 = stable C2, 0 = neither
    (validate_layer1.find_stable_frames' rule, vectorised)."""
    s = None
    try:  # fast path: a list of "C1"/"C2" strings joined into one byte buffer
        b = np.frombuffer("".join(states).encode("ascii"), np.uint8)
        if b.size == 2 * len(states) and np.all(b[0::2] == ord("C")):
            d = b[1::2]
            s = np.where(d == ord("1"), 1, np.where(d == ord("2"), 2, 0)).astype(np.int8)
    except (TypeError, UnicodeEncodeError):
        s = None
    if s is None:
        s = np.asarray([1 if v == "C1" else (2 if v == "C2" else 0) for v in states], np.int8)
    n = len(s)
    cls = np.zeros(n, np.int8)
    if n - 2 * margin <= 0:
        return cls
    win = np.lib.stride_tricks.sliding_window_view(s, 2 * margin + 1)  # starts at i - margin
    cls[margin:n - margin][np.all(win == 1, axis=1)] = 1
    cls[margin:n - margin][np.all(win == 2, axis=1)] = 2
    return cls


def find_stable_frames(states, margin=2):
    """validate_layer1.find_stable_frames: indices whose +-margin window is all
    C1 (first list) or all C2 (second list)."""
    cls = _stable_classes(states, margin)
    return np.nonzero(cls == 1)[0].tolist(), np.nonzero(cls == 2)[0].tolist()


def compute_conditional_spectrum(x, y, sr, states, n_fft, hop, level_threshold=-60):
    """validate_layer1.compute_conditional_spectrum ->
    (freqs, c1_db, c2_db, n_c1_frames, n_c2_frames).

    Per stable frame (fully inside x, level >= level_threshold) the ratio
    mean_c|Y_c| / max(mean_c|X_c|, 1e-10); median over frames per class;
    20 log10(median + EPS)."""
    _check_n_fft(n_fft)
    torch = _torch()
    xd = _dev(x, ch=True)
    yd = _dev(y, ch=True)
    n, ch = xd.shape
    if ch not in (1, 2) or yd.shape[1] != ch:
        raise ValueError("x and y must have the same channel count (1 or 2)")
    if yd.shape[0] < n:
        raise ValueError("y must be at least as long as x")
    yd = yd[:n].contiguous()
    freqs = np.fft.rfftfreq(n_fft, 1 / sr)
    nb = len(freqs)
    F = max(0, _n_frames(n, n_fft, hop))  # frames idx with idx*hop + n_fft <= len(x)
    cls = np.zeros(F, np.int8)
    sc = _stable_classes(states, margin=2)[:F]
    cls[:len(sc)] = sc
    out = []
    if F > 0:
        r = _frame_r(xd, n, ch, n_fft, hop, AN_LEVEL_CHMEAN)
        on_bits, on_exc, _, _ = dsp.gate_bits(float(level_threshold), float(level_threshold))
        cls_d = torch.from_numpy(cls).cuda()
        sel = [_select(r, on_bits, on_exc, keep_above=1, cls=cls_d, cls_want=v) for v in (1, 2)]
        spec = _spectra(xd, yd, n, ch, n_fft, hop, AN_RATIO, AN_SIG_RAW) \
            if any(c for _, c in sel) else None
    else:
        sel = [(None, 0), (None, 0)]
    for mask, cnt in sel:
        if cnt:
            med = frame_median(spec, mask, cnt).cpu().numpy()
            out.append(20 * np.log10(med + EPS))
        else:
            out.append(np.zeros(nb))
    return freqs, out[0], out[1], sel[0][1], sel[1][1]
