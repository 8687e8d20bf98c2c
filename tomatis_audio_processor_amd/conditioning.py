"""Flags for limiter / gain-protect scales that an ill-conditioned sample may set.

Where the OLA window sum is tiny, ``y = out / (sum w^2 + eps)`` amplifies the
float32 rounding of the FFT: the reference's own values there
are rounding noise, and any other implementation's noise differs.  Such a
sample can still set a whole chunk's limiter scale
(src/process_tomatis.py:331-357,447-453; xfade :305-312,335-337), the adaptive
global limiter (src/process_tomatis_adaptive.py:341-345) or the layer-2
gain-protect scale (src/layer2_apply_eq.py:173-179,211-214,220-233).  This
module decides, per chunk, whether the scale is *determined*: whether every
implementation whose per-sample error obeys the bound below must arrive at
the same scale within ``ETA``.

Error model (calibrated, not assumed): a float32 STFT-OLA output sample at
position p differs from the exact result by at most
``KAPPA_INT * A(p) + KAPPA_EDGE * A(p) * S1(p) / den(S2(p))`` where S1/S2 are
the sums of w and w^2 of the frames covering p, ``den`` is the processor's
normaliser and A(p) the local well-conditioned output amplitude.  The first
term is the rounding of the interior (result-sized), the second the FFT
rounding of the numerator divided by a tiny window sum.  numpy's pocketfft
(the reference) measured <= 2.8e-7 and <= 2.0e-8 for the two constants over
160 random streams at 2048/512, 4096/1024, 4096/2048 and 2048/300
(``tests/test_conditioning.py`` re-checks it at 4x); the constants below keep
an 8x margin per implementation, and two implementations then differ by at
most twice the bound.  Note that values at the window edges are not noise:
``z / w`` of the filter's time-aliased tail is large but deterministic, which
is why the edge term is small.

For chunk c with device peak P (before the limiter) and limit T:
  U = max(T, max_p |y(p)| + D(p)),  L = max(T, max_p |y(p)| - D(p))
bound the peak any admissible implementation can see; the scale ``T/peak``
is determined iff ``U - L <= ETA * L``.  Interior samples (full window sums)
contribute at most ``2*(KAPPA_INT + 1.5*KAPPA_EDGE)*A`` and are bounded from
the chunk peaks;
only the first and last ``2*n_fft`` output samples of a stream (where the
window sums differ from the interior) are examined individually.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

KAPPA_INT = 2e-6      # per-implementation, result-sized rounding (8x the measured 2.8e-7)
KAPPA_EDGE = 1.6e-7   # per-implementation, numerator rounding / tiny sum (8x 2.0e-8)
ETA = 5e-5            # scale agreement needed for the 1e-4 sample contract
TAU = 1e-3            # parity mask threshold on sum w^2


def window_sums(n_fft: int, hop: int, first_start: int, n_frames: int,
                pos: np.ndarray):
    """float64 (S1, S2) = (sum w, sum w^2) over the frames covering each
    absolute position in ``pos``; frame j starts at ``first_start + j*hop``."""
    w = np.hanning(n_fft)
    rel = np.asarray(pos, np.int64) - first_start
    s1 = np.zeros(len(rel))
    s2 = np.zeros(len(rel))
    if n_frames <= 0:
        return s1, s2
    jhi = np.minimum(np.floor_divide(rel, hop), n_frames - 1)
    jlo = np.maximum(np.floor_divide(rel - n_fft, hop) + 1, 0)
    for d in range(n_fft // hop + 2):
        j = jhi - d
        ok = (j >= jlo) & (j >= 0)
        idx = rel[ok] - j[ok] * hop
        inr = (idx >= 0) & (idx < n_fft)
        sel = np.nonzero(ok)[0][inr]
        s1[sel] += w[idx[inr]]
        s2[sel] += w[idx[inr]] ** 2
    return s1, s2


def _den(s2: np.ndarray, norm: str) -> np.ndarray:
    return np.maximum(s2, 1e-8) if norm == "max" else s2 + 1e-12


def edge_index(out_len: int, n_fft: int) -> np.ndarray:
    """Output indices of the head and tail ``2*n_fft`` samples (sorted, unique)."""
    k = min(out_len, 2 * n_fft)
    return np.unique(np.concatenate([np.arange(k), np.arange(out_len - k, out_len)]))


def _range_max(v: np.ndarray, lo: np.ndarray, hi: np.ndarray) -> np.ndarray:
    """max(v[lo[t]:hi[t]]) per query t (0 where the range is empty): a sparse
    table of power-of-two range maxima, two overlapping lookups per query
    (exact: the same elements' max as a slice per query)."""
    out = np.zeros(len(lo))
    ln = hi - lo
    ok = ln > 0
    if not ok.any():
        return out
    table = [v]
    k = 1
    while 2 * k <= len(v):
        prev = table[-1]
        table.append(np.maximum(prev[:-k], prev[k:]))  # table[j][i] = max v[i : i + 2^j]
        k *= 2
    idx = np.nonzero(ok)[0]
    j = np.floor(np.log2(ln[idx])).astype(np.int64)
    j = np.where((1 << (j + 1)) <= ln[idx], j + 1, j)  # guard log2 rounding
    j = np.where((1 << j) > ln[idx], j - 1, j)
    for lev in np.unique(j):
        sel = idx[j == lev]
        t = table[lev]
        out[sel] = np.maximum(t[lo[sel]], t[hi[sel] - (1 << lev)])
    return out


def chunk_flags(y_edge: np.ndarray, q_edge: np.ndarray, *, out_begin: int, first_start: int,
                n_frames: int, n_fft: int, hop: int, norm: str,
                chunk_lo: Sequence[int], chunk_hi: Sequence[int],
                peaks: Sequence[float], limit: float) -> List[dict]:
    """Per-chunk determination of a peak-limiter scale.

    ``y_edge`` [len(q_edge), ch]: the output *before* the limiter at output
    indices ``q_edge`` (see :func:`edge_index`); output index q is absolute
    position ``out_begin + q``.  Chunk c spans output indices
    ``[chunk_lo[c], chunk_hi[c])`` and its device peak (before the limiter) is
    ``peaks[c]``.  Returns one dict per chunk: ``flagged``, the admissible
    peak interval ``(lo, hi)`` and ``edge_peak`` (largest edge sample)."""
    y_edge = np.abs(np.asarray(y_edge, np.float64).reshape(len(q_edge), -1)).max(axis=1)
    q_edge = np.asarray(q_edge, np.int64)
    s1, s2 = window_sums(n_fft, hop, first_start, n_frames, out_begin + q_edge)
    good = s2 >= TAU
    # local amplitude: largest well-conditioned |y| within +-n_fft
    A = np.zeros(len(q_edge))
    gq, gy = q_edge[good], y_edge[good]
    if len(gq):
        lo_i = np.searchsorted(gq, q_edge - n_fft, "left")
        hi_i = np.searchsorted(gq, q_edge + n_fft, "right")
        A = _range_max(gy, lo_i, hi_i)
    D = 2.0 * (KAPPA_INT * A + KAPPA_EDGE * A * s1 / _den(s2, norm))
    out = []
    nc = len(peaks)
    # q_edge is sorted: chunk c's edge samples are one slice of it
    ia = np.searchsorted(q_edge, np.asarray(chunk_lo, np.int64), "left")
    ib = np.searchsorted(q_edge, np.asarray(chunk_hi, np.int64), "left")
    for c in range(nc):
        P = float(peaks[c])
        m = slice(int(ia[c]), int(max(ia[c], ib[c])))
        # interior samples: full window sums (S1/S2 <= 1.5 for the overlaps used)
        amp_int = max(float(peaks[max(c - 1, 0)]), P, float(peaks[min(c + 1, nc - 1)]))
        d_int = 2.0 * (KAPPA_INT + 1.5 * KAPPA_EDGE) * amp_int
        hi = P + d_int
        lo = P - d_int
        edge_peak = 0.0
        if m.stop > m.start:
            ye, de = y_edge[m], D[m]
            edge_peak = float(ye.max())
            hi = max(hi, float((ye + de).max()))
            if edge_peak >= P:        # the peak sample itself is an edge sample
                lo = float((ye - de).max())
            else:
                lo = max(lo, float((ye - de).max()))
        U, L = max(limit, hi), max(limit, lo)
        flagged = bool(U > limit and (U - L) > ETA * L)
        out.append(dict(flagged=flagged, lo=lo, hi=hi, edge_peak=edge_peak, peak=P))
    return out


def result_flags(res, i: int, *, n_fft: int, norm: str, limit: Optional[float],
                 chunk_ranges=None) -> List[dict]:
    """:func:`chunk_flags` for stream ``i`` of an ``engine.Result``.

    The device output is downloaded only at the stream's edges.  ``limit``:
    the limiter threshold whose scale was applied on the device (its effect is
    divided out), or the gain-protect target (nothing applied yet)."""
    n = res.out_lens[i]
    ch = res.ch
    if n == 0:
        return []
    q = edge_index(n, n_fft)
    a = res.out_offs[i]
    ydev = res.y[a:a + n * ch].view(-1, ch)
    import torch
    y = ydev[torch.as_tensor(q, device=ydev.device)].cpu().numpy().astype(np.float64)
    peaks = [float(p) for p in res.stream_peaks(i)]
    if chunk_ranges is None:
        chunk_ranges = [(0, n)]
    lo = [r[0] for r in chunk_ranges]
    hi = [r[1] for r in chunk_ranges]
    applied = limit is not None and res.extra.get("limiter_applied", False)
    if applied:
        # undo the device limiter on the edge samples: scale = limit / peak
        for c, (qa, qb) in enumerate(chunk_ranges):
            if peaks[c] > limit:
                sel = (q >= qa) & (q < qb)
                y[sel] *= peaks[c] / np.float32(limit)
    return chunk_flags(y, q, out_begin=res.extra.get("out_begin", [0] * (i + 1))[i],
                       first_start=res.first_start[i], n_frames=res.n_frames[i], n_fft=n_fft,
                       hop=res.hop, norm=norm, chunk_lo=lo, chunk_hi=hi, peaks=peaks,
                       limit=limit if limit is not None else np.inf)
