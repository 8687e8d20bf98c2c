"""Device orchestration of the STFT-gate-OLA hot path on MI355X.

A *stream set* is a batch of equal-format PCM streams (same sr, ch) resident
in one flat float32 HBM buffer (interleaved ``[n][ch]`` per stream).  A
pipeline builds one ``tomatis_plan`` for the set (work decomposition, tables)
and allocates every per-frame / per-chunk buffer up front, so ``run()`` only
launches kernels on the current stream (no host sync for the standard, xfade
and EQ paths; the adaptive path syncs once for the level percentiles).

Reference behaviour reproduced per mode (file:line):
  standard  src/process_tomatis.py:160-457
  xfade     src/process_tomatis_xfade.py:55-341
  adaptive  src/process_tomatis_adaptive.py:157-351
  layer2    src/layer2_apply_eq.py:66-233
  layer2b   src/layer2b_apply_residual_eq.py:57-160 (+ _safe.py)
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import time
import warnings
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import dsp
from ._lib import (E_UNSUPPORTED, ERR_GATE_CARRY, ERR_LIMITER_WAIT, ERR_PAIR_BARRIER, F32, F64, NORM_EPS, NORM_MAX,
                   OPT_FUSE_LIMITER, OPT_LIMITER_SPIN, OPT_MINHOLD_SERIAL, TomatisPlanDesc, TomatisStream, check, lib,
                   ptr, stream_handle)

PEAK_LIMIT = 0.999
# host<->HBM copies of file-sized buffers go through page-locked staging
PINNED_STAGING = True


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("tomatis_audio_processor_amd needs a ROCm GPU (MI355X); "
                           "torch.cuda.is_available() is False and there is no CPU fallback")
    return torch


@dataclass
class StreamSet:
    """Equal-format streams in one flat device buffer."""
    x: object                 # torch.float32 cuda tensor (flat)
    offs: List[int]           # float offset of each stream's sample 0
    lens: List[int]           # samples per channel
    ch: int
    sr: int

    @classmethod
    def from_arrays(cls, arrays: Sequence[np.ndarray], sr: int, device="cuda"):
        torch = _torch()
        arrays = [np.ascontiguousarray(np.asarray(a, np.float32).reshape(len(a), -1))
                  for a in arrays]
        ch = arrays[0].shape[1]
        if any(a.shape[1] != ch for a in arrays):
            raise ValueError("all streams of a set must have the same channel count")
        offs, tot = [], 0
        for a in arrays:
            offs.append(tot)
            tot += a.size
        if PINNED_STAGING and tot > 0 and str(device).startswith("cuda"):
            # concatenate straight into page-locked memory, then one DMA copy
            # (57 GB/s vs ~6-7 GB/s for a pageable source, tools/bench_e2e.py)
            stage = torch.empty(tot, dtype=torch.float32, pin_memory=True)
            np.concatenate([a.reshape(-1) for a in arrays], out=stage.numpy())
            x = stage.to(device, non_blocking=True)
            torch.cuda.current_stream().synchronize()  # stage may be reused after return
        else:
            flat = (np.concatenate([a.reshape(-1) for a in arrays]) if arrays
                    else np.zeros(0, np.float32))
            x = torch.from_numpy(flat).to(device)
        return cls(x=x, offs=offs, lens=[a.shape[0] for a in arrays], ch=ch, sr=sr)

    @classmethod
    def synthetic(cls, n_streams: int, n: int, ch: int, sr: int, seed0: int = 1000,
                  device="cuda"):
        """Seeded synthetic streams generated on the device (synth.py twin)."""
        torch = _torch()
        x = torch.empty(n_streams * n * ch, dtype=torch.float32, device=device)
        L = lib()
        hs = stream_handle()
        for i in range(n_streams):
            sub = x[i * n * ch:(i + 1) * n * ch]
            check(L.tomatis_synth_fill(ptr(sub), n, ch, sr, seed0 + i, 0, hs), "synth_fill")
        return cls(x=x, offs=[i * n * ch for i in range(n_streams)], lens=[n] * n_streams,
                   ch=ch, sr=sr)

    @property
    def n_streams(self):
        return len(self.lens)


class Plan:
    """Owns a ``tomatis_plan_t``."""

    def __init__(self, desc: TomatisPlanDesc, window: np.ndarray, streams: List[TomatisStream]):
        L = lib()
        self.L = L
        self.n = len(streams)
        self.streams = (TomatisStream * max(1, self.n))(*streams)
        win = np.ascontiguousarray(window, np.float32)
        self._win = win
        h = C.c_void_p()
        check(L.tomatis_plan_create(C.byref(h), C.byref(desc),
                                    win.ctypes.data_as(C.POINTER(C.c_float)),
                                    self.streams, self.n), "plan_create")
        self.h = h
        self._opts = {}
        self.total_frames = int(L.tomatis_plan_total_frames(h))
        self.total_chunks = int(L.tomatis_plan_total_chunks(h))

    def update(self):
        check(self.L.tomatis_plan_update_streams(self.h, self.streams, stream_handle()),
              "plan_update_streams")

    def check_device(self):
        """Raise if a device-side consistency check fired (synchronises)."""
        check(self.L.tomatis_plan_error(self.h, stream_handle()), "plan_error")

    def error_bits(self, reset: bool = True) -> int:
        """The plan's device error word (TOMATIS_ERR_* bits; synchronises the
        current stream), cleared when ``reset``."""
        b = C.c_uint32(0)
        check(self.L.tomatis_plan_error_bits(self.h, C.byref(b), 1 if reset else 0,
                                             stream_handle()), "plan_error_bits")
        return int(b.value)

    def set_option(self, option: int, value: int):
        check(self.L.tomatis_plan_set_option(self.h, option, int(value)), "plan_set_option")
        self._opts[option] = int(value)

    def option(self, option: int, default: int) -> int:
        """The value this wrapper last set for ``option`` (else ``default``)."""
        return self._opts.get(option, default)

    def set_limiter_spin(self, polls: int):
        """Fused-limiter wait bound (fault injection: 0 forces the recovery path)."""
        self.set_option(OPT_LIMITER_SPIN, polls)

    def close(self):
        if getattr(self, "h", None):
            self.L.tomatis_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceCheckError(RuntimeError):
    """A device-side consistency check fired and the output cannot be trusted."""


def finish_plan(plan: Plan, redo, what: str, redo_gate=None) -> int:
    """Read (and clear) ``plan``'s device error word after a pass; every product
    path calls this before it returns (synchronises the current stream).

    * TOMATIS_ERR_LIMITER_WAIT: a fused-limiter wave gave up waiting for its
      chunk and left its samples unscaled.  ``redo()`` re-launches the pass's
      transform with the limiter as a separate launch (the kernel's outputs and
      peaks are deterministic, so the result equals an undisturbed fused run);
      a warning says so.
    * TOMATIS_ERR_GATE_CARRY: a run of the in-kernel gate (tomatis_stft_ola_gated)
      found no state-fixing frame within its look-back, so the pass is invalid.
      ``redo_gate()`` re-runs the whole pass on the two-pass chain (levels,
      gate, transform), whose own bits are then checked as above.
    * TOMATIS_ERR_PAIR_BARRIER (or any bit after the redo): raise.
    Returns the bits first seen (0 normally)."""
    bits = plan.error_bits(reset=True)
    if bits & ERR_GATE_CARRY:
        if redo_gate is None:
            raise DeviceCheckError(f"{what}: in-kernel gate carry unresolved (bits {bits:#x})")
        redo_gate()
        finish_plan(plan, redo, what)
        return bits
    if bits & ERR_PAIR_BARRIER:
        raise DeviceCheckError(f"{what}: two-wave FFT exchange barrier timed out "
                               f"(device error bits {bits:#x}); the output is invalid")
    if bits & ERR_LIMITER_WAIT:
        if redo is None:
            raise DeviceCheckError(f"{what}: fused limiter wait timed out (bits {bits:#x})")
        warnings.warn(f"{what}: fused limiter wait timed out on the device; "
                      "re-running the transform with the separate limiter launch",
                      RuntimeWarning, stacklevel=3)
        prev = plan.option(OPT_FUSE_LIMITER, 1)  # the caller's setting is restored
        plan.set_option(OPT_FUSE_LIMITER, 0)
        try:
            redo()
        finally:
            plan.set_option(OPT_FUSE_LIMITER, prev)
        again = plan.error_bits(reset=True)
        if again:
            raise DeviceCheckError(f"{what}: device error bits {again:#x} after the unfused re-run")
    elif bits:
        raise DeviceCheckError(f"{what}: unknown device error bits {bits:#x}")
    return bits


_POOL = None


def _host_pool():
    """Threads for per-stream host statistics (the box gives a GPU 16 CPUs)."""
    global _POOL
    if _POOL is None:
        import concurrent.futures as cf
        import os
        n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        _POOL = cf.ThreadPoolExecutor(max_workers=max(1, min(16, n)))
    return _POOL


def _levels_threaded(r: np.ndarray, out: np.ndarray, tmp: np.ndarray = None):
    """``dsp.r_to_level(r)`` into ``out``: the same ufunc chain with in-place
    temporaries (bit-identical: the same loops on the same dtypes; the last
    multiply runs in r's dtype and casts into the float64 ``out`` in its inner
    loop), in slices on the host pool when TOMATIS_LOG10_THREADS > 1 (numpy's
    SIMD log10 does not scale over threads on the measured hosts, so one thread
    by default).  ``tmp``: a reusable buffer of r's dtype (a fresh one per call
    costs its page faults)."""
    n = len(r)
    dt = np.asarray(r).dtype
    if tmp is None or len(tmp) < n or tmp.dtype != dt:
        tmp = np.empty(n, dt)
    k = min(int(os.environ.get("TOMATIS_LOG10_THREADS", "1")), 16, os.cpu_count() or 1)

    def part(a, b):
        np.add(r[a:b], dsp.EPS, out=tmp[a:b])
        np.log10(tmp[a:b], out=tmp[a:b])
        np.multiply(tmp[a:b], 20.0, out=out[a:b], dtype=dt, casting="unsafe")

    if k <= 1 or n < (1 << 16):
        part(0, n)
        return
    edges = np.linspace(0, n, k + 1).astype(np.int64)
    # the slices go to their own executor: callers run on _host_pool() (a stream
    # group's host_levels task), and slices queued behind their own caller on
    # that pool would never start once every worker waits
    list(_slice_pool(k).map(lambda i: part(edges[i], edges[i + 1]), range(k)))


_SLICE_POOL = None
_SLICE_LOCK = threading.Lock()


def _slice_pool(k: int):
    """Workers for the log10 slices of _levels_threaded only (never the pool
    its callers run on): one executor of fixed size (min(16, CPUs)), created
    once under a lock; callers cap their slice count at its size."""
    global _SLICE_POOL
    with _SLICE_LOCK:
        if _SLICE_POOL is None:
            import concurrent.futures as cf
            _SLICE_POOL = cf.ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1)))
    return _SLICE_POOL


def _set_gate(st: TomatisStream, Ton: float, Toff: float):
    on, oe, off, fe = dsp.gate_bits(Ton, Toff)
    st.on_bits, st.off_bits = on, off
    st.n_on_exc, st.n_off_exc = len(oe), len(fe)
    for i, b in enumerate(oe):
        st.on_exc[i] = b
    for i, b in enumerate(fe):
        st.off_exc[i] = b
    st.t_on, st.t_off = Ton, Toff


@dataclass
class Result:
    y: object                       # flat float32 device tensor of all outputs
    out_offs: List[int]
    out_lens: List[int]
    ch: int
    frame_base: List[int]
    n_frames: List[int]
    first_start: List[int]
    hop: int
    states: object = None           # device uint8 per frame
    r: object = None                # device f32 (or f64) per frame
    alpha: object = None            # device f64 per frame
    chunk_peaks: object = None      # device uint32 bits per chunk
    chunk_base: List[int] = field(default_factory=list)
    n_chunks: List[int] = field(default_factory=list)
    extra: dict = field(default_factory=dict)

    def output(self, i: int) -> np.ndarray:
        a = self.out_offs[i]
        n = self.out_lens[i] * self.ch
        src = self.y[a:a + n]
        if PINNED_STAGING and n > 0 and src.is_cuda:
            import torch
            host = torch.empty(n, dtype=torch.float32, pin_memory=True)
            host.copy_(src, non_blocking=True)
            torch.cuda.current_stream().synchronize()
            return host.numpy().reshape(self.out_lens[i], self.ch)  # the view keeps it alive
        return src.cpu().numpy().reshape(self.out_lens[i], self.ch)

    def stream_states(self, i: int) -> np.ndarray:
        a = self.frame_base[i]
        return self.states[a:a + self.n_frames[i]].cpu().numpy()

    def stream_r(self, i: int) -> np.ndarray:
        a = self.frame_base[i]
        return self.r[a:a + self.n_frames[i]].cpu().numpy()

    def stream_alpha(self, i: int) -> np.ndarray:
        a = self.frame_base[i]
        return self.alpha[a:a + self.n_frames[i]].cpu().numpy()

    def stream_peaks(self, i: int) -> np.ndarray:
        a = self.chunk_base[i]
        b = self.chunk_peaks[a:a + self.n_chunks[i]].cpu().numpy().astype(np.uint32)
        return b.view(np.float32)

    def chunk_ranges(self, i: int):
        """Output-index range [lo, hi) of each limiter chunk of stream ``i``."""
        b = self.extra.get("bounds")
        n = self.out_lens[i]
        if not b or b[i] is None or self.n_chunks[i] <= 1:
            return [(0, n)]
        ob = self.extra.get("out_begin", [0] * len(self.out_lens))[i]
        bi = b[i]
        return [(min(n, max(0, int(bi[c]) - ob)), min(n, max(0, int(bi[c + 1]) - ob)))
                for c in range(len(bi) - 1)]

    def scale_flags(self, i: int, limit=None):
        """Per-chunk flags: True where an ill-conditioned sample (tiny window
        sum) may set the limiter scale, so the scale of this build
        and of the reference may differ (conditioning.py).  ``limit``: check a
        scale that is not applied on the device (layer-2 gain protect)."""
        from . import conditioning
        lim = self.extra.get("limit") if limit is None else limit
        if lim is None:
            return [False] * self.n_chunks[i]
        fl = conditioning.result_flags(self, i, n_fft=self.extra["n_fft"],
                                       norm=self.extra.get("norm", "eps"), limit=lim,
                                       chunk_ranges=self.chunk_ranges(i))
        return [f["flagged"] for f in fl]


def _alloc_out(torch, lens, ch, device):
    offs, tot = [], 0
    for n in lens:
        offs.append(tot)
        tot += n * ch
    return torch.empty(max(1, tot), dtype=torch.float32, device=device), offs


MAX_N_FFT = 1 << 16   # tm_shared.h kMaxNfft
MAX_CHANNELS = 128    # tm_shared.h kMaxCh


def _check_fft(n_fft, hop, ch):
    """Shapes the gfx950 library takes: register kernels for n_fft 2048 / 4096
    with <= 2 channels; the any-size path (tm_transform.hip: Stockham FFT,
    Bluestein for n_fft that are not powers of two) for every other n_fft in
    [2, 65536] and up to 128 channels.  The reference's np.fft.rfft/irfft take
    any length (src/process_tomatis.py:396-398); hop outside [1, n_fft] is the
    only shape it cannot run either (a zero hop never advances)."""
    if not (1 <= hop <= n_fft):
        raise ValueError(f"hop={hop} must be in [1, n_fft]")
    if not (2 <= n_fft <= MAX_N_FFT):
        raise ValueError(f"n_fft={n_fft}: the gfx950 kernels take 2 <= n_fft <= {MAX_N_FFT}")
    if not (1 <= ch <= MAX_CHANNELS):
        raise ValueError(f"{ch} channels: the gfx950 kernels handle 1 to {MAX_CHANNELS} channels")


# ---------------------------------------------------------------------------
# standard / xfade
# ---------------------------------------------------------------------------

class GatePipeline:
    """Standard (process_tomatis) or xfade (process_tomatis_xfade) processing."""

    def __init__(self, ss: StreamSet, *, gate_ui=50, gate_mode="log_percent",
                 dynamic_range=80.0, gate_scale=1.0, gate_offset=-100, hysteresis_db=3.0,
                 fc=1000.0, slope=12.0, c1_low=15.0, c1_high=-15.0, c2_low=-15.0,
                 c2_high=15.0, up_delay_ms=250.0, n_fft=4096, hop=2048,
                 output_gain_db=0.0, xfade_ms=None, geometry=None, fused_levels=True,
                 pipelined=False, second_buffer=True):
        """``geometry``: optional per-stream dicts (first_start, n_frames,
        out_begin, out_len, chunk_first, chunk_len, n_chunks) replacing the
        reference schedule -- a time shard of a longer stream (timeshard.py).
        ``fused_levels``: levels and gate states (cross-fade: and alpha) are
        computed inside the transform kernel (tomatis_stft_ola_gated) where the
        library takes the shape (standard 2048 / 256 or 512; standard or
        cross-fade 4096 / 1024); False, or a shape it declines, runs the
        two-pass chain.
        ``pipelined``: successive run() calls form a batch pipeline
        (tomatis_stft_ola_gated_pipelined; the two-pass chain -- xfade, n_fft
        4096 -- through tomatis_stft_ola_pipelined): each pass leaves its output
        unscaled and limits the PREVIOUS pass's output inside its own transform
        (two output buffers, alternating), so the limiter's HBM re-read overlaps
        compute instead of ending every pass.  A pass's output is final after
        the next run() or flush(); result() flushes.  Same results bit for bit.
        Shapes the pipelined calls decline run unpipelined.  The previous pass
        may also be ANOTHER pipeline's (a multi-file job whose batches differ:
        ``run(prev_pipe=...)``, the *_pipelined_after calls).
        ``second_buffer``: allocate the alternate output buffer up front (the
        default) or only when a second pass of this pipeline needs it (one pass
        per pipeline, as batch.py runs them: no idle 1x output of HBM)."""
        torch = _torch()
        _check_fft(n_fft, hop, ss.ch)
        self.ss, self.n_fft, self.hop = ss, n_fft, hop
        sr = ss.sr
        freqs = np.fft.rfftfreq(n_fft, d=1.0 / sr)
        g1_db = dsp.build_tilt_gain_db(freqs, fc, slope, c1_low, c1_high)
        g2_db = dsp.build_tilt_gain_db(freqs, fc, slope, c2_low, c2_high)
        g1, g2 = dsp.db_to_lin(g1_db), dsp.db_to_lin(g2_db)
        xf = 0
        rows = [g1, g2]
        self.xfade = xfade_ms is not None
        if self.xfade:
            frame_ms = hop / sr * 1000.0
            xf = max(1, int(np.ceil(xfade_ms / frame_ms))) if xfade_ms > 0 else 0
            for a in _alpha_lattice(xf):
                rows.append(dsp.db_to_lin((1 - a) * g1_db + a * g2_db))
            T = dsp.gate_ui_to_dbfs(gate_ui, gate_scale, gate_offset)
        elif gate_mode == "log_percent":
            T = dsp.gate_ui_to_dbfs_log_percent(gate_ui, dynamic_range)
        else:
            T = dsp.gate_ui_to_dbfs(gate_ui, gate_scale, gate_offset)
        self.T = T
        self.Ton, self.Toff = T + hysteresis_db / 2.0, T - hysteresis_db / 2.0
        D = int(sr * up_delay_ms / 1000.0)
        self.up_delay_samples = D
        Dk = max(0, -(-D // hop))
        self.up_delay_frames = Dk
        self.xf = xf
        out_scale = np.float32(10.0 ** (output_gain_db / 20.0)) if (
            output_gain_db != 0.0 and not self.xfade) else np.float32(1.0)
        streams = []
        self.bounds = []
        for i, (off, N) in enumerate(zip(ss.offs, ss.lens)):
            st = TomatisStream()
            if geometry is not None:
                g = geometry[i]
                st.in_off, st.n = off, N
                st.first_start, st.n_frames = g["first_start"], g["n_frames"]
                st.out_begin, st.out_len = g["out_begin"], g["out_len"]
                st.n_chunks, st.chunk_first, st.chunk_len = (g["n_chunks"], g["chunk_first"],
                                                             g["chunk_len"])
                self.bounds.append(g.get("bounds"))
            else:
                pad, pe, F, s0 = dsp.std_schedule(N, n_fft, hop)
                b = dsp.std_flush_bounds(N, n_fft, hop)
                self.bounds.append(b)
                st.in_off, st.n, st.first_start, st.n_frames = off, N, s0, F
                st.out_begin, st.out_len = 0, (N if F else 0)
                nch = max(1, len(b) - 1)
                st.n_chunks = nch
                st.chunk_first = b[1] if len(b) > 2 else 0
                st.chunk_len = ((b[2] - b[1]) if len(b) > 3 else
                                max(1, (b[-1] - b[1]) if len(b) > 2 else 1))
            st.in_scale, st.out_scale = 1.0, float(out_scale)
            _set_gate(st, self.Ton, self.Toff)
            streams.append(st)
        self.y, out_offs = _alloc_out(torch, [s.out_len for s in streams], ss.ch, ss.x.device)
        for st, o in zip(streams, out_offs):
            st.out_off = o
        desc = TomatisPlanDesc(n_fft=n_fft, hop=hop, ch=ss.ch, norm_mode=NORM_EPS,
                               up_delay_frames=Dk, min_hold_frames=0, xfade_frames=xf,
                               alpha_mode=1 if self.xfade else 0)
        self.plan = Plan(desc, dsp.hann(n_fft), streams)
        self.streams = list(self.plan.streams)[:len(streams)]
        Ft = max(1, self.plan.total_frames)
        dev = ss.x.device
        self.r = torch.empty(Ft, dtype=torch.float32, device=dev)
        self.states = torch.empty(Ft, dtype=torch.uint8, device=dev)
        self.rows = torch.empty(Ft + 1, dtype=torch.int16, device=dev)  # +1: read as u32 words
        self.alpha = torch.empty(Ft, dtype=torch.float64, device=dev) if self.xfade else None
        self.peaks = torch.zeros(max(1, self.plan.total_chunks), dtype=torch.int32, device=dev)
        self.gains = torch.from_numpy(np.stack(rows).astype(np.float32)).to(dev)
        self.n_rows = len(rows)
        self.out_offs = out_offs
        self.g1_db, self.g2_db = g1_db, g2_db
        self.fused_levels = bool(fused_levels)
        if self.xfade:  # the gated calls' per-frame alpha (cross-fade plans)
            check(lib().tomatis_plan_set_gate_alpha(self.plan.h, ptr(self.alpha)), "set_gate_alpha")
        self.gated_used = False   # the last run() took tomatis_stft_ola_gated
        self.gate_fallbacks = 0   # gated passes re-run on the two-pass chain
        self.pipelined = bool(pipelined)
        self.pending = False      # pipelined: self.y awaits its limiter
        self._after = None        # run(prev_pipe=...): another pipeline's pending pass
        if self.pipelined:
            self._ys = [self.y, torch.empty_like(self.y) if second_buffer else None]
            self._pks = [self.peaks, torch.zeros_like(self.peaks) if second_buffer else None]
            self._cur = 0

    def run(self, marks=None, check_device: bool = True, prev_pipe=None):
        """Launch the whole chain on the current stream.

        ``marks``: optional pair of torch.cuda.Event recorded on this stream
        around the fused STFT-OLA launch (bench.py's live kernel timing).
        ``check_device``: read the plan's device error word before returning
        (one host synchronisation; ``finish_plan``).  Only a caller that checks
        once after many passes (bench.py's timed loop) turns it off.
        ``prev_pipe``: another pipeline (same n_fft / hop / channels) whose last
        pass is pending: this pass limits it inside its transform (pipelined
        mode), or it is flushed here; either way its output is final once this
        pass's work on the stream has completed."""
        if prev_pipe is not None and prev_pipe.pending and self.pending:
            self.flush()          # one predecessor per pass: ours is limited now
        self._after = prev_pipe if (prev_pipe is not None and prev_pipe.pending) else None
        try:
            if self.fused_levels:
                self.gated_used = self._gated(marks)
                if self.gated_used:
                    if marks:
                        marks[1].record()
                    self._flush_after()
                    if check_device:
                        self.finish()
                    # pipelined: the output is final after the next pass or flush()
                    return None if self.pending else self.result()
                self.fused_levels = False  # declined: this plan's shape runs two passes
            self._two_pass(marks)
            self._flush_after()
        finally:
            self._after = None
        if check_device:
            self.finish()
        return None if self.pending else self.result()

    def _prev(self):
        """(plan, y, peaks) of the output this pass limits: another
        pipeline's pending pass (run(prev_pipe=...)), this pipeline's own, or
        none."""
        a = self._after
        if a is not None and a.pending:
            return a.plan, a.y, a.peaks
        if self.pending:
            return self.plan, self._ys[self._cur], self._pks[self._cur]
        return None, None, None

    def _out_slot(self) -> int:
        """The output buffer of a pipelined pass: the other one while this
        pipeline's own previous pass is pending, else the current one."""
        nxt = (1 - self._cur) if self.pending else self._cur
        if self._ys[nxt] is None:   # second_buffer=False: allocated on first need
            self._ys[nxt] = _torch().empty_like(self._ys[self._cur])
            self._pks[nxt] = _torch().zeros_like(self._pks[self._cur])
        return nxt

    def _took_prev(self, nxt: int):
        """Bookkeeping after a pipelined launch into buffer ``nxt``."""
        if self._after is not None:
            self._after.pending = False   # limited inside that launch
        self._cur = nxt
        self.y, self.peaks = self._ys[nxt], self._pks[nxt]
        self.pending = True

    def _flush_after(self):
        a = self._after
        if a is not None and a.pending:
            a.flush()

    def _gated(self, marks=None) -> bool:
        """levels + gate + transform + limiter in one pass over the input (the
        look-back pre-kernel, then the transform); False when the library
        declines this plan's shape (nothing launched).  ``marks`` bracket the
        transform launch."""
        L, hs = lib(), stream_handle()
        rc = L.tomatis_gate_lookback(self.plan.h, ptr(self.ss.x), hs)
        if rc == E_UNSUPPORTED:
            return False
        check(rc, "gate_lookback")
        if self.pipelined and self._pipelined_pass(marks):
            return True
        self.flush()
        self.peaks.zero_()
        if marks:
            marks[0].record()
        check(L.tomatis_stft_ola_gated_after_lookback(
            self.plan.h, ptr(self.ss.x), ptr(self.gains), self.n_rows, ptr(self.y),
            ptr(self.peaks), PEAK_LIMIT, ptr(self.r), ptr(self.states), hs), "stft_ola_gated")
        return True

    def _pipelined_pass(self, marks=None) -> bool:
        """One pipelined pass, limiting the pending output (this pipeline's
        previous pass, or run(prev_pipe=...)'s) inside the launch; False (nothing
        launched) when the library declines the shape (then pipelining stays
        off)."""
        L, hs = lib(), stream_handle()
        nxt = self._out_slot()
        pplan, prev_y, prev_pk = self._prev()
        if marks:  # (the call zeroes this pass's chunk peaks itself)
            marks[0].record()
        rc = L.tomatis_stft_ola_gated_pipelined_after(
            self.plan.h, ptr(self.ss.x), ptr(self.gains), self.n_rows, ptr(self._ys[nxt]),
            ptr(self._pks[nxt]), PEAK_LIMIT, ptr(self.r), ptr(self.states),
            pplan.h if pplan is not None else None, ptr(prev_y), ptr(prev_pk), hs)
        if rc == E_UNSUPPORTED and self._drop_foreign_prev(pplan):
            return self._pipelined_pass(marks)  # (marks[0] recorded again: same point)
        if rc == E_UNSUPPORTED:
            self.pipelined = False
            return False
        check(rc, "stft_ola_gated_pipelined")
        self._took_prev(nxt)
        return True

    def flush(self):
        """Pipelined: apply the limiter to the last pass's output (it has no
        next pass to do it); no-op otherwise."""
        if self.pending:
            check(lib().tomatis_apply_limiter(self.plan.h, ptr(self.y), ptr(self.peaks),
                                              PEAK_LIMIT, stream_handle()), "apply_limiter")
            self.pending = False

    def _two_pass(self, marks=None, pipelined=True):
        L, P, hs = lib(), self.plan.h, stream_handle()
        check(L.tomatis_levels(P, ptr(self.ss.x), ptr(self.r), F32, hs), "levels")
        check(L.tomatis_gate_std(P, ptr(self.r), ptr(self.states), ptr(self.rows),
                                 ptr(self.alpha), hs), "gate_std")
        if marks:
            marks[0].record()
        if not (pipelined and self.pipelined and self._rows_pipelined_pass()):
            self.flush()
            self._limited()
        if marks:
            marks[1].record()

    def _rows_pipelined_pass(self) -> bool:
        """The two-pass chain's transform as a pipelined pass (gain-row ids from
        tomatis_gate_std); False (nothing launched) when the library declines."""
        nxt = self._out_slot()
        pplan, prev_y, prev_pk = self._prev()
        rc = lib().tomatis_stft_ola_pipelined_after(  # (zeroes this pass's chunk peaks)
            self.plan.h, ptr(self.ss.x), ptr(self.gains), self.n_rows, ptr(self.rows),
            ptr(self._ys[nxt]), ptr(self._pks[nxt]), PEAK_LIMIT,
            pplan.h if pplan is not None else None, ptr(prev_y), ptr(prev_pk), stream_handle())
        if rc == E_UNSUPPORTED and self._drop_foreign_prev(pplan):
            return self._rows_pipelined_pass()
        if rc == E_UNSUPPORTED:
            self.pipelined = False
            return False
        check(rc, "stft_ola_pipelined")
        self._took_prev(nxt)
        return True

    def _drop_foreign_prev(self, pplan) -> bool:
        """A pipelined call declined another pipeline's pending pass (a plan of
        another n_fft / hop / channel count): flush that one on its own plan and
        let the caller retry with nothing to limit.  False when the decline is
        this plan's own shape."""
        a = self._after
        if a is None or pplan is None or pplan is self.plan:
            return False
        a.flush()
        self._after = None
        return True

    def _limited(self):
        """transform + OLA + per-chunk limiter (fused in-kernel when chunks are short)"""
        self.peaks.zero_()
        check(lib().tomatis_stft_ola_limited(self.plan.h, ptr(self.ss.x), ptr(self.gains),
                                             self.n_rows, ptr(self.rows), ptr(self.y),
                                             ptr(self.peaks), PEAK_LIMIT, stream_handle()),
              "stft_ola_limited")

    def finish(self) -> int:
        """Device checks of the last run() (finish_plan); an unresolved in-kernel
        gate carry re-runs the pass on the two-pass chain (same results)."""
        if self.gated_used:
            def redo_gate():
                # (a pipelined launch limited the previous output whatever its
                # own gate did; this pass is recomputed, limited, into self.y)
                self.gated_used = False
                self.gate_fallbacks += 1
                self.pending = False
                self._two_pass(pipelined=False)
            # a limiter-wait redo of the gated pass: the transform alone cannot
            # recompute states, so the two-pass chain runs with the unfused limiter
            return finish_plan(self.plan, redo_gate, "GatePipeline", redo_gate=redo_gate)

        def redo():  # (unpipelined, into the same buffer)
            self.pending = False
            self._limited()
        return finish_plan(self.plan, redo, "GatePipeline")

    def result(self) -> Result:
        self.flush()
        st = self.streams
        return Result(y=self.y, out_offs=self.out_offs, out_lens=[s.out_len for s in st],
                      ch=self.ss.ch, frame_base=[s.frame_base for s in st],
                      n_frames=[s.n_frames for s in st],
                      first_start=[s.first_start for s in st], hop=self.hop,
                      states=self.states, r=self.r, alpha=self.alpha,
                      chunk_peaks=self.peaks, chunk_base=[s.chunk_base for s in st],
                      n_chunks=[s.n_chunks for s in st],
                      extra=dict(Ton=self.Ton, Toff=self.Toff, T=self.T, xfade_frames=self.xf,
                                 up_delay_samples=self.up_delay_samples, bounds=self.bounds,
                                 n_fft=self.n_fft, norm="eps", limit=PEAK_LIMIT,
                                 limiter_applied=True, out_begin=[s.out_begin for s in st]))


def _alpha_lattice(xf: int):
    """alpha values m*step reached by repeated +step from 0 (reference accumulation),
    with the snapped end points 0.0 and 1.0 exact.  Rows 2+m of the gain table."""
    if xf <= 0:
        return [0.0, 1.0]
    step = 1.0 / xf
    out, a = [0.0], 0.0
    for _ in range(1, xf):
        a = a + step
        out.append(a)
    out.append(1.0)
    return [np.float64(v) for v in out]


# ---------------------------------------------------------------------------
# adaptive
# ---------------------------------------------------------------------------

class AdaptivePipeline:
    """process_tomatis_adaptive: attenuation, levels, bisection, min-hold gate,
    alpha cross-fade, mixed gains, OLA, restore, global limiter."""

    def __init__(self, ss: StreamSet, *, fc=1000.0, slope=12.0, c1_low=15.0, c1_high=-15.0,
                 c2_low=-15.0, c2_high=15.0, target_c2=0.5, hyst_db=3.0, min_hold_ms=250.0,
                 xfade_ms=500.0, headroom_margin=2.0, n_fft=4096, hop=2048, out=None,
                 pipelined=False, out2=None, second_buffer=True):
        """``out``: optional (y, offsets) output buffer shared with other
        pipelines (AdaptiveGroups).  ``pipelined``: a batch pipeline as
        GatePipeline's (tomatis_stft_ola_pipelined: each pass's transform
        applies the previous pass's global limiter; ``out2`` the second output
        buffer, same offsets, when ``out`` is shared; ``second_buffer=False``:
        none until a second pass of this pipeline needs it)."""
        torch = _torch()
        _check_fft(n_fft, hop, ss.ch)
        self.ss, self.n_fft, self.hop = ss, n_fft, hop
        sr = ss.sr
        frame_ms = hop / sr * 1000
        self.mh = int(np.ceil(min_hold_ms / frame_ms))
        self.xf = int(np.ceil(xfade_ms / frame_ms))
        self.target_c2, self.hyst_db = target_c2, hyst_db
        self.max_gain = max(abs(c1_low), abs(c2_high))
        self.margin = headroom_margin
        freqs = np.fft.rfftfreq(n_fft, 1 / sr)
        c1_db = dsp.build_tilt_gain_db(freqs, fc, slope, c1_low, c1_high)
        c2_db = dsp.build_tilt_gain_db(freqs, fc, slope, c2_low, c2_high)
        xfe = self.xf if self.xf > 0 else 1
        rows = [np.zeros(len(freqs), np.float32)] * 2  # rows 0/1 unused in adaptive mode
        for a in _alpha_lattice(xfe):
            rows.append((10 ** (np.asarray((1 - a) * c1_db + a * c2_db) / 20.0)).astype(np.float32))
        streams = []
        for off, N in zip(ss.offs, ss.lens):
            k0, F, s0 = dsp.adaptive_frames(N, n_fft, hop)
            st = TomatisStream()
            st.in_off, st.n, st.first_start, st.n_frames = off, N, s0, F
            # (a stream with no frame -- shorter than n_fft / 2 -- has no output
            # in the plan; its result is N zeros, below)
            st.out_begin, st.out_len = 0, (N if F else 0)
            st.n_chunks, st.chunk_first, st.chunk_len = 1, 0, 1
            st.in_scale, st.out_scale = 1.0, 1.0
            streams.append(st)
        # output slices of N samples for every stream: one with no frame
        # writes N zeros (process_tomatis_adaptive.py:289-334: y = zeros_like,
        # no frame adds to it, then / max(norm, 1e-8))
        self.res_lens = list(ss.lens)
        if out is None:
            self.y, out_offs = _alloc_out(torch, self.res_lens, ss.ch, ss.x.device)
        else:
            self.y, out_offs = out[0], list(out[1])
        for st, o in zip(streams, out_offs):
            st.out_off = o
        desc = TomatisPlanDesc(n_fft=n_fft, hop=hop, ch=ss.ch, norm_mode=NORM_MAX,
                               up_delay_frames=0, min_hold_frames=self.mh,
                               xfade_frames=self.xf, alpha_mode=2)
        self.plan = Plan(desc, dsp.hann(n_fft), streams)
        Ft = max(1, self.plan.total_frames)
        dev = ss.x.device
        self.r32 = torch.empty(Ft, dtype=torch.float32, device=dev)
        self.r64 = torch.empty(Ft, dtype=torch.float64, device=dev)
        self.levels = torch.empty(Ft, dtype=torch.float64, device=dev)
        self.states = torch.empty(Ft, dtype=torch.uint8, device=dev)
        self.rows = torch.empty(Ft + 1, dtype=torch.int16, device=dev)  # +1: read as u32 words
        self.alpha = torch.empty(Ft, dtype=torch.float64, device=dev)
        self.t_out = torch.empty(max(1, ss.n_streams), dtype=torch.float64, device=dev)
        self.peaks = torch.zeros(max(1, self.plan.total_chunks), dtype=torch.int32, device=dev)
        self.inpk = torch.zeros(max(1, ss.n_streams), dtype=torch.int32, device=dev)
        self._lv_pin = None   # page-locked staging of r and the host levels (allocated once)
        self._lv_tmp = None   # host temporaries of the level chain (allocated once)
        self._pk_pin = torch.empty(max(1, ss.n_streams), dtype=torch.int32, pin_memory=True)
        self.stream = None    # torch stream the pipeline runs on (None: the current one)
        self.done = torch.cuda.Event()
        self.prep_done = torch.cuda.Event()  # after the bisection / states launch
        self._tlh = torch.empty(3 * max(1, ss.n_streams), dtype=torch.float64, device=dev)
        self.gains = torch.from_numpy(np.stack(rows)).to(dev)
        self.n_rows = len(rows)
        self.out_offs = out_offs
        # output slices no kernel writes (streams without frames): zeroed in
        # every output buffer this pipeline gets
        self._idle = [(o, N * ss.ch) for o, N, st in zip(out_offs, self.res_lens, streams)
                      if st.n_frames == 0 and N > 0]
        self._clear_idle(self.y)
        self.pipelined = bool(pipelined)
        self.pending = False      # pipelined: self.y awaits its limiter
        self._after = None        # run(prev_pipe=...): another pipeline's pending pass
        if self.pipelined:
            self._ys = [self.y, out2 if out2 is not None else
                        (torch.empty_like(self.y) if second_buffer else None)]
            self._clear_idle(self._ys[1])
            self._pks = [self.peaks, torch.zeros_like(self.peaks)]
            self._cur = 0

    def _clear_idle(self, buf):
        if buf is not None:
            for o, n in self._idle:
                buf[o:o + n].zero_()

    def run(self, marks=None, timer=None, check_device: bool = True, prev_pipe=None):
        """``timer`` (a dict) collects synchronised wall-clock phases (profiling).
        ``check_device``, ``prev_pipe``: as GatePipeline.run."""
        for _ in self.steps(marks, timer, prev_pipe=prev_pipe):
            pass
        if check_device:
            self.finish()
        return None if self.pending else self.result()

    def _transform(self):
        """STFT-gain-OLA, normalise max(w,1e-8), restore, global limiter (one
        chunk per stream: fused into the transform when its runs allow;
        pipelined: the previous pass's limiter inside this transform)"""
        a = self._after
        if a is not None and a.pending and self.pending:
            self.flush()          # one predecessor per pass
        try:
            if self.pipelined and self._pipelined_pass():
                return
            self.flush()
            self._limited()
        finally:
            if a is not None and a.pending:
                a.flush()
            self._after = None

    def _limited(self):
        self.peaks.zero_()
        check(lib().tomatis_stft_ola_limited(self.plan.h, ptr(self.ss.x), ptr(self.gains),
                                             self.n_rows, ptr(self.rows), ptr(self.y),
                                             ptr(self.peaks), PEAK_LIMIT, stream_handle()),
              "stft_ola_limited")

    def _pipelined_pass(self) -> bool:
        a = self._after
        # the other buffer while this pipeline's own previous pass is pending,
        # else the current one (AdaptiveGroups: every group alternates in step)
        nxt = (1 - self._cur) if self.pending else self._cur
        if self._ys[nxt] is None:  # second_buffer=False, standalone: allocated on first need
            self._ys[nxt] = _torch().empty_like(self._ys[self._cur])
            self._clear_idle(self._ys[nxt])
        if a is not None and a.pending:
            pplan, prev_y, prev_pk = a.plan, a.y, a.peaks
        elif self.pending:
            pplan, prev_y, prev_pk = self.plan, self._ys[self._cur], self._pks[self._cur]
        else:
            pplan, prev_y, prev_pk = None, None, None
        rc = lib().tomatis_stft_ola_pipelined_after(  # (zeroes this pass's chunk peaks)
            self.plan.h, ptr(self.ss.x), ptr(self.gains), self.n_rows, ptr(self.rows),
            ptr(self._ys[nxt]), ptr(self._pks[nxt]), PEAK_LIMIT,
            pplan.h if pplan is not None else None, ptr(prev_y), ptr(prev_pk), stream_handle())
        if rc == E_UNSUPPORTED and a is not None and pplan is a.plan:
            a.flush()             # another shape: limited on its own plan, then retry
            self._after = None
            return self._pipelined_pass()
        if rc == E_UNSUPPORTED:
            self.pipelined = False
            return False
        check(rc, "stft_ola_pipelined")
        if a is not None:
            a.pending = False     # limited inside this launch
        self._cur = nxt
        self.y, self.peaks = self._ys[nxt], self._pks[nxt]
        self.pending = True
        return True

    def flush(self):
        """Pipelined: the last pass's global limiter (on the pipeline's stream)."""
        if self.pending:
            torch = _torch()
            with torch.cuda.stream(self.stream or torch.cuda.current_stream()):
                check(lib().tomatis_apply_limiter(self.plan.h, ptr(self.y), ptr(self.peaks),
                                                  PEAK_LIMIT, stream_handle()), "apply_limiter")
            self.pending = False

    def finish(self) -> int:
        """Device error check after the pass (on the pipeline's stream); a
        limiter-wait redo runs the transform unpipelined into the same buffer."""
        torch = _torch()

        def redo():
            self.pending = False
            self._limited()
        with torch.cuda.stream(self.stream or torch.cuda.current_stream()):
            return finish_plan(self.plan, redo, "AdaptivePipeline")

    def steps(self, marks=None, timer=None, after=None, prev_pipe=None):
        """The pass as a generator that yields wherever the host would wait for
        the device (the input peaks, the frame r) and before the transform, so a
        driver can interleave several pipelines on their own streams
        (AdaptiveGroups).  ``after``: a callable giving an event (or a list of
        events) the transform waits for.  ``prev_pipe``: as GatePipeline.run
        (the caller orders that pipeline's stream before this one's)."""
        torch = _torch()
        strm = self.stream or torch.cuda.current_stream()
        L, P = lib(), self.plan.h
        ss = self.ss
        sts = self.plan.streams
        t0 = [time.perf_counter()]
        ev = torch.cuda.Event()

        def phase(name):
            if timer is not None:
                torch.cuda.synchronize()
                t = time.perf_counter()
                timer[name] = timer.get(name, 0.0) + t - t0[0]
                t0[0] = t

        # 1. input peak per stream -> attenuation (process_tomatis_adaptive.py:201-215)
        with torch.cuda.stream(strm):
            hs = stream_handle()
            self.inpk.zero_()
            check(L.tomatis_absmax_streams(P, ptr(ss.x), ptr(self.inpk), hs), "absmax_streams")
            self._pk_pin.copy_(self.inpk, non_blocking=True)
            ev.record()
        yield
        ev.synchronize()
        pk = self._pk_pin.numpy().astype(np.uint32).view(np.float32)
        self.atten, prec = [], []
        for i in range(ss.n_streams):
            peak_db = 20 * np.log10(pk[i] + dsp.EPS)
            atten_db = max(0, peak_db + self.max_gain + self.margin)
            self.atten.append(atten_db)
            if atten_db > 0:   # float32 pipeline (NEP 50)
                sts[i].in_scale = float(10 ** (np.asarray(-atten_db) / 20.0))
                sts[i].out_scale = float(10 ** (np.asarray(atten_db) / 20.0))
                prec.append(F32)
            else:              # float64 pipeline: x * 1.0
                sts[i].in_scale, sts[i].out_scale = 1.0, 1.0
                prec.append(F64)
        Ft = self.plan.total_frames
        if self._lv_pin is None:
            self._lv_pin = torch.empty(max(1, Ft), dtype=torch.float64, pin_memory=True)
            self._lv32_pin = torch.empty(max(1, Ft), dtype=torch.float32, pin_memory=True)
            self._lv32_dev = torch.empty(max(1, Ft), dtype=torch.float32, device=ss.x.device)
            self._r_pin = {F32: torch.empty(max(1, Ft), dtype=torch.float32, pin_memory=True),
                           F64: torch.empty(max(1, Ft), dtype=torch.float64, pin_memory=True)}
        with torch.cuda.stream(strm):
            hs = stream_handle()
            self.plan.update()
            phase("peak+atten")
            # 2. per-frame levels (f32 and/or f64 r) -> page-locked host blocks
            if F32 in prec:
                check(L.tomatis_levels(P, ptr(ss.x), ptr(self.r32), F32, hs), "levels f32")
            if F64 in prec:
                check(L.tomatis_levels(P, ptr(ss.x), ptr(self.r64), F64, hs), "levels f64")
            phase("levels_kernel")
            for pr, rd in ((F32, self.r32), (F64, self.r64)):
                if pr in prec:
                    self._r_pin[pr][:Ft].copy_(rd[:Ft], non_blocking=True)
            ev.record()
        yield
        # levels of every frame by the same elementwise numpy call as the
        # reference's per-frame one, written into a page-locked upload block (on
        # a host thread, so several stream groups' chains overlap); per-stream
        # order statistics (p5, p95, median of the valid levels) then on the
        # device
        if self._lv_tmp is None:
            self._lv_tmp = {F32: np.empty(max(1, Ft), np.float32),
                            F64: np.empty(max(1, Ft), np.float64)}

        def host_levels():
            ev.synchronize()
            rs = {pr: self._r_pin[pr].numpy()[:Ft] for pr in (F32, F64) if pr in prec}
            if set(rs) == {F32}:
                # float32 levels (their float64 values are exact): the last
                # multiply stays in float32, the device widens them
                tmp = self._lv_tmp[F32][:Ft]
                np.add(rs[F32], dsp.EPS, out=tmp)
                np.log10(tmp, out=tmp)
                np.multiply(tmp, 20.0, out=self._lv32_pin.numpy()[:Ft])
                return F32
            lv = self._lv_pin.numpy()[:Ft]
            if len(rs) == 1:
                _levels_threaded(rs[F64], lv, self._lv_tmp[F64])
            else:
                lv32 = np.empty(Ft, np.float64)
                lv64 = np.empty(Ft, np.float64)
                _levels_threaded(rs[F32], lv32, self._lv_tmp[F32])
                _levels_threaded(rs[F64], lv64, self._lv_tmp[F64])
                for i in range(ss.n_streams):
                    a, F = sts[i].frame_base, sts[i].n_frames
                    lv[a:a + F] = (lv32 if prec[i] == F32 else lv64)[a:a + F]
            return F64

        fut = _host_pool().submit(host_levels)
        yield
        up = fut.result()
        phase("r_d2h+log10")
        with torch.cuda.stream(strm):
            hs = stream_handle()
            if up == F32:
                self._lv32_dev[:Ft].copy_(self._lv32_pin[:Ft], non_blocking=True)
                self.levels[:Ft].copy_(self._lv32_dev[:Ft])
            else:
                self.levels[:Ft].copy_(self._lv_pin[:Ft], non_blocking=True)
            tl = self._tlh
            check(L.tomatis_level_stats(P, ptr(self.levels), ptr(tl), hs), "level_stats")
            phase("upload+stats")
            # 3. bisection + min-hold states + alpha + rows
            check(L.tomatis_minhold_bisect(P, ptr(self.levels), ptr(tl), self.target_c2,
                                           self.hyst_db, ptr(self.t_out), ptr(self.states),
                                           ptr(self.rows), ptr(self.alpha), hs), "minhold_bisect")
            phase("bisect+minhold")
            self.prep_done.record()
        yield   # (a driver launches every group's statistics before the transforms)
        with torch.cuda.stream(strm):
            hs = stream_handle()
            # 4. STFT-gain-OLA, normalise, restore, global limiter
            if after is not None:
                evs = after()
                for e in (evs if isinstance(evs, (list, tuple)) else [evs]):
                    if e is not None:
                        strm.wait_event(e)
            if marks and marks[0] is not None:
                marks[0].record()
            self._after = prev_pipe if (prev_pipe is not None and prev_pipe.pending) else None
            self._transform()
            if marks and marks[1] is not None:
                marks[1].record()
            self.done.record()
            phase("transform+limiter")
        self.prec = prec

    def result(self) -> Result:
        self.flush()
        st = list(self.plan.streams)[:self.ss.n_streams]
        return Result(y=self.y, out_offs=self.out_offs, out_lens=list(self.res_lens),
                      ch=self.ss.ch, frame_base=[s.frame_base for s in st],
                      n_frames=[s.n_frames for s in st],
                      first_start=[s.first_start for s in st], hop=self.hop,
                      states=self.states, r=self.r32, alpha=self.alpha,
                      chunk_peaks=self.peaks, chunk_base=[s.chunk_base for s in st],
                      n_chunks=[s.n_chunks for s in st],
                      extra=dict(levels=self.levels, thresholds=self.t_out,
                                 atten_db=getattr(self, "atten", None),
                                 min_hold_frames=self.mh, xfade_frames=self.xf,
                                 prec=getattr(self, "prec", None), n_fft=self.n_fft,
                                 norm="max", limit=PEAK_LIMIT, limiter_applied=True,
                                 out_begin=[s.out_begin for s in st]))


def merge_results(results: Sequence[Result]) -> Result:
    """One Result over several pipelines' streams (same output buffer y; per-frame
    and per-chunk arrays concatenated, indices re-based)."""
    torch = _torch()
    r0 = results[0]
    if any(r.y.data_ptr() != r0.y.data_ptr() for r in results):
        raise ValueError("merge_results: pipelines must share one output buffer")
    fb, cb, ftot, ctot = [], [], 0, 0
    for r in results:
        fb += [ftot + v for v in r.frame_base]
        cb += [ctot + v for v in r.chunk_base]
        ftot += int(sum(r.n_frames))
        ctot += int(sum(r.n_chunks))

    def cat(get, n_of):
        parts = [get(r)[:n_of(r)] for r in results]
        return torch.cat(parts) if parts else None

    nf = lambda r: int(sum(r.n_frames))  # noqa: E731
    nc = lambda r: int(sum(r.n_chunks))  # noqa: E731
    ns = lambda r: len(r.out_lens)       # noqa: E731
    ex = dict(r0.extra)
    ex["levels"] = cat(lambda r: r.extra["levels"], nf)
    ex["thresholds"] = cat(lambda r: r.extra["thresholds"], ns)
    for k in ("atten_db", "prec", "out_begin"):
        ex[k] = [v for r in results for v in (r.extra.get(k) or [])]
    return Result(y=r0.y, out_offs=[o for r in results for o in r.out_offs],
                  out_lens=[o for r in results for o in r.out_lens], ch=r0.ch,
                  frame_base=fb, n_frames=[v for r in results for v in r.n_frames],
                  first_start=[v for r in results for v in r.first_start], hop=r0.hop,
                  states=cat(lambda r: r.states, nf), r=cat(lambda r: r.r, nf),
                  alpha=cat(lambda r: r.alpha, nf), chunk_peaks=cat(lambda r: r.chunk_peaks, nc),
                  chunk_base=cb, n_chunks=[v for r in results for v in r.n_chunks], extra=ex)


class AdaptiveGroups:
    """An adaptive batch (config C3) as G stream groups, each with its own plan
    and HIP stream, interleaved so the host phase of one group (peak ->
    attenuation, numpy log10 of its frame r) overlaps the device work of the
    others; the transforms launch in group order (each waits for the previous
    one: a fused-limiter launch never shares the dispatcher with another).
    Output in one buffer; ``result()`` merges the groups."""

    def __init__(self, ss: StreamSet, groups: int = 2, pipelined=False, second_buffer=True,
                 **params):
        """``pipelined``: every group pipelines its passes (AdaptivePipeline);
        the groups alternate between two shared output buffers in step
        (``second_buffer=False``: the second one allocated when a second pass
        needs it -- batch.py's single-pass batches never do)."""
        torch = _torch()
        n_fft, hop = params.get("n_fft", 4096), params.get("hop", 2048)
        G = max(1, min(int(groups), ss.n_streams))
        out_lens = list(ss.lens)  # (streams without frames: N zeros, AdaptivePipeline)
        self.y, offs = _alloc_out(torch, out_lens, ss.ch, ss.x.device)
        y2 = torch.empty_like(self.y) if (pipelined and second_buffer) else None
        # contiguous groups balanced by samples
        tot, acc, cuts = float(sum(ss.lens)) or 1.0, 0, [0]
        for i, N in enumerate(ss.lens):
            acc += N
            if len(cuts) < G and acc >= tot * len(cuts) / G and i + 1 < ss.n_streams:
                cuts.append(i + 1)
        cuts.append(ss.n_streams)
        self.pipes = []
        # bisection: speculative over the chip while no transform runs; with
        # TOMATIS_C3_SYNC=chain later groups' overlap the previous transform and
        # take one CU per stream (TOMATIS_MH_MODE=spec / serial: all groups)
        mh_mode = os.environ.get("TOMATIS_MH_MODE", "auto")
        chain = os.environ.get("TOMATIS_C3_SYNC", "first") == "chain"
        for g, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
            sub = StreamSet(x=ss.x, offs=ss.offs[a:b], lens=ss.lens[a:b], ch=ss.ch, sr=ss.sr)
            p = AdaptivePipeline(sub, out=(self.y, offs[a:b]), pipelined=pipelined, out2=y2,
                                 second_buffer=False, **params)
            p.stream = torch.cuda.Stream()
            serial = mh_mode == "serial" or (mh_mode == "auto" and chain and g > 0)
            p.plan.set_option(OPT_MINHOLD_SERIAL, int(serial))
            self.pipes.append(p)
        self.ss = ss

    def run(self, marks=None, check_device: bool = True, prev_pipe=None):
        """``prev_pipe``: another AdaptiveGroups (or AdaptivePipeline) whose
        last pass is pending: group g limits its group g inside its transform
        (groups it does not have are flushed)."""
        torch = _torch()
        cur = torch.cuda.current_stream()
        prevs = []
        if prev_pipe is not None:
            prevs = list(getattr(prev_pipe, "pipes", [prev_pipe]))
            for q in prevs[len(self.pipes):]:
                q.flush()
            for q in prevs:   # (their last transforms are ordered before cur)
                cur.wait_stream(q.stream or cur)
        for p in self.pipes:
            p.stream.wait_stream(cur)
            if p.pipelined and p.pending and p._ys[1 - p._cur] is None:
                # the groups' shared second buffer, on the first pass that needs it
                y2 = torch.empty_like(self.pipes[0]._ys[0])
                for q in self.pipes:
                    q._ys[1] = y2
                    q._clear_idle(y2)
        G = len(self.pipes)
        gens = []
        # transforms in group order; the first also waits for every group's
        # statistics: a later group's small bisection / states kernels launched
        # behind a running transform would wait for its workgroups to drain
        # (measured: 5.8 ms for a 0.35 ms kernel) and delay the next transform
        # (TOMATIS_C3_SYNC=chain: only the previous transform)
        first_all = os.environ.get("TOMATIS_C3_SYNC", "first") != "chain"
        for g, p in enumerate(self.pipes):
            mk = None
            if marks:
                mk = (marks[0] if g == 0 else None, marks[1] if g == G - 1 else None)
            if g:
                after = (lambda q=self.pipes[g - 1]: q.done)
            elif first_all and G > 1:
                after = (lambda: [q.prep_done for q in self.pipes[1:]])
            else:
                after = None
            gens.append(p.steps(mk, after=after, prev_pipe=prevs[g] if g < len(prevs) else None))
        live = list(gens)
        while live:
            for gen in list(live):
                try:
                    next(gen)
                except StopIteration:
                    live.remove(gen)
        for p in self.pipes:
            cur.wait_stream(p.stream)
        self._lockstep()
        if check_device:
            self.finish()
        return None if self.pending else self.result()

    def _lockstep(self):
        """Pipelining is decided for all groups at once: if any
        group's pass declined it, every group flushes and stops pipelining, and
        outputs left in the other buffer move into the first group's."""
        if all(p.pipelined for p in self.pipes) or not any(p.pipelined for p in self.pipes):
            return
        torch = _torch()
        cur = torch.cuda.current_stream()
        for p in self.pipes:
            p.flush()
            cur.wait_stream(p.stream)
            p.pipelined = False
        y0 = self.pipes[0].y
        for p in self.pipes[1:]:
            if p.y.data_ptr() != y0.data_ptr():
                for o, n in zip(p.out_offs, p.res_lens):
                    y0[o:o + n * p.ss.ch].copy_(p.y[o:o + n * p.ss.ch])
                p.y = y0
        self.y = y0

    @property
    def pending(self) -> bool:
        return any(p.pending for p in self.pipes)

    @property
    def pipelined(self) -> bool:
        return all(p.pipelined for p in self.pipes)

    def flush(self):
        """Pipelined: every group's last global limiter (then the current
        stream waits for them)."""
        torch = _torch()
        cur = torch.cuda.current_stream()
        for p in self.pipes:
            p.flush()
            cur.wait_stream(p.stream)
        self.y = self.pipes[0].y

    def finish(self) -> int:
        bits = 0
        for p in self.pipes:
            bits |= p.finish()
        return bits

    def result(self) -> Result:
        self.flush()
        return merge_results([p.result() for p in self.pipes])


# ---------------------------------------------------------------------------
# static EQ (layer2 / layer2b)
# ---------------------------------------------------------------------------

class StaticEqPipeline:
    """One static gain row through the STFT-OLA (layer2_apply_eq with/without pad,
    layer2b_apply_residual_eq = no pad).  Output keeps the head pad (layer2)."""

    def __init__(self, ss: StreamSet, gain_bins: np.ndarray, *, n_fft=4096, hop=2048,
                 pad=True, global_gain_db=0.0):
        torch = _torch()
        _check_fft(n_fft, hop, ss.ch)
        self.ss, self.n_fft, self.hop = ss, n_fft, hop
        pl = n_fft // 2 if pad else 0
        g_global = 10.0 ** (global_gain_db / 20.0)
        streams = []
        for off, N in zip(ss.offs, ss.lens):
            total = N + 2 * pl
            F = (total - n_fft) // hop + 1 if total >= n_fft else 0
            st = TomatisStream()
            st.in_off, st.n, st.first_start, st.n_frames = off, N, -pl, F
            st.out_begin = -pl
            st.out_len = (F - 1) * hop + n_fft if F else 0
            st.n_chunks, st.chunk_first, st.chunk_len = 1, 0, 1
            st.in_scale, st.out_scale = float(np.float32(g_global)), 1.0
            streams.append(st)
        self.y, out_offs = _alloc_out(torch, [s.out_len for s in streams], ss.ch, ss.x.device)
        for st, o in zip(streams, out_offs):
            st.out_off = o
        desc = TomatisPlanDesc(n_fft=n_fft, hop=hop, ch=ss.ch, norm_mode=NORM_EPS,
                               up_delay_frames=0, min_hold_frames=0, xfade_frames=0,
                               alpha_mode=0)
        self.plan = Plan(desc, dsp.hann(n_fft), streams)
        Ft = max(1, self.plan.total_frames)
        dev = ss.x.device
        self.rows = torch.zeros(Ft + 1, dtype=torch.int16, device=dev)  # +1: read as u32 words
        self.peaks = torch.zeros(max(1, self.plan.total_chunks), dtype=torch.int32, device=dev)
        self.gains = torch.from_numpy(np.asarray(gain_bins, np.float32)[None, :].copy()).to(dev)
        self.out_offs = out_offs

    def run(self, marks=None, check_device: bool = True):
        L, P, hs = lib(), self.plan.h, stream_handle()
        self.peaks.zero_()
        if marks:
            marks[0].record()
        check(L.tomatis_stft_ola(P, ptr(self.ss.x), ptr(self.gains), 1, ptr(self.rows),
                                 ptr(self.y), ptr(self.peaks), hs), "stft_ola")
        if marks:
            marks[1].record()
        if check_device:
            self.finish()
        return self.result()

    def finish(self) -> int:
        # no limiter in this pass: only the exchange-barrier check applies
        return finish_plan(self.plan, None, "StaticEqPipeline")

    def result(self) -> Result:
        st = list(self.plan.streams)[:self.ss.n_streams]
        return Result(y=self.y, out_offs=self.out_offs, out_lens=[s.out_len for s in st],
                      ch=self.ss.ch, frame_base=[s.frame_base for s in st],
                      n_frames=[s.n_frames for s in st],
                      first_start=[s.first_start for s in st], hop=self.hop,
                      chunk_peaks=self.peaks, chunk_base=[s.chunk_base for s in st],
                      n_chunks=[s.n_chunks for s in st],
                      extra=dict(n_fft=self.n_fft, norm="eps", limit=None,
                                 limiter_applied=False, out_begin=[s.out_begin for s in st]))


def scale_copy(src, scale: float):
    """Device ``src * float32(scale)`` into a new tensor (layer-2 gain protect)."""
    torch = _torch()
    out = torch.empty_like(src)
    check(lib().tomatis_scale_copy(ptr(src), ptr(out), src.numel(), float(np.float32(scale)),
                                   stream_handle()), "scale_copy")
    return out


def frame_r(x: np.ndarray, sr: int, n_fft: int, hop: int, first_start: int, n_frames: int,
            precision=F32, in_scale: float = 1.0) -> np.ndarray:
    """Per-frame RMS r of one stream on the GPU (levels kernel), returned to host."""
    torch = _torch()
    ss = StreamSet.from_arrays([x], sr)
    st = TomatisStream()
    st.in_off, st.n, st.first_start, st.n_frames = 0, len(x), first_start, n_frames
    st.out_begin, st.out_len, st.n_chunks, st.chunk_len = first_start, 0, 1, 1
    st.in_scale, st.out_scale = in_scale, 1.0
    desc = TomatisPlanDesc(n_fft=n_fft, hop=hop, ch=ss.ch, norm_mode=NORM_EPS,
                           up_delay_frames=0, min_hold_frames=0, xfade_frames=0, alpha_mode=0)
    plan = Plan(desc, dsp.hann(n_fft), [st])
    dt = torch.float32 if precision == F32 else torch.float64
    r = torch.empty(max(1, n_frames), dtype=dt, device=ss.x.device)
    check(lib().tomatis_levels(plan.h, ptr(ss.x), ptr(r), precision, stream_handle()), "levels")
    out = r[:n_frames].cpu().numpy()
    plan.close()
    return out


def compute_frame_levels(x, sr, n_fft, hop, silence_threshold=-70):
    """GPU version of process_tomatis_adaptive.compute_frame_levels
    (src/process_tomatis_adaptive.py:57-84): (levels, valid_mask, times).

    The input dtype decides the level precision as in the reference."""
    x = np.asarray(x)
    if x.ndim == 1:
        x = x.reshape(-1, 1)
    N = len(x)
    k0, F, s0 = dsp.adaptive_frames(N, n_fft, hop)
    prec = F64 if x.dtype == np.float64 else F32
    if x.dtype == np.float64 and not np.array_equal(x.astype(np.float32).astype(np.float64), x):
        raise ValueError("float64 input must be exactly representable in float32 "
                         "(the reference feeds float32 PCM scaled by 1.0)")
    r = frame_r(x.astype(np.float32), sr, n_fft, hop, s0, F, precision=prec)
    levels = dsp.r_to_level(r)
    valid = levels > silence_threshold
    frame_sec = hop / sr
    times = [(i + 1) * frame_sec for i in range(len(levels))]
    return levels, valid, times


def simulate_gate(levels, threshold_dbfs, hyst_db=3.0, min_hold_frames=6):
    """GPU min-hold gate (src/process_tomatis_adaptive.py:87-121): list of 'C1'/'C2'."""
    st = _minhold_states(np.asarray(levels, np.float64), [(np.nan, np.nan, threshold_dbfs)],
                         hyst_db, min_hold_frames, 0.5)[0]
    return ["C1" if s == 1 else "C2" for s in st]


def find_optimal_threshold(levels, valid_mask, hyst_db=3.0, min_hold_frames=6, target_c2=0.5):
    """GPU bisection (src/process_tomatis_adaptive.py:124-154)."""
    levels = np.asarray(levels, np.float64)
    valid = levels[valid_mask]
    if len(valid) == 0:
        return np.median(levels)
    tlh = (np.percentile(valid, 5), np.percentile(valid, 95), np.median(valid))
    return _minhold_states(levels, [tlh], hyst_db, min_hold_frames, target_c2)[1][0]


def _minhold_states(levels, tlhs, hyst_db, mh, target):
    torch = _torch()
    F = len(levels)
    st = TomatisStream()
    st.n, st.first_start, st.n_frames = 0, 0, F
    st.out_begin, st.out_len, st.n_chunks, st.chunk_len = 0, 0, 1, 1
    st.in_scale, st.out_scale = 1.0, 1.0
    desc = TomatisPlanDesc(n_fft=2048, hop=512, ch=1, norm_mode=NORM_MAX, up_delay_frames=0,
                           min_hold_frames=mh, xfade_frames=1, alpha_mode=2)
    plan = Plan(desc, dsp.hann(2048), [st])
    dev = "cuda"
    lv = torch.from_numpy(levels).to(dev)
    tl = torch.tensor(np.asarray(tlhs, np.float64).reshape(-1), device=dev)
    states = torch.empty(max(1, F), dtype=torch.uint8, device=dev)
    t_out = torch.empty(1, dtype=torch.float64, device=dev)
    check(lib().tomatis_minhold_bisect(plan.h, ptr(lv), ptr(tl), target, hyst_db, ptr(t_out),
                                       ptr(states), None, None, stream_handle()), "minhold")
    out = states[:F].cpu().numpy(), t_out.cpu().numpy()
    plan.close()
    return out


__all__ = ["StreamSet", "Plan", "DeviceCheckError", "finish_plan", "GatePipeline", "AdaptivePipeline", "AdaptiveGroups", "StaticEqPipeline",
           "Result", "merge_results", "scale_copy", "frame_r", "compute_frame_levels", "simulate_gate",
           "find_optimal_threshold"]
