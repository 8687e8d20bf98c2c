"""Time sharding of one long stream across ranks.

A 60-min stream (config C2) is one unit of the file-parallel path, so on N GPUs
it would run on one of them.  Here its frames are cut into N contiguous shards,
one per rank (one process per GPU), each computed by the same kernels as a
whole stream, with two small exchanges:

* **gate carry** — the standard gate (src/process_tomatis.py:373-385) is
  sequential, but in its run-scan form it is an associative scan over
  per-segment summaries (include/tomatis_hip.h, "Time sharding").  Each rank
  reduces the summaries of its own frames to 5 int32, one ``all_gather``
  collects them, and every rank composes its predecessors' into its carry-in.
* **limiter peaks** — the 0.999 limiter's chunks (src/process_tomatis.py:
  331-357) are global; a chunk may straddle shards, so each rank's chunk
  maxima go through one ``all_reduce(MAX)`` before the fix-up scale.

The input needs no exchange: a rank reads its slice of the stream plus a halo
of ``rmax - 1`` warm-up frames (``n_fft - hop`` samples) before it, recomputes
those frames (they are the previous rank's last frames) and emits only its own
hop blocks.  Shard boundaries are placed so that every rank's summary range is
a whole number of gate segments.  Every output sample is the same frame-ordered
float32 sum as in the unsharded run, so the concatenated shards are
bit-identical to it (tests/test_gpu_timeshard.py).

Standard mode only (the xfade alpha and the adaptive bisection are further
sequential scans; not sharded).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence

import numpy as np

from . import dsp
from ._lib import GATE_NONE as NONE, GATE_SEGMENT

C1_IDLE = (-1, NONE, NONE)


# ---------------------------------------------------------------------------
# run-scan algebra (host mirror of tm_kernels.hip gs_cat / gs_apply)
# ---------------------------------------------------------------------------

def gs_identity():
    return (1, NONE, NONE, NONE, NONE)


def gs_cat(X, Y, D: int):
    """Summary of X followed by Y (associative)."""
    all_on = X[0] & Y[0]
    not_on = max(X[1], Y[1])
    off = max(X[4], Y[4])
    if X[0]:
        l_end = Y[2] if Y[2] != NONE else X[2]
        e_int = Y[3]
    else:
        l_end = X[2]
        lead = Y[2] if (Y[2] != NONE and Y[2] >= X[1] + D + 1) else NONE
        e_int = max(X[3], Y[3], lead)
    return (all_on, not_on, l_end, e_int, off)


def gs_apply(c, S, D: int):
    """Carry after a segment with summary S, from carry c = (a, e, f)."""
    a = c[0] if S[0] else S[1]
    lead = S[2] if (S[2] != NONE and S[2] >= c[0] + D + 1) else NONE
    return (a, max(c[1], S[3], lead), max(c[2], S[4]))


def _shift(v, off: int):
    return v if v == NONE else v + off


def gs_shift(S, off: int):
    """Re-index a summary by +off frames."""
    return (S[0], _shift(S[1], off), _shift(S[2], off), _shift(S[3], off), _shift(S[4], off))


def carry_shift(c, off: int):
    return (c[0] + off, _shift(c[1], off), _shift(c[2], off))


def summarize(pred: Sequence[int], D: int, k0: int = 0):
    """Summary of frames k0.. (host reference of k_gate_sum)."""
    S = gs_identity()
    for i, p in enumerate(pred):
        k = k0 + i
        fr = (1, NONE, k, NONE, NONE) if (p & 1) else (0, k, NONE, NONE, k if (p & 2) else NONE)
        S = gs_cat(S, fr, D)
    return S


def resolve(pred: Sequence[int], D: int, carry=C1_IDLE, k0: int = 0) -> np.ndarray:
    """States (1 = C1, 2 = C2) of frames k0.. from a carry (host reference of
    k_gate_states)."""
    c = carry
    out = np.empty(len(pred), np.uint8)
    for i, p in enumerate(pred):
        k = k0 + i
        fr = (1, NONE, k, NONE, NONE) if (p & 1) else (0, k, NONE, NONE, k if (p & 2) else NONE)
        c = gs_apply(c, fr, D)
        out[i] = 2 if c[1] > c[2] else 1
    return out


def carry_in(summaries_global: Sequence, rank: int, D: int):
    """Carry at the first frame of ``rank``'s summary range, from the summaries
    (global frame indices) of ranks 0..rank-1."""
    c = C1_IDLE
    for q in range(rank):
        c = gs_apply(c, summaries_global[q], D)
    return c


# ---------------------------------------------------------------------------
# shard geometry
# ---------------------------------------------------------------------------

@dataclass
class Shard:
    rank: int
    world: int
    b: int            # first local frame (global index): own frames minus warm-up
    k0: int           # first emitted frame
    k1: int           # one past the last emitted frame
    tf_frames: int    # frames [b, b + tf_frames) form this rank's gate summary
    lo: int           # input slice [lo, hi) (samples of the stream)
    hi: int
    p0: int           # output range [p0, p1) (samples of the stream)
    p1: int
    geometry: Dict = field(default_factory=dict)   # GatePipeline geometry (local)
    chunk_lo: int = 0                              # global index of local chunk 0
    edge_mask: int = 0    # bit 0: local chunk 0 shared with rank-1; bit 1: last with rank+1


def plan_shards(N: int, n_fft: int, hop: int, world: int, seg: int = GATE_SEGMENT,
                flush: int = 48000 * 5) -> List[Shard]:
    """Cut the standard-mode frames of an N-sample stream into ``world`` shards."""
    pad, pe, F, s0 = dsp.std_schedule(N, n_fft, hop)
    W = -(-n_fft // hop) - 1                     # warm-up frames of the register OLA
    bounds = dsp.std_flush_bounds(N, n_fft, hop, flush)
    nch = max(1, len(bounds) - 1)
    chunk_first = bounds[1] if len(bounds) > 2 else 0
    chunk_len = (bounds[2] - bounds[1]) if len(bounds) > 3 else max(
        1, (bounds[-1] - bounds[1]) if len(bounds) > 2 else 1)

    def chunk_of(p):
        if nch <= 1 or p < chunk_first:
            return 0
        return min(1 + (p - chunk_first) // chunk_len, nch - 1)

    def sk(k):
        return s0 + k * hop

    # b_0 = 0, b_{r+1} = b_r + seg * m_r; rank r emits [k0_r, k0_{r+1}), k0_r = b_r + W
    per = F / max(1, world)
    bs = [0]
    for r in range(1, world):
        m = max(1, int(round((r * per - W) / seg)) - (bs[-1] // seg))
        nb = bs[-1] + seg * m
        if nb + W >= F - 1:
            break
        bs.append(nb)
    R = len(bs)
    k0s = [0] + [b + W for b in bs[1:]]
    shards = []
    for r in range(R):
        b, k0 = bs[r], k0s[r]
        last = r == R - 1
        k1 = F if last else k0s[r + 1]
        kl = k1 - 1                                  # last local frame
        lo = max(0, sk(b))
        hi = N if last else min(N, sk(kl) + n_fft)
        p0 = 0 if r == 0 else sk(k0)
        p1 = N if last else sk(k1)
        c_lo, c_hi = chunk_of(p0), chunk_of(max(p0, p1 - 1))
        n_loc = c_hi - c_lo + 1
        geom = dict(first_start=sk(b) - lo, n_frames=kl - b + 1, out_begin=p0 - lo,
                    out_len=p1 - p0, n_chunks=n_loc,
                    chunk_first=(bounds[c_lo + 1] - lo) if n_loc > 1 else 0,
                    chunk_len=chunk_len if n_loc > 1 else 1,
                    bounds=[max(p0, bounds[c]) - lo for c in range(c_lo, c_hi + 1)] + [p1 - lo])
        tf = (bs[r + 1] - b) if not last else (kl - b + 1)
        edge = (1 if r > 0 and chunk_of(p0 - 1) == c_lo else 0) | \
               (2 if not last and chunk_of(p1) == c_hi else 0)
        shards.append(Shard(rank=r, world=R, b=b, k0=k0, k1=k1, tf_frames=tf, lo=lo, hi=hi,
                            p0=p0, p1=p1, geometry=geom, chunk_lo=c_lo, edge_mask=edge))
    return shards


def n_chunks_global(N: int, n_fft: int, hop: int, flush: int = 48000 * 5) -> int:
    return max(1, len(dsp.std_flush_bounds(N, n_fft, hop, flush)) - 1)


# ---------------------------------------------------------------------------
# one rank's pipeline, phase by phase
# ---------------------------------------------------------------------------

class ShardRunner:
    """The standard pipeline on one shard, device-resident end to end:
    levels -> gate summary (5 int32 on the device) | all_gather | carry-in and
    gate -> transform with the limiter fused for this shard's own chunks |
    all_reduce(MAX) of the shared edge chunks' peaks | limiter on those."""

    def __init__(self, x_slice, sr: int, shard: Shard, ch: int = 2, **params):
        """``x_slice``: the shard's input samples [lo, hi), host [n, ch] array or
        flat device float32 tensor (interleaved)."""
        import torch
        from . import engine
        self.shard = shard
        if hasattr(x_slice, "data_ptr"):
            ss = engine.StreamSet(x=x_slice, offs=[0], lens=[x_slice.numel() // ch], ch=ch, sr=sr)
        else:
            ss = engine.StreamSet.from_arrays([x_slice], sr)
        self.pipe = engine.GatePipeline(ss, geometry=[shard.geometry], **params)
        self.sum5 = torch.empty(5, dtype=torch.int32, device=ss.x.device)
        self.n_chunks = shard.geometry["n_chunks"]

    # phase 1
    def summary(self):
        """Levels, then this rank's gate summary in global frame indices
        (device int32[5], the all_gather input)."""
        from ._lib import check, lib, ptr, stream_handle, F32
        L, P, hs = lib(), self.pipe.plan.h, stream_handle()
        check(L.tomatis_levels(P, ptr(self.pipe.ss.x), ptr(self.pipe.r), F32, hs), "levels")
        n_tf_segs = -(-self.shard.tf_frames // GATE_SEGMENT)
        check(L.tomatis_ts_summary(P, ptr(self.pipe.r), n_tf_segs, self.shard.b, ptr(self.sum5),
                                   hs), "ts_summary")
        return self.sum5

    # phase 2
    def gate_and_transform(self, sums_all, marks=None):
        """Gate from the carry composed of ``sums_all`` (device int32[5 * world],
        rank order), then the transform; own chunks limited in the kernel.
        Returns the local chunk peaks (device, uint32 float bits as int32)."""
        from ._lib import check, lib, ptr, stream_handle
        from .engine import PEAK_LIMIT
        L, P, hs = lib(), self.pipe.plan.h, stream_handle()
        pp = self.pipe
        check(L.tomatis_ts_gate(P, ptr(pp.r), ptr(sums_all), self.shard.rank, -self.shard.b,
                                ptr(pp.states), ptr(pp.rows), hs), "ts_gate")
        pp.peaks.zero_()
        if marks:
            marks[0].record()
        check(L.tomatis_stft_ola_limited_edges(P, ptr(pp.ss.x), ptr(pp.gains), pp.n_rows,
                                               ptr(pp.rows), ptr(pp.y), ptr(pp.peaks), PEAK_LIMIT,
                                               self.shard.edge_mask, hs), "stft_ola_limited_edges")
        if marks:
            marks[1].record()
        return pp.peaks[:self.n_chunks]

    def redo_unfused(self):
        """Recovery after a fused-limiter wait timeout (engine.finish_plan): the
        transform again with the shard-local chunks limited by the separate
        launch.  Its peaks equal the first pass's (deterministic), so the edge
        chunks are then scaled with the already exchanged ``pipe.peaks``; no
        collective is repeated."""
        import torch
        from ._lib import check, lib, ptr, stream_handle
        from .engine import PEAK_LIMIT
        pp = self.pipe
        tmp = torch.zeros_like(pp.peaks)
        check(lib().tomatis_stft_ola_limited_edges(pp.plan.h, ptr(pp.ss.x), ptr(pp.gains),
                                                   pp.n_rows, ptr(pp.rows), ptr(pp.y), ptr(tmp),
                                                   PEAK_LIMIT, self.shard.edge_mask,
                                                   stream_handle()), "stft_ola_limited_edges")
        self.limit_edges()

    def finish(self) -> int:
        from .engine import finish_plan
        return finish_plan(self.pipe.plan, self.redo_unfused, f"time shard {self.shard.rank}")

    # phase 3
    def limit_edges(self):
        """Limiter on the shared edge chunks, whose exchanged peaks are in
        ``pipe.peaks``."""
        from ._lib import check, lib, ptr, stream_handle
        from .engine import PEAK_LIMIT
        pp = self.pipe
        check(lib().tomatis_apply_limiter_edges(pp.plan.h, ptr(pp.y), ptr(pp.peaks), PEAK_LIMIT,
                                                self.shard.edge_mask, stream_handle()),
              "limiter_edges")
        return pp.result()


def run_emulated(x: np.ndarray, sr: int, world: int, **params):
    """All shards of one stream in this process, the exchanges done with device
    tensor ops.  Returns (y [N, ch], states [F], per-chunk peaks as float) — the
    same values a ``world``-rank run produces."""
    import torch
    N, ch = x.shape
    n_fft, hop = params["n_fft"], params["hop"]
    shards = plan_shards(N, n_fft, hop, world)
    runners = [ShardRunner(x[s.lo:s.hi], sr, s, ch=ch, **params) for s in shards]
    sums_all = torch.cat([rn.summary() for rn in runners])
    G = n_chunks_global(N, n_fft, hop)
    gpk = torch.zeros(G, dtype=torch.int32, device=sums_all.device)
    for rn in runners:
        pk = rn.gate_and_transform(sums_all)
        c0, n = rn.shard.chunk_lo, rn.n_chunks
        gpk[c0:c0 + n] = torch.maximum(gpk[c0:c0 + n], pk)
    ys, sts = [], []
    for rn in runners:
        c0, n = rn.shard.chunk_lo, rn.n_chunks
        rn.pipe.peaks[:n].copy_(gpk[c0:c0 + n])
        res = rn.limit_edges()
        rn.finish()
        ys.append(res.output(0))
        s = rn.shard
        st = res.stream_states(0)
        sts.append(st[s.k0 - s.b:s.k1 - s.b])
    torch.cuda.synchronize()
    return (np.concatenate(ys), np.concatenate(sts),
            gpk.cpu().numpy().astype(np.uint32).view(np.float32))


# ---------------------------------------------------------------------------
# distributed run: one shard per rank (torch.distributed; RCCL on device
# tensors with the nccl backend, gloo on CPU tensors in the tests)
# ---------------------------------------------------------------------------

def _world():
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_initialized() else 1


def all_gather_cat(t):
    """Concatenation of every rank's tensor ``t`` (rank order)."""
    import torch
    import torch.distributed as dist
    if _world() == 1:
        return t
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.cat(out)


def all_reduce_max(t):
    """In-place MAX over ranks (non-negative float bit patterns order as ints)."""
    import torch.distributed as dist
    if _world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def exchange_summaries(S, device=None):
    """Host form of the summary exchange: every rank's 5-int summary."""
    import torch
    t = all_gather_cat(torch.tensor(S, dtype=torch.int64, device=device))
    return [tuple(int(v) for v in t[5 * q:5 * q + 5].cpu()) for q in range(t.numel() // 5)]


def exchange_peaks(global_bits: np.ndarray, device=None) -> np.ndarray:
    """Host form of the peak exchange: all_reduce(MAX) of per-chunk peak bits."""
    import torch
    t = all_reduce_max(torch.from_numpy(global_bits.astype(np.int64)).to(device or "cpu"))
    return t.cpu().numpy().astype(np.uint32)


class RankStep:
    """One rank's shard, set up once; ``run()`` = one pass with both exchanges,
    device-resident (no host synchronisation): bench.py workload c2ts."""

    def __init__(self, x_slice, sr: int, N: int, rank: int, world: int, ch: int = 2,
                 device="cuda", **params):
        import torch
        shards = plan_shards(N, params["n_fft"], params["hop"], world)
        if len(shards) != world:
            raise ValueError(f"stream too short for {world} shards")
        self.sh = shards[rank]
        self.rn = ShardRunner(x_slice, sr, self.sh, ch=ch, **params)
        self.G = n_chunks_global(N, params["n_fft"], params["hop"])
        self.gpk = torch.zeros(self.G, dtype=torch.int32, device=device)

    def run(self, marks=None, check_device: bool = True):
        """``check_device``: read the device error word at the end (engine.
        finish_plan; bench.py checks once after its timed loop instead)."""
        rn, sh = self.rn, self.sh
        sums_all = all_gather_cat(rn.summary())
        pk = rn.gate_and_transform(sums_all, marks)
        if _world() > 1:
            c0, n = sh.chunk_lo, rn.n_chunks
            self.gpk.zero_()
            self.gpk[c0:c0 + n] = pk
            all_reduce_max(self.gpk)
            pk.copy_(self.gpk[c0:c0 + n])
        res = rn.limit_edges()
        if check_device:
            rn.finish()
        return res

    def finish(self) -> int:
        return self.rn.finish()

    def result(self):
        return self.rn.pipe.result()


def run_rank(x_slice, sr: int, N: int, rank: int, world: int, ch: int = 2, device="cuda",
             **params):
    """This rank's shard of an N-sample stream (``x_slice`` = samples
    [shard.lo, shard.hi), host array or device tensor).  Returns (shard, Result).
    Collectives: one all_gather (gate summaries), one all_reduce (chunk peaks)."""
    st = RankStep(x_slice, sr, N, rank, world, ch=ch, device=device, **params)
    return st.sh, st.run()
