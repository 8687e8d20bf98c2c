"""File-parallel multi-GPU sharding.

Streams are independent (per-stream gate, thresholds, limiter chunks), so the
batch is partitioned across ranks with longest-processing-time balancing on
``n * ch`` and each rank processes its shard as one stream set on its own GPU.
There is no data-path collective.  The only exchange is one all_gather of
fixed-size per-stream manifest records (RCCL over xGMI with the ``nccl``
backend on device tensors; ``gloo`` on CPU tensors in the tests).
"""
from __future__ import annotations

import heapq
from typing import List, Sequence

import numpy as np

# manifest record layout (int64)
MANIFEST_FIELDS = ("stream", "rank", "frames", "c2_frames", "switches", "chunks",
                   "limited_chunks", "peak_bits", "ill_chunks")
REC = len(MANIFEST_FIELDS)


def lpt_partition(costs: Sequence[int], n_ranks: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment; deterministic for equal costs
    (ties broken by stream index, then rank index)."""
    order = sorted(range(len(costs)), key=lambda i: (-int(costs[i]), i))
    heap = [(0, r) for r in range(n_ranks)]
    heapq.heapify(heap)
    out: List[List[int]] = [[] for _ in range(n_ranks)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + int(costs[i]), r))
    return [sorted(s) for s in out]


def stream_records(res, stream_ids, rank: int) -> np.ndarray:
    """Manifest rows for the streams of one ``engine.Result`` (host numpy).

    ``ill_chunks``: limiter chunks whose scale an ill-conditioned edge sample
    may set (``Result.scale_flags``, conditioning.py), i.e. chunks whose scale
    may differ from the reference's."""
    rows = []
    for j, sid in enumerate(stream_ids):
        st = res.stream_states(j) if res.states is not None else np.zeros(0, np.uint8)
        pk = res.stream_peaks(j) if res.chunk_peaks is not None else np.zeros(1, np.float32)
        limited = int(np.count_nonzero(pk > 0.999))
        ill = int(sum(res.scale_flags(j))) if hasattr(res, "scale_flags") else 0
        rows.append([sid, rank, len(st), int(np.count_nonzero(st == 2)),
                     int(np.count_nonzero(st[1:] != st[:-1])) if len(st) else 0,
                     len(pk), limited, int(np.float32(pk.max() if len(pk) else 0).view(np.uint32)),
                     ill])
    return np.asarray(rows, np.int64).reshape(-1, REC)


def gather_manifest(records: np.ndarray, device=None) -> np.ndarray:
    """all_gather fixed-size records from every rank (pads to the max count).

    ``device``: torch device for the collective tensors ("cuda" with nccl/RCCL,
    None/"cpu" with gloo).  Returns the concatenated records, stream-sorted.
    """
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return records[np.argsort(records[:, 0], kind="stable")] if len(records) else records
    ws = dist.get_world_size()
    dev = torch.device(device) if device is not None else torch.device("cpu")
    n = torch.tensor([records.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(counts, n)
    m = int(max(int(c.item()) for c in counts))
    buf = torch.full((max(1, m), REC), -1, dtype=torch.int64, device=dev)
    if records.shape[0]:
        buf[:records.shape[0]] = torch.from_numpy(records).to(dev)
    bufs = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(bufs, buf)
    allr = torch.cat([b[:int(c.item())] for b, c in zip(bufs, counts)]).cpu().numpy()
    return allr[np.argsort(allr[:, 0], kind="stable")]
