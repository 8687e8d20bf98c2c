"""World-size-2 gloo run of the multi-GPU data path's host logic: LPT shard of a
512-stream batch and the manifest all_gather (the only collective)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    import torch.distributed as dist
    from tomatis_audio_processor_amd import sharding
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    costs = [14_400_000 * 2] * 509 + [1000, 2000, 3000]
    mine = sharding.lpt_partition(costs, ws)[rank]
    rec = np.array([[i, rank, 28124, 14000 + i, 7, 18, 18, 0x3F7FBE77, 0] for i in mine],
                   np.int64).reshape(-1, sharding.REC)
    allr = sharding.gather_manifest(rec)
    q.put((rank, len(mine), allr.shape, allr[:, 0].tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2])
def test_gloo_manifest_gather(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    counts = {r: n for r, n, _, _ in out}
    assert sum(counts.values()) == 512 and abs(counts[0] - counts[1]) <= 2
    for _, _, shape, ids in out:
        from tomatis_audio_processor_amd import sharding
        assert shape == (512, sharding.REC) and ids == list(range(512))


def _ts_worker(rank, ws, port, q):
    """Time-shard exchanges over gloo: gate summaries (all_gather) and chunk
    peaks (all_reduce MAX) reproduce the single-rank results."""
    import numpy as np
    import torch.distributed as dist
    from tomatis_audio_processor_amd import timeshard as T
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    rng = np.random.default_rng(5)
    pred = rng.choice([0, 1, 2], size=4096, p=[0.3, 0.5, 0.2]).astype(np.uint8)
    pred = np.repeat(pred[:512], 8)  # runs of 8 frames
    D = 7
    bs = [0, 2560, 4096]
    a, b = bs[rank], bs[rank + 1]
    sums = T.exchange_summaries(T.gs_shift(T.summarize(pred[a:b], D), a))
    mine = T.resolve(pred[a:b], D, T.carry_in(sums, rank, D), k0=a)
    g = np.zeros(16, np.uint32)
    g[rank * 6:rank * 6 + 10] = np.arange(10, dtype=np.uint32) + 100 * rank
    gmax = T.exchange_peaks(g)
    q.put((rank, mine.tolist(), gmax.tolist(), T.resolve(pred, D).tolist()))
    dist.destroy_process_group()


def test_gloo_timeshard_exchanges():
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ts_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(ws)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    states = out[0][1] + out[1][1]
    assert states == out[0][3]
    exp = np.zeros(16, np.uint32)
    for r in range(ws):
        g = np.zeros(16, np.uint32)
        g[r * 6:r * 6 + 10] = np.arange(10, dtype=np.uint32) + 100 * r
        exp = np.maximum(exp, g)
    assert out[0][2] == exp.tolist() == out[1][2]
