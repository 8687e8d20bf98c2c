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
    rec = np.array([[i, rank, 28124, 14000 + i, 7, 18, 18, 0x3F7FBE77] for i in mine],
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
        assert shape == (512, 8) and ids == list(range(512))
