#!/usr/bin/env python3
"""Multi-process check of the time-sharded path (timeshard.run_rank): W ranks
on one GPU (gloo for the two host-side exchanges), each computing its shard of
one stream; rank 0 compares the concatenated shards with the unsharded run
bit for bit.  Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29531 tools/timeshard_check.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from tomatis_audio_processor_amd import engine, timeshard
    from tomatis_audio_processor_amd.synth import synth_stream
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    sr, N = 44100, 44100 * 180 + 77
    params = dict(gate_ui=50, n_fft=2048, hop=512)
    x = synth_stream(42, N, 2, sr)
    sh = timeshard.plan_shards(N, 2048, 512, ws)[rank]
    sh2, res = timeshard.run_rank(x[sh.lo:sh.hi], sr, N, rank, ws, device=None, **params)
    torch.cuda.synchronize()
    y = torch.from_numpy(res.output(0).reshape(-1).copy())
    st = res.stream_states(0)[sh.k0 - sh.b:sh.k1 - sh.b]
    ys = [None] * ws
    sts = [None] * ws
    dist.all_gather_object(ys, y.numpy())
    dist.all_gather_object(sts, st)
    if rank == 0:
        ss = engine.StreamSet.from_arrays([x], sr)
        r = engine.GatePipeline(ss, **params).run()
        torch.cuda.synchronize()
        y_ref = r.output(0).reshape(-1)
        ok_y = np.concatenate(ys).tobytes() == y_ref.tobytes()
        ok_s = np.array_equal(np.concatenate(sts), r.stream_states(0))
        print(f"timeshard x{ws}: samples bit-identical={ok_y} states identical={ok_s}", flush=True)
        code = 0 if (ok_y and ok_s) else 1
    else:
        code = 0
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(code)


if __name__ == "__main__":
    main()
