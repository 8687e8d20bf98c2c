"""Multi-file, multi-GPU batch processing (file-parallel).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 -m tomatis_audio_processor_amd.batch \
        --mode standard --out_dir out/ -i a.wav b.wav ...

Every rank reads the headers of all inputs, takes its LPT shard
(``sharding.lpt_partition`` on frames*channels), processes the shard as one
batched stream set per (sr, ch) format on its own GPU, writes its outputs, and
contributes fixed-size manifest records to one all_gather (RCCL over xGMI).
Rank 0 writes ``manifest.json``.  Single-process runs need no launcher.
"""
from __future__ import annotations

import argparse
import json
import os
from collections import defaultdict

import numpy as np

from . import audio_io, sharding


def _dist():
    import torch
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        dist.init_process_group(backend=backend, rank=rank, world_size=ws)
    return rank, ws


def output_names(inputs, ext):
    """``<stem>_tomatis.<ext>`` per input; inputs whose stems collide (same file
    name in different directories) get their input index appended, so no rank
    overwrites another stream's output.  Every rank computes the same names."""
    stems = [os.path.splitext(os.path.basename(p))[0] for p in inputs]
    count = defaultdict(int)
    for s in stems:
        count[s] += 1
    return [f"{s}_tomatis.{ext}" if count[s] == 1 else f"{s}_{i}_tomatis.{ext}"
            for i, s in enumerate(stems)]


def run(args):
    import torch
    from . import engine
    rank, ws = _dist()
    names = output_names(args.input, args.out_ext)
    infos = [audio_io.info(p) for p in args.input]
    costs = [fr * ch for (sr, ch, fr) in infos]
    mine = sharding.lpt_partition(costs, ws)[rank]
    groups = defaultdict(list)
    for i in mine:
        groups[(infos[i][0], infos[i][1])].append(i)
    os.makedirs(args.out_dir, exist_ok=True)
    recs = []
    params = dict(n_fft=args.n_fft, hop=args.hop)
    from . import fileio
    for (sr, ch), ids in sorted(groups.items()):
        # files decoded into HBM (fileio: FLAC via page-locked ranges, int -> float on device)
        parts = [fileio.read_device(args.input[i]) for i in ids]
        x = torch.cat([p[0] for p in parts]) if parts else torch.zeros(1, device="cuda")
        lens = [p[1] for p in parts]
        offs = list(np.cumsum([0] + [n * ch for n in lens[:-1]]).astype(int))
        del parts
        ss = engine.StreamSet(x=x, offs=offs, lens=lens, ch=ch, sr=sr)
        if args.mode == "adaptive":   # >= 4 files: two interleaved stream groups
            pipe = (engine.AdaptiveGroups(ss, groups=2, **params) if len(ids) >= 4
                    else engine.AdaptivePipeline(ss, **params))
        elif args.mode == "xfade":
            pipe = engine.GatePipeline(ss, gate_ui=args.gate_ui, gate_offset=args.gate_offset,
                                       xfade_ms=args.xfade_ms, **params)
        else:
            pipe = engine.GatePipeline(ss, gate_ui=args.gate_ui, gate_mode=args.gate_mode,
                                       gate_offset=args.gate_offset, **params)
        res = pipe.run()
        torch.cuda.synchronize()
        for j, i in enumerate(ids):
            out = os.path.join(args.out_dir, names[i])
            if args.out_ext == "wav":
                audio_io.write(out, res.output(j), sr, "WAV", "PCM_24")
            else:
                a = res.out_offs[j]
                fileio.write_device(out, res.y[a:a + res.out_lens[j] * ch], res.out_lens[j], ch,
                                    sr, log=lambda m: None)
        recs.append(sharding.stream_records(res, ids, rank))
    rec = np.concatenate(recs) if recs else np.zeros((0, sharding.REC), np.int64)
    dev = "cuda" if (ws > 1 and torch.cuda.is_available()) else None
    allrec = sharding.gather_manifest(rec, device=dev)
    if rank == 0:
        man = [dict(zip(sharding.MANIFEST_FIELDS, map(int, r)), path=args.input[int(r[0])],
                    out=names[int(r[0])]) for r in allrec]
        with open(os.path.join(args.out_dir, "manifest.json"), "w") as f:
            json.dump({"world_size": ws, "streams": man}, f, indent=1)
        print(f"[DONE] {len(man)} streams on {ws} GPU(s) -> {args.out_dir}/manifest.json")
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(description="Batch Tomatis processing on 1..8 MI355X")
    ap.add_argument("-i", "--input", nargs="+", required=True)
    ap.add_argument("--out_dir", required=True)
    ap.add_argument("--mode", choices=["standard", "xfade", "adaptive"], default="standard")
    ap.add_argument("--gate_ui", type=float, default=50)
    ap.add_argument("--gate_mode", choices=["linear", "log_percent"], default="log_percent")
    ap.add_argument("--gate_offset", type=float, default=-100)
    ap.add_argument("--xfade_ms", type=float, default=500.0)
    ap.add_argument("--n_fft", type=int, default=4096)
    ap.add_argument("--hop", type=int, default=2048)
    ap.add_argument("--out_ext", choices=["wav", "flac"], default="wav")
    return run(ap.parse_args(argv))


if __name__ == "__main__":
    raise SystemExit(main())
