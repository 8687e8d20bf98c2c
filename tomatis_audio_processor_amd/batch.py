"""Multi-file, multi-GPU batch processing (file-parallel).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 -m tomatis_audio_processor_amd.batch \
        --mode standard --out_dir out/ -i a.wav b.wav ...

Every rank reads the headers of all inputs, takes its LPT shard
(``sharding.lpt_partition`` on frames*channels), cuts it per (sr, ch) format
into batches of at most ``--batch_gb`` of float input (``split_batches``),
processes them on its own GPU as a batch pipeline, writes its outputs, and
contributes fixed-size manifest records to one all_gather (RCCL over xGMI).
Rank 0 writes ``manifest.json``.  Single-process runs need no launcher.

Batch pipeline (the mode bench.py's headline times): batch k+1's transform
applies batch k's per-chunk limiter inside its frame loops
(``GatePipeline.run(prev_pipe=...)``, tomatis_stft_ola_gated_pipelined_after:
the batches' plans differ, their n_fft / hop / channels do not), so no batch
but the last pays the limiter's HBM re-read as a tail; while batch k runs on
the device the host decodes batch k+1's files and writes batch k-1's, whose
output the launch of batch k has just finalised.  ``--no_pipeline`` runs each
batch with its own limiter.  Outputs are byte-identical either way
(src/process_tomatis.py:331-357 limits each file's chunks; the pipeline only
moves where that multiply runs).
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


def split_batches(ids, samples, budget):
    """Consecutive batches of ``ids`` whose summed ``samples[i]`` (floats of
    input) stay within ``budget``; a file larger than the budget is a batch of
    its own.  Every id lands in exactly one batch, in order."""
    out, cur, acc = [], [], 0
    for i in ids:
        if cur and acc + samples[i] > budget:
            out.append(cur)
            cur, acc = [], 0
        cur.append(i)
        acc += samples[i]
    if cur:
        out.append(cur)
    return out


def _make_pipe(engine, args, ss, n_files, pipelined):
    params = dict(n_fft=args.n_fft, hop=args.hop)
    if args.mode == "adaptive":   # >= 4 files: two interleaved stream groups
        if n_files >= 4:
            return engine.AdaptiveGroups(ss, groups=2, pipelined=pipelined, second_buffer=False,
                                         **params)
        return engine.AdaptivePipeline(ss, pipelined=pipelined, second_buffer=False, **params)
    if args.mode == "xfade":
        return engine.GatePipeline(ss, gate_ui=args.gate_ui, gate_offset=args.gate_offset,
                                   xfade_ms=args.xfade_ms, pipelined=pipelined,
                                   second_buffer=False, **params)
    return engine.GatePipeline(ss, gate_ui=args.gate_ui, gate_mode=args.gate_mode,
                               gate_offset=args.gate_offset, pipelined=pipelined,
                               second_buffer=False, **params)


def run(args):
    import torch
    from . import engine, fileio
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
    budget = max(1, int(args.batch_gb * 2 ** 30 / 4))  # floats of input per batch
    pipelined = not args.no_pipeline

    def load(ids, ch, sr):
        # files decoded into HBM (fileio: FLAC via page-locked ranges, int -> float on device)
        parts = [fileio.read_device(args.input[i]) for i in ids]
        x = torch.cat([p[0] for p in parts]) if parts else torch.zeros(1, device="cuda")
        lens = [p[1] for p in parts]
        offs = list(np.cumsum([0] + [n * ch for n in lens[:-1]]).astype(int))
        return engine.StreamSet(x=x, offs=offs, lens=lens, ch=ch, sr=sr)

    def store(pipe, ids, ch, sr):
        """a batch whose output is final: device error check, files, manifest rows"""
        pipe.finish()             # (a gate / limiter redo rewrites its output, limited)
        res = pipe.result()
        for j, i in enumerate(ids):
            out = os.path.join(args.out_dir, names[i])
            if args.out_ext == "wav":
                audio_io.write(out, res.output(j), sr, "WAV", "PCM_24")
            else:
                a = res.out_offs[j]
                fileio.write_device(out, res.y[a:a + res.out_lens[j] * ch], res.out_lens[j], ch,
                                    sr, log=lambda m: None)
        recs.append(sharding.stream_records(res, ids, rank))

    for (sr, ch), ids in sorted(groups.items()):
        batches = split_batches(ids, {i: infos[i][2] * ch for i in ids}, budget)
        prev = None                 # (pipeline, ids) of the batch before
        ss = load(batches[0], ch, sr)
        for b, bids in enumerate(batches):
            pipe = _make_pipe(engine, args, ss, len(bids), pipelined)
            # batch b's transform limits batch b-1's output (or flushes it)
            pipe.run(check_device=False, prev_pipe=prev[0] if prev else None)
            if b + 1 < len(batches):
                ss = load(batches[b + 1], ch, sr)   # host decode overlaps batch b
            if prev is not None:
                store(*prev, ch, sr)
                prev = None
            prev = (pipe, bids)
        store(*prev, ch, sr)        # result() flushes the last batch's limiter
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
    ap.add_argument("--batch_gb", type=float, default=16.0,
                    help="float input per batch (GiB): a rank's files run as a pipeline of "
                         "batches of at most this size")
    ap.add_argument("--no_pipeline", action="store_true",
                    help="every batch applies its own limiter (no overlap with the next batch)")
    return run(ap.parse_args(argv))


if __name__ == "__main__":
    raise SystemExit(main())
