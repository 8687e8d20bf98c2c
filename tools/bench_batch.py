#!/usr/bin/env python3
"""File -> file rate of the multi-file batch runner (batch.py) on one GPU: a
C4-share job (64 x 5 min stereo 48 kHz FLAC PCM_24 files by default, standard
mode, 2048/512) run as a pipeline of batches (batch k+1's transform limits
batch k's output; host decode of k+1 and encode of k-1 overlap batch k) and
with --no_pipeline, same files; outputs compared byte for byte.  One JSON line.

    BATCH_FILES=64 BATCH_SECS=300 BATCH_GB=8 python tools/bench_batch.py
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import batch, engine, fileio
    nf = int(os.environ.get("BATCH_FILES", "64"))
    secs = int(os.environ.get("BATCH_SECS", "300"))
    gb = float(os.environ.get("BATCH_GB", "8"))
    sr, ch = 48000, 2
    n = secs * sr
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        files = []
        for i in range(nf):
            ss = engine.StreamSet.synthetic(1, n, ch, sr, seed0=1000 + i)
            p = os.path.join(d, f"in{i:03d}.flac")
            with open(p, "wb") as f:
                f.write(fileio.encode_flac_device(ss.x, n, ch, sr, 24))
            files.append(p)
            del ss
        torch.cuda.synchronize()
        base = ["-i", *files, "--n_fft", "2048", "--hop", "512", "--out_ext", "flac",
                "--batch_gb", str(gb)]
        # warm-up (kernels, pinned allocator, codec threads) on the first 4 files
        batch.main(["-i", *files[:4], "--n_fft", "2048", "--hop", "512", "--out_ext", "flac",
                    "--out_dir", os.path.join(d, "warm")])
        times = {}
        for name, extra in (("pipelined", []), ("unpipelined", ["--no_pipeline"])):
            od = os.path.join(d, name)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            assert batch.main(base + ["--out_dir", od] + extra) == 0
            torch.cuda.synchronize()
            times[name] = time.perf_counter() - t0
        same = all(open(os.path.join(d, "pipelined", f"in{i:03d}_tomatis.flac"), "rb").read() ==
                   open(os.path.join(d, "unpipelined", f"in{i:03d}_tomatis.flac"), "rb").read()
                   for i in range(nf))
        man_same = (open(os.path.join(d, "pipelined", "manifest.json")).read() ==
                    open(os.path.join(d, "unpipelined", "manifest.json")).read())
        in_mb = sum(os.path.getsize(f) for f in files) / 1e6
    S = nf * n * ch / 1e6
    n_batches = len(batch.split_batches(list(range(nf)), {i: n * ch for i in range(nf)},
                                        int(gb * 2 ** 30 / 4)))
    print(json.dumps({
        "workload": f"C4 share file->file: {nf} x {secs} s stereo {sr} Hz FLAC PCM_24 "
                    f"({in_mb:.0f} MB), standard 2048/512, batch.py --batch_gb {gb} "
                    f"({n_batches} batches)",
        "pipelined_s": round(times["pipelined"], 3),
        "unpipelined_s": round(times["unpipelined"], 3),
        "pipelined_msamples_s": round(S / times["pipelined"], 1),
        "unpipelined_msamples_s": round(S / times["unpipelined"], 1),
        "outputs_byte_identical": same, "manifests_identical": man_same,
    }), flush=True)


if __name__ == "__main__":
    main()
