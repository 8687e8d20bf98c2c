#!/usr/bin/env python3
"""File -> file timing of the layer-2 CLI path (``layer2_apply_eq.apply_eq_stft``,
src/layer2_apply_eq.py:66-237): one stereo 48 kHz FLAC PCM_24 file through the
device file path (fileio ingest, static-EQ STFT/OLA, streaming FLAC egress, and
the gain-protected ``_gp`` copy re-quantised and scaled on the device), against
the host path the CLI used before (audio_io.read -> StreamSet.from_arrays ->
Result.output -> audio_io.write, ``_gp`` scaled and encoded from host arrays).
One JSON line; ``BENCH_L2_SECS`` sets the file length (default 600 s)."""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import audio_io, engine, fileio, layer2_apply_eq as L2
    from tests.golden.cases import eq_csv_rows
    secs = int(os.environ.get("BENCH_L2_SECS", "600"))
    sr, ch = 48000, 2
    n = secs * sr
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        src, out1, out2, eq = (os.path.join(d, f) for f in ("in.flac", "dev.flac", "host.flac",
                                                             "eq.csv"))
        open(eq, "w").write(eq_csv_rows())
        ss = engine.StreamSet.synthetic(1, n, ch, sr, seed0=77)
        with open(src, "wb") as f:
            f.write(fileio.encode_flac_device(ss.x, n, ch, sr, 24))
        del ss
        torch.cuda.synchronize()
        L2.apply_eq_stft(src, out1, eq)            # warm
        times = []
        for _ in range(2):
            t0 = time.perf_counter()
            r = L2.apply_eq_stft(src, out1, eq)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        gp = out1.replace(".flac", "_gp.flac")
        has_gp = os.path.exists(gp)
        # the host path of round 2
        t0 = time.perf_counter()
        x, _ = audio_io.read(src)
        fr, db = L2.load_eq_csv(eq)
        gb = L2.build_gain_per_bin(sr, 4096, fr, db)
        pipe = engine.StaticEqPipeline(engine.StreamSet.from_arrays([x], sr), gb, n_fft=4096,
                                       hop=2048, pad=True)
        res = pipe.run()
        y = res.output(0)
        audio_io.write(out2, y, sr, "FLAC", "PCM_24")
        peak = float(res.stream_peaks(0)[0])
        if peak > 0.99:
            audio_io.write(out2.replace(".flac", "_gp.flac"),
                           (y * np.float32(0.99 / peak)).astype(np.float32), sr, "FLAC", "PCM_24")
        t_host = time.perf_counter() - t0
        same = open(out1, "rb").read() == open(out2, "rb").read()
    S = n * ch / 1e6
    print(json.dumps({
        "workload": f"layer-2 file->file: {secs} s stereo 48 kHz FLAC PCM_24, 4096/2048, pad, "
                    f"gain protect {'on' if has_gp else 'off'} (peak {r['peak_seen']:.3f})",
        "device_path_s": round(min(times), 3),
        "device_path_msamples_s": round(S / min(times), 1),
        "host_path_s": round(t_host, 3),
        "host_path_msamples_s": round(S / t_host, 1),
        "main_outputs_byte_identical": same,
    }))


if __name__ == "__main__":
    main()
