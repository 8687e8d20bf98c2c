#!/usr/bin/env python3
"""PCIe- and codec-inclusive rates for C2 (one 60-min stereo 44.1 kHz stream):
host array -> HBM (StreamSet.from_arrays), the device step, HBM -> host output,
and the native FLAC codec (PCM_24) on the host.  One JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import audio_io, engine
    sr, n, ch = 44100, 3600 * 44100, 2
    ss0 = engine.StreamSet.synthetic(1, n, ch, sr, seed0=1000)
    x_host = ss0.x.cpu().numpy().reshape(n, ch)
    del ss0
    torch.cuda.synchronize()
    engine.PINNED_STAGING = False
    t0 = time.perf_counter()
    ss = engine.StreamSet.from_arrays([x_host], sr)
    torch.cuda.synchronize()
    t_h2d = time.perf_counter() - t0
    del ss
    engine.PINNED_STAGING = True
    t_stage = []
    for _ in range(2):  # first call allocates the page-locked block, the second reuses it
        t0 = time.perf_counter()
        ss = engine.StreamSet.from_arrays([x_host], sr)
        torch.cuda.synchronize()
        t_stage.append(time.perf_counter() - t0)
    pipe = engine.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    pipe.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = pipe.run()
    torch.cuda.synchronize()
    t_run = time.perf_counter() - t0
    engine.PINNED_STAGING = False
    t0 = time.perf_counter()
    y = res.output(0)
    t_d2h = time.perf_counter() - t0
    engine.PINNED_STAGING = True
    t_ostage = []
    for _ in range(2):
        t0 = time.perf_counter()
        y2 = res.output(0)
        t_ostage.append(time.perf_counter() - t0)
    assert np.array_equal(y2, y)
    del y2
    # pinned-staging variant of the two copies
    pin = torch.empty(n * ch, dtype=torch.float32, pin_memory=True)
    pin.numpy()[:] = x_host.reshape(-1)
    t0 = time.perf_counter()
    xd = pin.to("cuda", non_blocking=True)
    torch.cuda.synchronize()
    t_h2d_pin = time.perf_counter() - t0
    t0 = time.perf_counter()
    pin.copy_(xd, non_blocking=True)
    torch.cuda.synchronize()
    t_d2h_pin = time.perf_counter() - t0
    # FLAC PCM_24 codec on 60 s of the output (host, 1 thread)
    m = 60 * sr
    v = np.clip(np.rint(y[:m].astype(np.float64) * 8388607.0), -8388608, 8388607).astype(np.int32)
    t0 = time.perf_counter()
    blob = audio_io.flac_encode_int(v, sr, 24)
    t_enc = time.perf_counter() - t0
    t0 = time.perf_counter()
    back, _, _ = audio_io.flac_decode_int(blob)
    t_dec = time.perf_counter() - t0
    assert np.array_equal(back, v)
    S = n * ch / 1e6
    out = {
        "workload": "C2: 60 min stereo 44.1 kHz, standard, 2048/512",
        "bytes_each_way": n * ch * 4,
        "h2d_pageable_ms": round(t_h2d * 1e3, 1), "h2d_pageable_gbs": round(n * ch * 4 / t_h2d / 1e9, 1),
        "h2d_pinned_gbs": round(n * ch * 4 / t_h2d_pin / 1e9, 1),
        "device_step_ms": round(t_run * 1e3, 2),
        "d2h_pageable_ms": round(t_d2h * 1e3, 1), "d2h_pageable_gbs": round(n * ch * 4 / t_d2h / 1e9, 1),
        "d2h_pinned_gbs": round(n * ch * 4 / t_d2h_pin / 1e9, 1),
        "from_arrays_staged_ms": [round(t * 1e3, 1) for t in t_stage],
        "output_staged_ms": [round(t * 1e3, 1) for t in t_ostage],
        "e2e_host_to_host_msamples_s": round(S / (t_h2d + t_run + t_d2h), 1),
        "e2e_staged_msamples_s": round(S / (t_stage[1] + t_run + t_ostage[1]), 1),
        "e2e_pinned_msamples_s": round(S / (t_h2d_pin + t_run + t_d2h_pin), 1),
        "flac_pcm24_encode_msamples_s_threads": round(m * ch / t_enc / 1e6, 1),
        "flac_pcm24_decode_msamples_s_threads": round(m * ch / t_dec / 1e6, 1),
        "flac_ratio": round(len(blob) / (m * ch * 3), 3),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
