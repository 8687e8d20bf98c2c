#!/usr/bin/env python3
"""Throughput of the analysis spectra on one MI355X, next
to the oracle (numpy, 1 thread) on the same input.  Prints one JSON line per
function.  Inputs resident in HBM; HIP events on the library's stream.

  compare:  stft_mag_avg of power_mono, 60 min stereo 48 kHz, 4096/2048
  analyze:  stft_logpower_median, 6 min stereo 48 kHz, 8192/4096, -65 dBFS
  validate: compute_conditional_spectrum, 60 min stereo 44.1 kHz, 2048/512
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import analysis as an
    from tomatis_audio_processor_amd._lib import check, lib, ptr, stream_handle
    from oracle import tomatis_oracle as orc
    steps = int(os.environ.get("AN_STEPS", "5"))

    def dev_synth(n, sr, seed):
        x = torch.empty(n * 2, dtype=torch.float32, device="cuda")
        check(lib().tomatis_synth_fill(ptr(x), n, 2, sr, seed, 0, stream_handle()), "synth")
        return x.view(n, 2)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    def spec_kernel_ms(x, n, ch, n_fft, hop, kind, sig, y=None):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        an._spectra(x, y, n, ch, n_fft, hop, kind, sig)
        e0.record(s)
        for _ in range(steps):
            an._spectra(x, y, n, ch, n_fft, hop, kind, sig)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    out = []
    # compare_audio
    n, sr = 3600 * 48000, 48000
    x = dev_synth(n, sr, 2000)
    t = timeit(lambda: an.stft_mag_avg(x, sr, 4096, 2048, premix="power_mono", as_tensor=True))
    F = 1 + (n - 4096) // 2048
    kms = spec_kernel_ms(x, n, 2, 4096, 2048, an.AN_MAG, an.AN_SIG_POWER_MONO)
    rd = F * 4096 * 8  # frame bytes read (stereo f32), 2x overlap
    xs = x[: 300 * sr].cpu().numpy()
    t0 = time.perf_counter()
    orc.stft_mag_avg(orc.power_mono(xs), sr, 4096, 2048)
    cpu = 300 * sr * 2 / (time.perf_counter() - t0) / 1e6
    out.append(dict(fn="stft_mag_avg", workload="60 min stereo 48k power-mono, 4096/2048",
                    ms=round(t * 1e3, 3), msamples_s=round(n * 2 / t / 1e6, 1),
                    spec_kernel_ms=round(kms, 3),
                    spec_kernel_gbs=round((rd + F * 2049 * 4) / kms / 1e6, 1),
                    cpu_oracle_msamples_s=round(cpu, 2), cpu_sample="first 5 min, 1 thread"))
    # layer2_analyze_eq
    n = 360 * sr
    x6 = x[:n]
    t = timeit(lambda: an.stft_logpower_median(x6, sr, 8192, 4096, -65.0))
    xs = x6.cpu().numpy()
    t0 = time.perf_counter()
    orc.stft_logpower_median(xs, sr, 8192, 4096, -65.0)
    cpu = n * 2 / (time.perf_counter() - t0) / 1e6
    out.append(dict(fn="stft_logpower_median", workload="6 min stereo 48k, 8192/4096",
                    ms=round(t * 1e3, 3), msamples_s=round(n * 2 / t / 1e6, 1),
                    cpu_oracle_msamples_s=round(cpu, 2), cpu_sample="whole input, 1 thread"))
    # validate_layer1
    sr = 44100
    n = 3600 * sr
    xv = dev_synth(n, sr, 2001)
    yv = (xv * 0.7).contiguous()
    nf = 1 + n // 512
    states = (["C1"] * 40 + ["C2"] * 35) * (nf // 75 + 1)
    states = states[:nf]
    t = timeit(lambda: an.compute_conditional_spectrum(xv, yv, sr, states, 2048, 512, -60))
    F = 1 + (n - 2048) // 512
    kms = spec_kernel_ms(xv, n, 2, 2048, 512, an.AN_RATIO, an.AN_SIG_RAW, y=yv)
    xs, ys = xv[: 120 * sr].cpu().numpy(), yv[: 120 * sr].cpu().numpy()
    t0 = time.perf_counter()
    orc.compute_conditional_spectrum(xs, ys, sr, states[: 1 + 120 * sr // 512], 2048, 512, -60)
    cpu = 120 * sr * 2 / (time.perf_counter() - t0) / 1e6
    out.append(dict(fn="compute_conditional_spectrum", workload="60 min stereo 44.1k, 2048/512",
                    ms=round(t * 1e3, 3), msamples_s=round(n * 2 / t / 1e6, 1),
                    spec_kernel_ms=round(kms, 3),
                    spec_kernel_gbs=round((F * 2048 * 16 + F * 1025 * 4) / kms / 1e6, 1),
                    cpu_oracle_msamples_s=round(cpu, 2), cpu_sample="first 2 min, 1 thread"))
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
