#!/usr/bin/env python3
"""tomatis_levels (k_leaves + k_frame_r) time for one input size cut into 1..64
streams (diagnostic): 96 kHz stereo, n_fft 4096 hop 1024, 1.84 GB in all."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import engine
    from tomatis_audio_processor_amd._lib import F32, F64, check, lib, ptr, stream_handle
    sr, ch, total_s = 96000, 2, 4800
    for ns in (1, 4, 16, 64):
        n = total_s // ns * sr
        ss = engine.StreamSet.synthetic(ns, n, ch, sr, seed0=1000)
        pipe = engine.GatePipeline(ss, gate_ui=50, gate_offset=-90, n_fft=4096, hop=1024,
                                   xfade_ms=500.0)
        for prec, r in ((F32, pipe.r), (F64, torch.empty(pipe.r.numel(), dtype=torch.float64,
                                                           device="cuda"))):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            for k in range(13):
                if k == 3:
                    ev[0].record()
                check(lib().tomatis_levels(pipe.plan.h, ptr(ss.x), ptr(r), prec, stream_handle()),
                      "levels")
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / 10
            gb = ns * n * ch * 4 / 1e9
            print(f"streams {ns:3d} x {n / sr:6.0f} s  {'f32' if prec == F32 else 'f64'}: "
                  f"{ms:.3f} ms = {gb / ms:.2f} TB/s", flush=True)
        del pipe, ss
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
