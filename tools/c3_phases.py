#!/usr/bin/env python3
"""Wall-clock phases of one adaptive (C3) step: monkeypatched timers around the
library calls and host statistics of AdaptivePipeline.run."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import engine, dsp
    ss = engine.StreamSet.synthetic(64, 300 * 44100, 2, 44100, seed0=1000)
    pipe = engine.AdaptivePipeline(ss, n_fft=2048, hop=512)
    pipe.run()
    torch.cuda.synchronize()
    acc = {}
    orig_lib = engine.lib
    orig_r2l = dsp.r_to_level

    class Timed:
        def __init__(self, h):
            self.h = h

        def __getattr__(self, name):
            f = getattr(self.h, name)
            if not name.startswith("tomatis_"):
                return f

            def g(*a):
                t = time.perf_counter()
                rc = f(*a)
                torch.cuda.synchronize()
                acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
                return rc
            return g

    def r2l(r):
        t = time.perf_counter()
        out = orig_r2l(r)
        acc["host_log10(sum over threads)"] = acc.get("host_log10(sum over threads)", 0) + \
            time.perf_counter() - t
        return out
    engine.lib = lambda: Timed(orig_lib())
    dsp.r_to_level = r2l
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.run()
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    print(f"step {tot * 1e3:.1f} ms")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:40s} {v * 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
