#!/usr/bin/env python3
"""Synchronised phase breakdown of one C3 adaptive step (64 x 5 min stereo
44.1 kHz, 2048/512) — where the non-kernel time goes.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import engine
    nstr = int(os.environ.get("PROF_STREAMS", "64"))
    sr, ch, secs = 44100, 2, 300
    ss = engine.StreamSet.synthetic(nstr, secs * sr, ch, sr, seed0=1000)
    pipe = engine.AdaptivePipeline(ss, n_fft=2048, hop=512)
    for _ in range(3):
        pipe.run()
    torch.cuda.synchronize()
    K = 5
    tm = {}
    for _ in range(K):
        pipe.run(timer=tm)
    out = {k: round(v / K * 1e3, 3) for k, v in tm.items()}
    out["sum_ms"] = round(sum(tm.values()) / K * 1e3, 3)
    out["frames"] = pipe.plan.total_frames
    out["prec"] = sorted(set(pipe.prec))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
