"""Is the fused kernel bound by something shared by a CU pair (the SQC
instruction cache) or by per-CU resources?  Times the C2 transform on streams
whose CU mask enables all CUs, every other CU, or half of them
(hipExtStreamCreateWithCUMask).  Diagnostic only.

usage: python tools/cumask_probe.py [--input-gain G]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tomatis_audio_processor_amd import engine
    gain = float(sys.argv[sys.argv.index("--input-gain") + 1]) if "--input-gain" in sys.argv else 1.0
    hip = C.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32

    def mask(pred):
        m = [0] * words
        for c in range(ncu):
            if pred(c):
                m[c // 32] |= 1 << (c % 32)
        return (C.c_uint32 * words)(*m)

    # mask bit c -> XCC c % 8, local index l = c // 8 -> SE l % 4, l // 4 the
    # CU's rank in its SE (tools/cumask_probe.py --layout); an SQC (instruction
    # cache) serves hardware CUs 2k and 2k+1, i.e. ranks (2j, 2j+1)
    rank = lambda c: (c // 8) // 4  # noqa: E731
    masks = {"all": lambda c: True,
             "sqc_one": lambda c: rank(c) % 2 == 0,       # one CU of every SQC pair
             "sqc_both": lambda c: rank(c) % 4 < 2,       # both CUs of half the pairs
             "sqc_one_q": lambda c: rank(c) % 4 == 0,     # one CU of every other pair
             "sqc_both_q": lambda c: rank(c) < 2}         # both CUs of a quarter of pairs
    sr, n = 44100, 3600 * 44100
    ss = engine.StreamSet.synthetic(1, n, 2, sr, seed0=1000)
    if gain != 1.0:
        ss.x = engine.scale_copy(ss.x, gain)
    pipe = engine.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    pipe.run()
    torch.cuda.synchronize()
    for name, pred in masks.items():
        h = C.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(C.byref(h), words, mask(pred))
        assert rc == 0, rc
        st = torch.cuda.ExternalStream(h.value)
        with torch.cuda.stream(st):
            for _ in range(2):
                pipe.run(check_device=False)
            ts = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                pipe.run(marks=(a, b), check_device=False)
                ts.append((a, b))
            st.synchronize()
            ms = float(np.median([x.elapsed_time(y) for x, y in ts]))
            bits = pipe.plan.error_bits()
        n_on = sum(1 for c in range(ncu) if pred(c))
        print(f"{name:9s} CUs {n_on:3d}  kernel {ms:.3f} ms  ({ms * n_on / ncu:.3f} ms x CUs/all)"
              f"  err {bits}", flush=True)
        hip.hipStreamDestroy(h)




def where(masks_only=False):
    """Distinct (xcc, se, sh, cu) that run workgroups under each CU mask."""
    import torch
    hip = C.CDLL("libamdhip64.so")
    pl = C.CDLL(os.path.join(ROOT, "variants", "libcu_probe.so"))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    for name, pred in [("all", lambda c: True), ("even", lambda c: c % 2 == 0),
                       ("mod4_0", lambda c: c % 4 == 0), ("low_half", lambda c: c < ncu // 2),
                       ("bits0_31", lambda c: c < 32)]:
        m = [0] * words
        for c in range(ncu):
            if pred(c):
                m[c // 32] |= 1 << (c % 32)
        h = C.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(C.byref(h), words, (C.c_uint32 * words)(*m)) == 0
        out = torch.zeros(4096, dtype=torch.int32, device="cuda")
        assert pl.cu_probe(C.c_void_p(out.data_ptr()), 4096, 200, h) == 0
        hip.hipStreamSynchronize(h)
        v = out.cpu().numpy().astype(np.uint32)
        ids = set(v.tolist())
        xcc = sorted(set((x >> 16) for x in ids))
        print(f"{name:9s} mask bits {sum(bin(w).count('1') for w in m):3d}: {len(ids)} distinct CUs, "
              f"XCCs {xcc}, per-XCC {[sum(1 for x in ids if x >> 16 == q) for q in xcc]}", flush=True)
        hip.hipStreamDestroy(h)


def layout():
    """Mask bit -> hardware (xcc, se, sh, cu): one local index l at a time,
    bits 8l..8l+7 (one CU per XCC)."""
    import torch
    hip = C.CDLL("libamdhip64.so")
    pl = C.CDLL(os.path.join(ROOT, "variants", "libcu_probe.so"))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    for l in range(ncu // 8):
        m = [0] * words
        for c in range(8 * l, 8 * l + 8):
            m[c // 32] |= 1 << (c % 32)
        h = C.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(C.byref(h), words, (C.c_uint32 * words)(*m)) == 0
        out = torch.zeros(256, dtype=torch.int32, device="cuda")
        assert pl.cu_probe(C.c_void_p(out.data_ptr()), 256, 20, h) == 0
        hip.hipStreamSynchronize(h)
        ids = sorted(set(out.cpu().numpy().astype(np.uint32).tolist()))
        desc = [f"x{v >> 16}.se{(v >> 8) & 7}.sh{(v >> 4) & 1}.cu{v & 15}" for v in ids if v >> 16 == 0]
        print(f"l={l:2d}: {len(ids)} CUs; XCC0: {desc}", flush=True)
        hip.hipStreamDestroy(h)


if __name__ == "__main__":
    if "--where" in sys.argv:
        where()
    elif "--layout" in sys.argv:
        layout()
    else:
        main()

