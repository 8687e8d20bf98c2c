"""Cycles per instruction by loop-body code size and waves per SIMD
(diagnostic; tools/fetch_probe.hip)."""
import ctypes as C
import os
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "variants", "libfetch_probe.so"))
kinds = [("add 64 (256 B)", 64, 256), ("add 1024 (4 KB)", 1024, 16), ("add 4096 (16 KB)", 4096, 4),
         ("fma 64 (512 B)", 64, 256), ("fma 1024 (8 KB)", 1024, 16), ("fma 4096 (32 KB)", 4096, 4)]
for wps in (1, 2, 3, 4):
    threads = 64 * 4 * wps
    row = []
    for k, (name, n, rep) in enumerate(kinds):
        iters = 20 * rep
        out = torch.zeros(256 * threads // 64, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            assert lib.fetch_probe(k, C.c_void_p(out.data_ptr()), 256, threads, iters, C.c_void_p(s)) == 0
        torch.cuda.synchronize()
        row.append(float(np.median(out.cpu().numpy())) / (iters * n))
    print(f"{wps} waves/SIMD: " + "  ".join(f"{kn[0]}: {c:.2f}" for kn, c in zip(kinds, row)), flush=True)
