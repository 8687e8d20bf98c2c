"""Cycles per VALU instruction by operand VGPR banks and waves per SIMD
(diagnostic; tools/bank_probe.hip)."""
import ctypes as C
import os
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "variants", "libbank_probe.so"))
names = ["fma 3 banks", "fma 1 bank", "add 2 banks", "add 1 bank", "fmac 3 banks", "fmac 1 bank",
         "fmamk lit", "fma dep x4"]
iters = 200
per_iter = 256
for waves_per_simd in (1, 2, 3, 4):
    threads = 64 * 4 * waves_per_simd    # one block per CU: waves spread over 4 SIMDs
    blocks = 256
    row = []
    for k in range(8):
        out = torch.zeros(blocks * threads // 64, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            assert lib.bank_probe(k, C.c_void_p(out.data_ptr()), blocks, threads, iters, C.c_void_p(s)) == 0
        torch.cuda.synchronize()
        cyc = float(np.median(out.cpu().numpy())) * 1.0   # s_memtime: 100 MHz? shader clock on gfx950
        row.append(cyc / (iters * per_iter))
    print(f"{waves_per_simd} waves/SIMD: " + "  ".join(f"{n}: {c:.2f}" for n, c in zip(names, row)), flush=True)
