"""debug: two-round limiter on ragged batches under the fused gate vs the one-round two-pass chain"""
import numpy as np, torch
from tomatis_audio_processor_amd import engine as E
from tomatis_audio_processor_amd.synth import synth_stream
sr = 44100
xs = [synth_stream(31 + i, n, 2, sr) for i, n in
      enumerate([sr * 70 + 13, 1500, sr * 3 + 1, 2048, sr * 41 + 999])]
ss = E.StreamSet.from_arrays(xs, sr)
ref = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512, fused_levels=False)
ref.run(); y0 = ref.y.clone()
res = ref.result()
prev = None
for rep in range(3):
    p = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512, fused_levels=True)
    p.plan.set_limiter_rounds(2)
    p.run()
    d = (p.y != y0).nonzero().flatten().cpu().numpy()
    print("rep", rep, "ndiff", len(d), "same as prev", prev is not None and np.array_equal(prev, d))
    prev = d
    a = res.out_offs[0]
    yy = p.y.cpu().numpy(); zz = y0.cpu().numpy()
    for bl in (3, 4, 100, 1000):
        s0 = a + bl * 1024
        idx = np.nonzero(yy[s0:s0 + 1024] != zz[s0:s0 + 1024])[0]
        print(f"  block {bl}: float idx {idx.tolist()}")
        if len(idx):
            print("     y", yy[s0 + idx][:8], "ref", zz[s0 + idx][:8], "ratio", (yy[s0 + idx] / zz[s0 + idx])[:8])
