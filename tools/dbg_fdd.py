"""debug: the first own-encoder stream whose device decode differs"""
import numpy as np, torch, tempfile, os
from tomatis_audio_processor_amd import audio_io, fileio
from tests.test_gpu_flac_device import _signals
bps = 8
rng = np.random.default_rng(bps)
d = tempfile.mkdtemp()
for n in (4096 * 7 + 555, 4096, 100):
    for name, x in _signals(rng, n, bps).items():
        for ch in (2, 1):
            pcm = np.ascontiguousarray(x[:, :ch])
            blob = audio_io.flac_encode_int(pcm, 44100, bps)
            p = os.path.join(d, "a.flac")
            open(p, "wb").write(blob)
            tm = fileio.Timer()
            xx, nn, cc, sr = fileio.read_device(p, tm)
            got = np.rint(xx[:nn * cc].cpu().numpy() * 128).astype(np.int64).reshape(nn, cc)
            bad = np.nonzero((got != pcm).any(1))[0]
            if len(bad):
                print(name, n, ch, "device" if "decode" in tm else "host", "bad samples", len(bad),
                      "first", bad[:10], "blocks", sorted(set((bad // 4096).tolist()))[:10])
                b0 = bad[0]
                print("  got", got[b0:b0 + 8, 0], "want", pcm[b0:b0 + 8, 0])
                blk = b0 // 4096
                print("  block samples want[0:16]", pcm[blk * 4096: blk * 4096 + 16, 0])
                print("  nonzero in block", np.count_nonzero(pcm[blk*4096:(blk+1)*4096, 0]))
                raise SystemExit
print("all equal")
