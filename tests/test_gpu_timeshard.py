"""GPU: one stream time-sharded over W ranks (emulated in one process, the two
exchanges done on the host) is bit-identical to the unsharded run: samples,
gate states and limiter chunk peaks (timeshard.py)."""
import numpy as np
import pytest

from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine, timeshard
    return torch, engine, timeshard


@pytest.mark.parametrize("secs,sr,n_fft,hop,world", [(150, 44100, 2048, 512, 2),
                                                     (150, 44100, 2048, 512, 8),
                                                     (97, 48000, 4096, 1024, 3),
                                                     (300, 48000, 4096, 2048, 4)])
def test_timeshard_bit_identical(secs, sr, n_fft, hop, world):
    torch, E, T = _engine()
    N = sr * secs + 123
    x = synth_stream(31, N, 2, sr)
    params = dict(gate_ui=50, n_fft=n_fft, hop=hop)
    ss = E.StreamSet.from_arrays([x], sr)
    pipe = E.GatePipeline(ss, **params)
    res = pipe.run()
    torch.cuda.synchronize()
    y_ref, st_ref, pk_ref = res.output(0), res.stream_states(0), res.stream_peaks(0)
    y, st, pk = T.run_emulated(x, sr, world, **params)
    assert np.array_equal(st, st_ref)
    assert pk.tobytes() == pk_ref.tobytes()
    assert y.shape == y_ref.shape
    assert y.tobytes() == y_ref.tobytes()


@pytest.mark.parametrize("secs,sr,n_fft,hop,world", [(150, 44100, 2048, 512, 4),
                                                     (97, 48000, 4096, 1024, 3)])
def test_timeshard_vs_oracle(secs, sr, n_fft, hop, world):
    """The concatenated shards against the oracle directly (not only against the
    unsharded GPU run): states bit-exact, chunk scales and masked samples."""
    torch, E, T = _engine()
    from oracle import tomatis_oracle as orc
    N = sr * secs + 777
    x = synth_stream(41, N, 2, sr)
    params = dict(gate_ui=50, n_fft=n_fft, hop=hop)
    y, st, pk = T.run_emulated(x, sr, world, **params)
    ref = orc.process_standard(x, sr, **params)
    assert np.array_equal(st, ref["states"])
    m = ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3
    b = ref["bounds"]
    assert len(pk) == len(b) - 1
    for c in range(len(b) - 1):
        lo, hi = max(0, int(b[c])), min(N, int(b[c + 1]))
        gs = float(np.float32(0.999) / np.float32(pk[c])) if pk[c] > 0.999 else 1.0
        rs = ref["scales"][c] or 1.0
        mm = m[lo:hi]
        err = np.abs(y[lo:hi][mm] / gs - ref["y"][lo:hi][mm] / rs) * min(gs, rs)
        assert err.max() <= 1e-4
        if c < len(b) - 2:   # interior chunks: no ill-conditioned sample in them
            assert abs(gs / rs - 1) <= 5e-5
