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
