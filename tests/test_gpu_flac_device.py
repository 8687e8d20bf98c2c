"""GPU: FLAC frames encoded on the device (csrc/tm_flacenc.hip) against the
host encoder (csrc/tm_flac.cpp, the format reference of this build's output
files, SURVEY.md §8 row f1 — the reference writes FLAC PCM_24 through
libsndfile, src/process_tomatis.py:242-251): the whole stream byte for byte,
and decoded back to the same integers.  Inputs cover every subframe kind and
stereo assignment the planner can pick: noise (VERBATIM / high-order FIXED),
tones (FIXED orders, Rice partitions), silence and DC (CONSTANT), identical
and opposite channels (side / mid), impulses (large quotients, Rice2
parameters), 8 / 16 / 20 / 24 bits, mono, short last blocks and streams
shorter than one block, and the 60-min C2 output."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mods():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import audio_io, fileio
    from tomatis_audio_processor_amd._lib import lib, ptr, stream_handle, check
    return torch, audio_io, fileio, (lib, ptr, stream_handle, check)


def _host_encode(audio_io, pcm, sr, bps):
    import ctypes as C
    h = audio_io._flac()
    out = C.POINTER(C.c_uint8)()
    ln = C.c_int64()
    n, ch = pcm.shape
    a = np.ascontiguousarray(pcm, np.int32)
    rc = h.tomatis_flac_encode(a.ctypes.data_as(C.c_void_p), n, ch, sr, bps, C.byref(out),
                               C.byref(ln))
    assert rc == 0
    b = bytes((C.c_uint8 * ln.value).from_address(C.addressof(out.contents)))
    h.tomatis_flac_free(out)
    return b


def _device_encode(torch, fileio, pcm, bps):
    n, ch = pcm.shape
    yi = torch.from_numpy(np.ascontiguousarray(pcm, np.int32).reshape(-1)).cuda()
    r = fileio._device_frames(yi, n, ch, bps)
    assert r is not None, "the device encoder declined"
    out, total, st = r
    return fileio._streaminfo_header(n, ch, 44100, bps, *st) + out[:total].cpu().numpy().tobytes()


def _signals(rng, n, bps):
    top = (1 << (bps - 1)) - 1
    t = np.arange(n)
    tone = (np.sin(2 * np.pi * 440 * t / 44100) * top * 0.6).astype(np.int64)
    noise = rng.integers(-top // 8, top // 8, n)
    imp = np.zeros(n, np.int64)
    imp[rng.integers(0, n, max(1, n // 997))] = top
    imp[rng.integers(0, n, max(1, n // 1499))] = -top - 1
    ramp = (np.linspace(-top, top, n)).astype(np.int64)
    cases = {
        "noise": np.stack([noise, rng.integers(-top, top, n)], 1),
        "tone_ident": np.stack([tone, tone], 1),
        "tone_opposite": np.stack([tone, np.clip(-tone, -top - 1, top)], 1),
        "tone_noise": np.stack([tone + noise // 64, tone - noise // 64], 1),
        "silence": np.zeros((n, 2), np.int64),
        "dc_and_tone": np.stack([np.full(n, top // 3), tone], 1),
        "impulses": np.stack([imp, tone // 4 + imp // 2], 1),
        "ramp_extremes": np.stack([ramp, np.clip(ramp[::-1], -top - 1, top)], 1),
        "alternating": np.stack([np.where(t % 2, top, -top - 1), np.where(t % 3, 1, -1)], 1),
    }
    return {k: np.clip(v, -top - 1, top).astype(np.int32) for k, v in cases.items()}


@pytest.mark.parametrize("bps", [24, 16, 20, 8])
@pytest.mark.parametrize("n", [4096 * 6 + 1234, 4096 * 3, 777, 1, 5])
def test_device_flac_bytes_equal_host(bps, n):
    torch, audio_io, fileio, _ = _mods()
    rng = np.random.default_rng(1000 * bps + n)
    for name, x in _signals(rng, n, bps).items():
        for ch in (2, 1):
            pcm = x[:, :ch]
            h = _host_encode(audio_io, pcm, 44100, bps)
            d = _device_encode(torch, fileio, pcm, bps)
            assert len(d) == len(h), (name, ch, len(d), len(h))
            if d != h:
                i = next(j for j in range(len(h)) if d[j] != h[j])
                pytest.fail(f"{name} ch={ch} bps={bps} n={n}: first byte difference at {i} "
                            f"of {len(h)}")


def test_device_flac_decodes_back():
    """The device stream decodes (host decoder: CRC-8 / CRC-16 verified per
    frame) to the integers it encoded."""
    torch, audio_io, fileio, _ = _mods()
    rng = np.random.default_rng(7)
    x = _signals(rng, 4096 * 9 + 99, 24)["tone_noise"]
    d = _device_encode(torch, fileio, x, 24)
    import ctypes as C
    h = audio_io._flac()
    buf = np.frombuffer(d, np.uint8)
    n = x.shape[0]
    pcm = np.zeros(n * 2, np.int32)
    got = C.c_int64()
    rc = h.tomatis_flac_decode(buf.ctypes.data_as(C.c_void_p), len(d),
                               pcm.ctypes.data_as(C.c_void_p), n, C.byref(got))
    assert rc == 0 and got.value == n
    assert np.array_equal(pcm.reshape(n, 2), x)


def test_device_flac_c2_output_equals_host_path():
    """The 60-min C2 output (PCM_24): the device-encoded stream equals the host
    encoder's (fileio's segment path) byte for byte."""
    torch, audio_io, fileio, _ = _mods()
    from tomatis_audio_processor_amd import engine as E
    sr, n = 44100, 3600 * 44100
    ss = E.StreamSet.synthetic(1, n, 2, sr, seed0=1000)
    pipe = E.GatePipeline(ss, gate_ui=50, n_fft=2048, hop=512)
    res = pipe.run()
    y = res.y[:n * 2]
    d = fileio.encode_flac_device(y, n, 2, sr, 24, device_encoder=True)
    h = fileio.encode_flac_device(y, n, 2, sr, 24, device_encoder=False)
    assert len(d) == len(h)
    assert d == h
