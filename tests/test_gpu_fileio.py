"""GPU file ingest / egress (fileio.py): the device path
gives exactly what the host codec path gives — decoded floats bit-identical to
audio_io.read, and output files byte-identical to audio_io.write (same PCM_24
quantisation, same FLAC encoder)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mods():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import audio_io, fileio
    return torch, audio_io, fileio


@pytest.mark.parametrize("n,ch,sub", [(48000 * 7 + 11, 2, "PCM_24"), (44100 * 3, 1, "PCM_16"),
                                      (4096 * 300 + 5, 2, "PCM_24")])
def test_flac_read_device_matches_host(tmp_path, n, ch, sub):
    torch, audio_io, fileio = _mods()
    from tomatis_audio_processor_amd.synth import synth_stream
    x = synth_stream(17, n, ch, 48000)
    p = str(tmp_path / "a.flac")
    audio_io.write(p, x, 48000, "FLAC", sub)
    host, sr = audio_io.read(p)
    xd, n2, ch2, sr2 = fileio.read_device(p)
    assert (n2, ch2, sr2) == (n, ch, 48000)
    np.testing.assert_array_equal(xd.cpu().numpy().reshape(n, ch).view(np.uint32),
                                  host.view(np.uint32))


@pytest.mark.parametrize("n,ch", [(48000 * 5 + 3, 2), (4096 * 1024 * 2 + 4096 * 3 + 17, 2),
                                  (1000, 1)])
def test_flac_write_device_byte_identical(tmp_path, n, ch):
    torch, audio_io, fileio = _mods()
    rng = np.random.default_rng(n)
    y = (rng.standard_normal((n, ch)) * 0.4).astype(np.float32)
    y[::997] = 1.5           # clipped
    y[1::991] = -1.25
    y[2::983] = 0.5 / 8388607.0   # exact halfway cases of the rounding
    p1, p2 = str(tmp_path / "h.flac"), str(tmp_path / "d.flac")
    audio_io.write(p1, y, 44100, "FLAC", "PCM_24")
    yd = torch.from_numpy(y.reshape(-1)).cuda()
    written, is_flac = fileio.write_device(p2, yd, n, ch, 44100, log=lambda m: None)
    assert is_flac and written == p2
    assert open(p1, "rb").read() == open(p2, "rb").read()


def test_pcm_conversions_match_numpy():
    torch, audio_io, fileio = _mods()
    from tomatis_audio_processor_amd._lib import lib, ptr, stream_handle
    rng = np.random.default_rng(3)
    for bps in (16, 24, 32):
        v = rng.integers(-(1 << (bps - 1)), (1 << (bps - 1)) - 1, size=100003,
                         dtype=np.int64).astype(np.int32)
        vd = torch.from_numpy(v).cuda()
        out = torch.empty(len(v), dtype=torch.float32, device="cuda")
        assert lib().tomatis_pcm_to_float(ptr(vd), len(v), bps, ptr(out), stream_handle()) == 0
        ref = (v.astype(np.float64) / float(1 << (bps - 1))).astype(np.float32)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    f = (rng.standard_normal(100003) * 0.7).astype(np.float32)
    fd = torch.from_numpy(f).cuda()
    o = torch.empty(len(f), dtype=torch.int32, device="cuda")
    assert lib().tomatis_float_to_pcm(ptr(fd), len(f), 24, ptr(o), stream_handle()) == 0
    ref = np.clip(np.rint(f.astype(np.float64) * 8388607.0), -8388608, 8388607).astype(np.int32)
    np.testing.assert_array_equal(o.cpu().numpy(), ref)
