"""GPU: FLAC frames decoded on the device (csrc/tm_flacdec.hip, the ingest of
the file path; the reference reads its input through libsndfile,
src/process_tomatis.py:225-235) against the host decoder (csrc/tm_flac.cpp):
the same integers.  Streams from this build's encoder (every subframe kind
and stereo assignment it picks, 4-24 bits, mono / stereo, short last blocks)
and from the independent Python writer of test_flac_codec.py (LPC subframes,
escape partitions, Rice2, wasted bits, side/right and mid/side, variable
block size, 16-bit sample-rate headers).  A stream with trailing non-audio
bytes (an ID3v1 tag) does not chain to the end of the file and goes to the
host decoder, with the same result."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mods():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import audio_io, fileio
    return torch, audio_io, fileio


def _device_read(fileio, path):
    tm = fileio.Timer()
    x, n, ch, sr = fileio.read_device(str(path), tm)
    return x, n, ch, sr, ("decode" in tm)


def _check(torch, audio_io, fileio, tmp_path, blob, name, expect_device=True):
    p = tmp_path / f"{name}.flac"
    p.write_bytes(blob)
    x, n, ch, sr, on_dev = _device_read(fileio, p)
    ref, sr2, bps = audio_io.flac_decode_int(blob)
    assert on_dev == expect_device, name
    assert (n, ch, sr) == (ref.shape[0], ref.shape[1], sr2)
    # the device's int -> float rule is the host's (v / 2^(bps-1)); compare floats
    want = (ref.astype(np.float64) / float(1 << (bps - 1))).astype(np.float32)
    got = x[:n * ch].cpu().numpy().reshape(n, ch)
    assert np.array_equal(got, want), name


@pytest.mark.parametrize("bps", [24, 20, 16, 12, 8, 4])
def test_device_decode_own_encoder(tmp_path, bps):
    torch, audio_io, fileio = _mods()
    from tests.test_gpu_flac_device import _signals
    rng = np.random.default_rng(bps)
    for n in (4096 * 7 + 555, 4096, 100):
        for name, x in _signals(rng, n, bps).items():
            for ch in (2, 1):
                blob = audio_io.flac_encode_int(np.ascontiguousarray(x[:, :ch]), 44100, bps)
                _check(torch, audio_io, fileio, tmp_path, blob, f"{name}_{n}_{ch}_{bps}")


@pytest.mark.parametrize("assign", [9, 10])
def test_device_decode_independent_writer(tmp_path, assign):
    torch, audio_io, fileio = _mods()
    from tests.test_flac_codec import py_flac
    rng = np.random.default_rng(100 + assign)
    frames = []
    for n in (256, 200, 256, 128, 256, 178):  # even: partition order 1
        t = np.arange(n)
        base = (np.sin(t * 0.05) * 3e6).astype(np.int64)
        L = base + rng.integers(-50, 50, n)
        R = base // 2 + rng.integers(-50, 50, n)
        if assign == 10:
            R = L - 4 * ((L - R) // 4)
        frames.append(np.stack([L, R], 1))
    blob = py_flac(frames, 48000, 24, assign)
    _check(torch, audio_io, fileio, tmp_path, blob, f"indep_{assign}")


def _set_total(blob, n):
    """STREAMINFO's 36-bit total-samples field (bytes 18..25 hold sample rate,
    channels, bits and the total) set to n."""
    b = bytearray(blob)
    v = int.from_bytes(b[18:26], "big")
    b[18:26] = ((v & ~((1 << 36) - 1)) | n).to_bytes(8, "big")
    return bytes(b)


@pytest.mark.parametrize("total", [700, 456, 300])
def test_device_decode_short_total_falls_back(tmp_path, total):
    """STREAMINFO declaring fewer samples than the LPC frames hold: the frames
    past the total (or straddling it) cannot be decoded whole into the PCM
    buffer, so the device declines (no read outside the frames' written
    samples) and the host decoder's truncated result is returned."""
    torch, audio_io, fileio = _mods()
    from tests.test_flac_codec import py_flac
    rng = np.random.default_rng(5)
    frames = []
    for n in (256, 200, 256, 128):
        t = np.arange(n)
        base = (np.sin(t * 0.05) * 3e6).astype(np.int64)
        frames.append(np.stack([base + rng.integers(-50, 50, n),
                                base // 2 + rng.integers(-50, 50, n)], 1))
    blob = _set_total(py_flac(frames, 48000, 24, 9), total)
    _check(torch, audio_io, fileio, tmp_path, blob, f"short_{total}", expect_device=False)


def test_device_decode_trailing_tag_falls_back(tmp_path):
    torch, audio_io, fileio = _mods()
    rng = np.random.default_rng(3)
    x = rng.integers(-(1 << 20), 1 << 20, size=(30000, 2)).astype(np.int32)
    blob = audio_io.flac_encode_int(x, 44100, 24) + b"TAG" + bytes(125)
    _check(torch, audio_io, fileio, tmp_path, blob, "tagged", expect_device=False)


def test_device_decode_c2_file(tmp_path):
    """The bench's 60-min C2 input file: device and host decodes agree."""
    torch, audio_io, fileio = _mods()
    from tomatis_audio_processor_amd import engine
    sr, n = 44100, 3600 * 44100
    ss = engine.StreamSet.synthetic(1, n, 2, sr, seed0=1000)
    blob = fileio.encode_flac_device(ss.x, n, 2, sr, 24)
    p = tmp_path / "c2.flac"
    p.write_bytes(blob)
    del blob
    x, n2, ch, sr2, on_dev = _device_read(fileio, p)
    assert on_dev and n2 == n
    ref, _, bps = audio_io.flac_decode_int(p.read_bytes())
    want = torch.from_numpy((ref.reshape(-1).astype(np.float64) /
                             float(1 << (bps - 1))).astype(np.float32)).cuda()
    assert torch.equal(x[:n * 2], want)



def test_device_decode_corrupted_bytes(tmp_path):
    """Single-byte corruptions anywhere in a stream (metadata, frame headers,
    subframe headers, residuals, CRCs): the device kernels must stay inside the
    file's bytes, and the device read must return what the host decoder
    returns (or raise what it raises) — a corrupted frame fails its CRC-8 /
    CRC-16 or breaks the frame chain, and the read goes to the host decoder."""
    torch, audio_io, fileio = _mods()
    from tests.test_gpu_flac_device import _signals
    rng = np.random.default_rng(77)
    from tests.test_flac_codec import py_flac
    x = _signals(rng, 4096 * 3 + 301, 24)["tone_noise"]
    own = audio_io.flac_encode_int(np.ascontiguousarray(x), 44100, 24)
    frames = []
    for n in (256, 200, 256, 128):  # LPC, escapes, Rice2, wasted bits
        t = np.arange(n)
        base = (np.sin(t * 0.05) * 3e6).astype(np.int64)
        L = base + rng.integers(-50, 50, n)
        frames.append(np.stack([L, L - 4 * ((L - base // 2) // 4)], 1))
    indep = py_flac(frames, 48000, 24, 10)
    p = tmp_path / "fz.flac"
    for t in range(160):
        blob = own if t % 2 else indep
        b = bytearray(blob)
        pos = int(rng.integers(0, len(b))) if t % 4 else int(rng.integers(0, min(len(b), 200)))
        b[pos] ^= int(rng.integers(1, 256))
        p.write_bytes(bytes(b))
        try:
            ref, sr2, bps = audio_io.flac_decode_int(bytes(b))
            ref_err = None
        except Exception as e:  # noqa: BLE001 - the host's verdict is the reference
            ref_err = type(e)
        try:
            got, n, ch, sr = fileio.read_device(str(p), fileio.Timer())
            got_err = None
        except Exception as e:  # noqa: BLE001
            got_err = type(e)
        torch.cuda.synchronize()
        if ref_err is not None:
            assert got_err is not None, (t, pos)
            continue
        assert got_err is None, (t, pos, got_err)
        want = (ref.astype(np.float64) / float(1 << (bps - 1))).astype(np.float32)
        assert (n, ch) == ref.shape, (t, pos)
        assert np.array_equal(got[:n * ch].cpu().numpy().reshape(n, ch), want), (t, pos)
