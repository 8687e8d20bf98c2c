"""Native FLAC codec (csrc/tm_flac.cpp, include/tomatis_flac.h).

* lossless round trips through the C encoder and decoder (bit depths 8..32,
  1..6 channels, empty / short / block-boundary lengths, constant blocks,
  full-scale extremes);
* the decoder against streams written by an INDEPENDENT pure-Python FLAC
  writer below, which emits what the C encoder never does (LPC subframes,
  wasted bits, escape-coded and Rice2 partitions, mid/side and side/right,
  variable-blocksize headers with 8-bit block-size and 16-bit sample-rate
  fields) — parity is against the format (RFC 9639), the integers are known;
* corruption detection (CRC-8 / CRC-16), and audio_io's FLAC PCM_24 files.
No external FLAC tool exists in the image, so interoperability with libFLAC
itself is not checked here ("parity unpinned" for that).
"""
import numpy as np
import pytest

from tomatis_audio_processor_amd import audio_io


def rt(pcm, sr, bps):
    blob = audio_io.flac_encode_int(pcm, sr, bps)
    out, sr2, bps2 = audio_io.flac_decode_int(blob)
    assert sr2 == sr and bps2 == bps
    return out, blob


@pytest.mark.parametrize("bps", [8, 12, 16, 20, 24, 32])
@pytest.mark.parametrize("ch", [1, 2, 6])
def test_roundtrip_random(bps, ch):
    rng = np.random.default_rng(bps * 10 + ch)
    lo, hi = -(1 << (bps - 1)), (1 << (bps - 1)) - 1
    for n in (0, 1, 15, 4095, 4096, 4097, 20000):
        x = rng.integers(lo, hi + 1, size=(n, ch), dtype=np.int64)
        if n > 100:  # some smooth content, a constant block, extremes
            t = np.arange(n)
            x[:, 0] = np.clip((np.sin(t * 0.01) * hi * 0.8).astype(np.int64), lo, hi)
            x[:min(n, 4096), -1] = 7 if ch > 1 else x[:min(n, 4096), -1]
            x[n // 2, :] = lo
            x[n // 2 + 1, :] = hi
        x = x.astype(np.int32)
        y, _ = rt(x, 48000, bps)
        assert y.shape == x.shape and np.array_equal(y, x)


def test_compresses_smooth_audio():
    t = np.arange(48000 * 2)
    x = (np.stack([np.sin(t * 0.013), np.sin(t * 0.013 + 0.1)], 1) * 4e6).astype(np.int32)
    y, blob = rt(x, 48000, 24)
    assert np.array_equal(y, x) and len(blob) < x.size * 3 * 0.5


def test_corruption_detected():
    rng = np.random.default_rng(1)
    x = rng.integers(-1000, 1000, size=(9000, 2)).astype(np.int32)
    blob = bytearray(audio_io.flac_encode_int(x, 44100, 16))
    for pos in (len(blob) // 2, len(blob) - 1, 42 + 3):
        b = bytearray(blob)
        b[pos] ^= 0x10
        with pytest.raises(audio_io.AudioFormatError):
            audio_io.flac_decode_int(bytes(b))
    with pytest.raises(audio_io.AudioFormatError):
        audio_io.flac_decode_int(b"RIFF" + bytes(60))


def _decode_bytes(blob, lo, hi, n, ch):
    """tomatis_flac_decode_bytes over bytes [lo, hi): (rc, s_lo, s_hi)."""
    import ctypes as C
    from tomatis_audio_processor_amd import fileio
    h = fileio._flac()
    buf = np.frombuffer(blob, np.uint8)
    pcm = np.zeros((n, ch), np.int32)
    a, b = C.c_int64(), C.c_int64()
    rc = h.tomatis_flac_decode_bytes(buf.ctypes.data, len(blob), lo, hi, pcm.ctypes.data, n,
                                     C.byref(a), C.byref(b))
    return rc, a.value, b.value


def _first_frame_at_or_after(blob, pos, n, ch):
    """Byte offset of the first frame (sync code + verified CRCs) at or after pos:
    decode_bytes over [q, q + 2) finds a frame iff one starts at q."""
    q = pos
    while True:
        q = blob.index(b"\xff", q)
        if blob[q + 1] & 0xFE == 0xF8:
            rc, a, b = _decode_bytes(blob, q, q + 2, n, ch)
            if rc == 0 and b > a:
                return q
        q += 1


@pytest.mark.parametrize("entry", ["decode", "decode_bytes"])
def test_corrupt_frame_at_thread_boundary(monkeypatch, entry):
    """A frame that fails its CRC right after a decoder thread's range start is
    skipped by that thread's sync search; the threads' sample ranges then leave
    a gap, which must be an error, not uninitialised samples."""
    import ctypes as C
    from tomatis_audio_processor_amd import fileio
    monkeypatch.setenv("TOMATIS_FLAC_THREADS", "4")
    rng = np.random.default_rng(5)
    n, ch = 1 << 21, 2
    x = rng.integers(-3000, 3000, size=(n, ch)).astype(np.int32)
    blob = audio_io.flac_encode_int(x, 44100, 16)
    first = int(fileio._flac().tomatis_flac_first_frame(blob, len(blob)))
    body = len(blob) - first
    assert body > 4 << 20            # 4 threads in both entry points
    y, _, _ = audio_io.flac_decode_int(blob)
    assert np.array_equal(y, x)      # intact: threads tile the stream
    rc, a, b = _decode_bytes(blob, first, len(blob), n, ch)
    assert (rc, a, b) == (0, 0, n)
    for t in (1, 2, 3):
        q = _first_frame_at_or_after(blob, first + body * t // 4, n, ch)
        bad = bytearray(blob)
        bad[q + 24] ^= 0x5A          # inside the frame: its CRC-16 fails
        if entry == "decode":
            with pytest.raises(audio_io.AudioFormatError):
                audio_io.flac_decode_int(bytes(bad))
        else:
            rc, a, b = _decode_bytes(bytes(bad), first, len(blob), n, ch)
            assert rc != 0, (t, a, b)


def test_audio_io_flac_pcm24(tmp_path):
    from tomatis_audio_processor_amd.synth import synth_stream
    x = synth_stream(9, 30011, 2, 48000)
    p = str(tmp_path / "a.flac")
    audio_io.write(p, x, 48000, "FLAC", "PCM_24")
    assert audio_io.info(p) == (48000, 2, 30011)
    y, sr = audio_io.read(p)
    q = str(tmp_path / "a.wav")
    audio_io.write(q, x, 48000, "WAV", "PCM_24")
    z, _ = audio_io.read(q)
    assert sr == 48000 and y.dtype == np.float32 and np.array_equal(y, z)  # same PCM_24 values
    path, is_flac = audio_io.write_with_fallback(str(tmp_path / "o.flac"), x, 48000,
                                                 log=lambda m: None)
    assert is_flac and path.endswith("o.flac")


# ---------------------------------------------------------------------------
# independent pure-Python FLAC writer (RFC 9639 grammar)
# ---------------------------------------------------------------------------
class Bits:
    def __init__(self):
        self.b = []

    def put(self, v, n):
        for i in range(n - 1, -1, -1):
            self.b.append((v >> i) & 1)

    def sput(self, v, n):
        self.put(v & ((1 << n) - 1), n)

    def unary(self, q):
        self.b += [0] * q + [1]

    def align(self):
        while len(self.b) % 8:
            self.b.append(0)

    def tobytes(self):
        assert len(self.b) % 8 == 0
        return bytes(int("".join(map(str, self.b[i:i + 8])), 2) for i in range(0, len(self.b), 8))


def crc8(data):
    c = 0
    for x in data:
        c ^= x
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data):
    c = 0
    for x in data:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def rice_part(w, vals, k):
    for r in vals:
        u = (r << 1) if r >= 0 else ((-r) << 1) - 1
        w.unary(u >> k)
        w.put(u & ((1 << k) - 1), k)


def lpc_subframe(w, s, bps, coefs, prec, shift, wasted=0, method=0, escape_first=True):
    s = [v >> wasted for v in s]
    sb = bps - wasted
    order = len(coefs)
    w.put(0, 1)
    w.put(0x20 | (order - 1), 6)
    if wasted:
        w.put(1, 1)
        w.unary(wasted - 1)
    else:
        w.put(0, 1)
    for i in range(order):
        w.sput(s[i], sb)
    w.put(prec - 1, 4)
    w.sput(shift, 5)
    for c in coefs:
        w.sput(c, prec)
    res = [s[t] - (sum(coefs[j] * s[t - 1 - j] for j in range(order)) >> shift)
           for t in range(order, len(s))]
    n = len(s)
    w.put(method, 2)
    w.put(1, 4)  # partition order 1
    half = n // 2
    p0, p1 = res[:half - order], res[half - order:]
    if escape_first:
        nb = max(1, max(abs(v) for v in p0).bit_length() + 1)
        w.put(31 if method else 15, 5 if method else 4)
        w.put(nb, 5)
        for v in p0:
            w.sput(v, nb)
    else:
        w.put(3, 5 if method else 4)
        rice_part(w, p0, 3)
    k = 18 if method else 5
    w.put(k, 5 if method else 4)
    rice_part(w, p1, k)


def py_flac(frames, sr, bps, assign):
    """frames: list of [n, 2] int arrays (stereo)."""
    out = bytearray(b"fLaC")
    si = Bits()
    si.put(16, 16); si.put(4096, 16); si.put(0, 24); si.put(0, 24)
    si.put(sr, 20); si.put(1, 3); si.put(bps - 1, 5)
    si.put(sum(len(f) for f in frames), 36)
    si.put(0, 128)
    out += bytes([0x80, 0, 0, 34]) + si.tobytes()
    pos = 0
    for f in frames:
        n = len(f)
        L, R = [int(v) for v in f[:, 0]], [int(v) for v in f[:, 1]]
        if assign == 10:
            chans = [[(a + b) >> 1 for a, b in zip(L, R)], [a - b for a, b in zip(L, R)]]
            sbs = [bps, bps + 1]
        else:  # 9: side/right
            chans = [[a - b for a, b in zip(L, R)], R]
            sbs = [bps + 1, bps]
        w = Bits()
        w.put(0x3FFE, 14); w.put(0, 1); w.put(1, 1)  # variable blocksize
        w.put(6, 4)                                  # 8-bit blocksize-1 at header end
        w.put(13, 4)                                 # 16-bit sample rate in Hz
        w.put(assign, 4); w.put(6 if bps == 24 else 4, 3); w.put(0, 1)
        v = pos                                      # UTF-8 coded sample number
        if v < 0x80:
            w.put(v, 8)
        else:
            nb = 2
            while v >= (1 << (5 * nb + 1)):
                nb += 1
            w.put(((0xFF00 >> nb) & 0xFF) | (v >> (6 * (nb - 1))), 8)
            for i in range(nb - 2, -1, -1):
                w.put(0x80 | ((v >> (6 * i)) & 0x3F), 8)
        w.put(n - 1, 8)
        w.put(sr, 16)
        w.put(crc8(w.tobytes()), 8)
        for ci, (c, sb) in enumerate(zip(chans, sbs)):
            wasted = 2 if ci == 1 and assign == 10 else 0
            lpc_subframe(w, c, sb, coefs=[1800, -800], prec=12, shift=10, wasted=wasted,
                         method=ci % 2, escape_first=(pos // n) % 2 == 0)
        w.align()
        fb = w.tobytes()
        out += fb + crc16(fb).to_bytes(2, "big")
        pos += n
    return bytes(out)


@pytest.mark.parametrize("assign", [9, 10])
def test_decoder_vs_independent_writer(assign):
    rng = np.random.default_rng(assign)
    bps = 24
    frames = []
    for n in (256, 200, 256):
        t = np.arange(n)
        base = (np.sin(t * 0.05) * 3e6).astype(np.int64)
        L = base + rng.integers(-50, 50, n)
        R = base // 2 + rng.integers(-50, 50, n)
        if assign == 10:  # side multiple of 4 and mid even -> wasted bits on the side channel
            R = L - 4 * ((L - R) // 4)
        frames.append(np.stack([L, R], 1))
    blob = py_flac(frames, 48000, bps, assign)
    pcm, sr, b = audio_io.flac_decode_int(blob)
    assert (sr, b) == (48000, bps)
    assert np.array_equal(pcm, np.concatenate(frames).astype(np.int32))


def test_threaded_decode_and_encode_exact(monkeypatch):
    """Block ranges (encoder) and byte ranges with sync search (decoder) on
    several host threads give the same stream / samples as one thread."""
    rng = np.random.default_rng(11)
    n = 48000 * 40
    x = (rng.standard_normal((n, 2)) * 2e5).astype(np.int32)
    monkeypatch.setenv("TOMATIS_FLAC_THREADS", "1")
    b1 = audio_io.flac_encode_int(x, 48000, 24)
    y1, _, _ = audio_io.flac_decode_int(b1)
    monkeypatch.setenv("TOMATIS_FLAC_THREADS", "5")
    b5 = audio_io.flac_encode_int(x, 48000, 24)
    assert b5 == b1 and len(b1) > 5 * (1 << 20)
    y5, _, _ = audio_io.flac_decode_int(b5)
    assert np.array_equal(y1, x) and np.array_equal(y5, x)


def _zero_total(blob: bytes) -> bytes:
    """STREAMINFO total samples (36 bits at byte 8+13.5) set to 0 = unknown."""
    b = bytearray(blob)
    b[8 + 13] &= 0xF0
    b[8 + 14:8 + 18] = b"\0\0\0\0"
    return bytes(b)


def test_unknown_total_decodes_exactly(tmp_path):
    """A STREAMINFO total of 0 ("unknown", legal; written by encoders that
    stream to a pipe) decodes to the exact samples, through audio_io too."""
    rng = np.random.default_rng(5)
    x = rng.integers(-(1 << 23), 1 << 23, size=(50001, 2)).astype(np.int32)
    blob = _zero_total(audio_io.flac_encode_int(x, 48000, 24))
    assert audio_io.flac_info_bytes(blob)[3] == 0
    y, sr, bps = audio_io.flac_decode_int(blob)
    assert np.array_equal(y, x)
    p = tmp_path / "u.flac"
    p.write_bytes(blob)
    assert audio_io.info(str(p)) == (48000, 2, 50001)
    z, _ = audio_io.read(str(p))
    assert z.shape == (50001, 2)


@pytest.mark.parametrize("unknown_total", [False, True])
def test_id3_tags_are_skipped(tmp_path, unknown_total):
    """A leading ID3v2 tag and a trailing 128-byte ID3v1 'TAG' block (both
    accepted by libsndfile) do not stop the decode or change the samples."""
    rng = np.random.default_rng(6)
    x = rng.integers(-30000, 30000, size=(30000, 1)).astype(np.int32)
    blob = audio_io.flac_encode_int(x, 44100, 16)
    if unknown_total:
        blob = _zero_total(blob)
    body = b"\x00" * 300
    sz = len(body)
    id3 = b"ID3\x04\x00\x00" + bytes([(sz >> 21) & 0x7F, (sz >> 14) & 0x7F, (sz >> 7) & 0x7F,
                                      sz & 0x7F]) + body
    tag = b"TAG" + b"title".ljust(30, b"\0") + bytes(95)
    p = tmp_path / "t.flac"
    p.write_bytes(id3 + blob + tag)
    assert audio_io.info(str(p)) == (44100, 1, 30000)
    z, sr = audio_io.read(str(p))
    assert sr == 44100 and np.array_equal(np.rint(z * 32768.0).astype(np.int32), x)
    y, _, _ = audio_io.flac_decode_int(blob + tag)
    assert np.array_equal(y, x)


def test_corrupt_last_frame_of_unknown_total_is_an_error():
    rng = np.random.default_rng(7)
    x = rng.integers(-1000, 1000, size=(9000, 2)).astype(np.int32)
    b = bytearray(_zero_total(audio_io.flac_encode_int(x, 44100, 16)))
    b[len(b) - 1] ^= 0x10          # frame CRC-16 of a frame that starts with a sync code
    with pytest.raises(audio_io.AudioFormatError):
        audio_io.flac_decode_int(bytes(b))


def test_streaming_encoder_byte_identical():
    """Segments pushed to the streaming encoder (whole 4096-blocks, short last
    push) give exactly the whole-buffer stream (fileio egress)."""
    import ctypes as C
    from tomatis_audio_processor_amd import fileio
    h = fileio._flac()
    rng = np.random.default_rng(8)
    for n, ch, segs in ((4096 * 10 + 123, 2, [4096 * 3, 4096 * 3, 4096 * 4 + 123]),
                        (4096 * 5, 1, [4096 * 5]), (77, 2, [77])):
        x = rng.integers(-(1 << 23), 1 << 23, size=(n, ch)).astype(np.int32)
        whole = audio_io.flac_encode_int(x, 48000, 24)
        enc = C.c_void_p()
        assert h.tomatis_flac_enc_open(ch, 48000, 24, C.byref(enc)) == 0
        a = 0
        for m in segs:
            seg = np.ascontiguousarray(x[a:a + m])
            assert h.tomatis_flac_enc_push(enc, seg.ctypes.data, m) == 0
            a += m
        out = C.POINTER(C.c_uint8)()
        ln = C.c_int64()
        assert h.tomatis_flac_enc_finish(enc, C.byref(out), C.byref(ln)) == 0
        blob = C.string_at(out, ln.value)
        h.tomatis_flac_free(out)
        h.tomatis_flac_enc_close(enc)
        assert blob == whole


def test_byte_range_decode_reassembles():
    """Consecutive byte ranges decode to consecutive sample ranges covering the
    stream (fileio ingest), for several range counts."""
    import ctypes as C
    from tomatis_audio_processor_amd import fileio
    h = fileio._flac()
    rng = np.random.default_rng(9)
    n, ch = 4096 * 37 + 1000, 2
    x = rng.integers(-30000, 30000, size=(n, ch)).astype(np.int32)
    blob = audio_io.flac_encode_int(x, 44100, 16)
    first = h.tomatis_flac_first_frame(blob, len(blob))
    assert first == 42
    for K in (1, 3, 8, 50):
        pcm = np.zeros((n, ch), np.int32)
        edges = np.linspace(first, len(blob), K + 1).astype(np.int64)
        got = 0
        lo, hi = C.c_int64(), C.c_int64()
        for k in range(K):
            assert h.tomatis_flac_decode_bytes(blob, len(blob), int(edges[k]), int(edges[k + 1]),
                                               pcm.ctypes.data, n, C.byref(lo), C.byref(hi)) == 0
            if hi.value > lo.value:
                assert lo.value == got
                got = hi.value
        assert got == n and np.array_equal(pcm, x)


def test_streaming_encoder_take_and_header():
    """take() drains the frame bytes as they are encoded; header + the drained
    parts == the whole-buffer stream (fileio's streamed file write)."""
    import ctypes as C
    from tomatis_audio_processor_amd import fileio
    h = fileio._flac()
    rng = np.random.default_rng(10)
    n, ch = 4096 * 9 + 5, 2
    x = rng.integers(-(1 << 23), 1 << 23, size=(n, ch)).astype(np.int32)
    whole = audio_io.flac_encode_int(x, 96000, 24)
    enc = C.c_void_p()
    assert h.tomatis_flac_enc_open(ch, 96000, 24, C.byref(enc)) == 0
    parts = []
    out = C.POINTER(C.c_uint8)()
    ln = C.c_int64()
    for a, b in ((0, 4096 * 4), (4096 * 4, 4096 * 8), (4096 * 8, n)):
        seg = np.ascontiguousarray(x[a:b])
        assert h.tomatis_flac_enc_push(enc, seg.ctypes.data, b - a) == 0
        assert h.tomatis_flac_enc_take(enc, C.byref(out), C.byref(ln)) == 0
        parts.append(C.string_at(out, ln.value))
        h.tomatis_flac_free(out)
    hdr = (C.c_uint8 * 42)()
    assert h.tomatis_flac_enc_header(enc, hdr) == 0
    h.tomatis_flac_enc_close(enc)
    assert bytes(hdr) + b"".join(parts) == whole
