"""Audio file I/O for the drop-in CLIs (codec boundary).

``soundfile`` (libsndfile) is used when importable, exactly like the
reference (FLAC PCM_24 output).  The build image has no libsndfile, so the
package carries its own codecs: FLAC through the native host library
``libtomatis_flac.so`` (``csrc/tm_flac.cpp``, C ABI ``include/tomatis_flac.h``:
lossless encode of PCM 8..32, decode of any FLAC stream with CRC checks) and a
built-in RIFF/WAVE codec (PCM 8/16/24/32 and IEEE float 32/64 input, PCM_24 /
PCM_16 / float output).  If FLAC encoding fails, the processors take the
reference's own fallback branch: write ``out_path.replace(".flac", ".wav")`` as
WAV PCM_24 (src/process_tomatis.py:242-251).

Sample conversion follows libsndfile's normalisation: int -> float divides by
2^(bits-1); float -> PCM_24 multiplies by 0x7FFFFF and rounds to nearest.
"""
from __future__ import annotations

import ctypes as C
import os
import struct

import numpy as np

try:  # pragma: no cover - not installed in this image
    import soundfile as _sf  # type: ignore
except Exception:  # pragma: no cover
    _sf = None

WAVE_FORMAT_PCM = 0x0001
WAVE_FORMAT_IEEE_FLOAT = 0x0003
WAVE_FORMAT_EXTENSIBLE = 0xFFFE


class AudioFormatError(RuntimeError):
    pass


def have_soundfile() -> bool:
    return _sf is not None


# ---------------------------------------------------------------------------
# native FLAC (libtomatis_flac.so)
# ---------------------------------------------------------------------------
_FLAC = None
FLAC_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtomatis_flac.so")


def _flac():
    global _FLAC
    if _FLAC is None:
        if not os.path.exists(FLAC_LIB):
            raise AudioFormatError(f"{FLAC_LIB} not built (tomatis_audio_processor_amd.build"
                                   ".build_flac)")
        h = C.CDLL(FLAC_LIB)
        P, I32, I64 = C.c_void_p, C.c_int32, C.c_int64
        h.tomatis_flac_encode.argtypes = [P, I64, I32, I32, I32, C.POINTER(C.POINTER(C.c_uint8)),
                                          C.POINTER(I64)]
        h.tomatis_flac_free.argtypes = [C.POINTER(C.c_uint8)]
        h.tomatis_flac_free.restype = None
        h.tomatis_flac_info.argtypes = [P, I64, C.POINTER(I32), C.POINTER(I32), C.POINTER(I32),
                                        C.POINTER(I64)]
        h.tomatis_flac_decode.argtypes = [P, I64, P, I64, C.POINTER(I64)]
        _FLAC = h
    return _FLAC


_FLAC_ERR = {-1: "bad argument", -2: "not a FLAC stream / unsupported", -3: "CRC mismatch",
             -4: "out of memory"}


def flac_encode_int(pcm: np.ndarray, sr: int, bps: int) -> bytes:
    """Lossless FLAC stream of int32 PCM [frames, ch] at ``bps`` bits."""
    pcm = np.ascontiguousarray(pcm, np.int32)
    if pcm.ndim == 1:
        pcm = pcm[:, None]
    out = C.POINTER(C.c_uint8)()
    n = C.c_int64()
    rc = _flac().tomatis_flac_encode(pcm.ctypes.data, pcm.shape[0], pcm.shape[1], sr, bps,
                                     C.byref(out), C.byref(n))
    if rc:
        raise AudioFormatError(f"FLAC encode failed: {_FLAC_ERR.get(rc, rc)}")
    try:
        return C.string_at(out, n.value)
    finally:
        _flac().tomatis_flac_free(out)


def flac_info_bytes(data: bytes):
    sr, ch, bps, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    rc = _flac().tomatis_flac_info(data, len(data), C.byref(sr), C.byref(ch), C.byref(bps),
                                   C.byref(n))
    if rc:
        raise AudioFormatError(f"FLAC: {_FLAC_ERR.get(rc, rc)}")
    return sr.value, ch.value, bps.value, n.value


def flac_count_frames(data: bytes) -> int:
    """Decoded length of a FLAC stream (decodes without storing samples)."""
    got = C.c_int64()
    rc = _flac().tomatis_flac_decode(data, len(data), None, 0, C.byref(got))
    if rc:
        raise AudioFormatError(f"FLAC decode failed: {_FLAC_ERR.get(rc, rc)}")
    return got.value


def flac_decode_int(data: bytes):
    """(int32 PCM [frames, ch], sr, bps) of an in-memory FLAC stream.

    A STREAMINFO total of 0 means "unknown" in the FLAC format (encoders
    writing to a pipe leave it so); the length is then counted first."""
    sr, ch, bps, n = flac_info_bytes(data)
    if n == 0:
        n = flac_count_frames(data)
    pcm = np.empty((n, ch), np.int32)
    got = C.c_int64()
    rc = _flac().tomatis_flac_decode(data, len(data), pcm.ctypes.data, n, C.byref(got))
    if rc:
        raise AudioFormatError(f"FLAC decode failed: {_FLAC_ERR.get(rc, rc)}")
    return pcm[:got.value], sr, bps


def id3v2_size(head: bytes) -> int:
    """Bytes taken by a leading ID3v2 tag (0 if none): 10-byte header, syncsafe
    size, plus a 10-byte footer when flagged.  libsndfile skips it too."""
    if len(head) < 10 or head[:3] != b"ID3":
        return 0
    sz = 0
    for b in head[6:10]:
        sz = (sz << 7) | (b & 0x7F)
    return 10 + sz + (10 if head[5] & 0x10 else 0)


def _flac_bytes(path: str) -> bytes:
    with open(path, "rb") as f:
        data = f.read()
    return data[id3v2_size(data[:10]):]


def _read_flac(path: str):
    pcm, sr, bps = flac_decode_int(_flac_bytes(path))
    # libsndfile's int -> float normalisation: v / 2^(bps-1)
    x = (pcm.astype(np.float64) / float(1 << (bps - 1))).astype(np.float32)
    return np.ascontiguousarray(x), sr


def _write_flac(path: str, data: np.ndarray, sr: int, subtype: str = "PCM_24"):
    st = subtype.upper()
    if st == "PCM_24":
        v = np.clip(np.rint(np.asarray(data, np.float64) * 8388607.0), -8388608, 8388607)
        bps = 24
    elif st == "PCM_16":
        v = np.clip(np.rint(np.asarray(data, np.float64) * 32767.0), -32768, 32767)
        bps = 16
    else:
        raise AudioFormatError(f"FLAC subtype {subtype} not supported")
    blob = flac_encode_int(v.astype(np.int32), sr, bps)
    with open(path, "wb") as f:
        f.write(blob)


def _sniff(path: str):
    """Container by content, like libsndfile (the reference writes FLAC to
    whatever name ``-o`` gives, src/process_tomatis_xfade.py:115)."""
    try:
        with open(path, "rb") as f:
            head = f.read(10)
            k = id3v2_size(head)
            f.seek(k)
            m = f.read(4)
    except OSError:
        return None
    return {b"fLaC": "flac", b"RIFF": "wav", b"RF64": "wav"}.get(m)


def info(path: str):
    """(samplerate, channels, frames) without decoding the samples."""
    if _sf is not None and not path.lower().endswith(".wav"):
        i = _sf.info(path)
        return i.samplerate, i.channels, i.frames
    if _sniff(path) == "flac":
        with open(path, "rb") as f:
            k = id3v2_size(f.read(10))
            f.seek(k)
            head = f.read(42)
        sr, ch, _, n = flac_info_bytes(head)
        if n == 0:   # total unknown in STREAMINFO: count the frames
            n = flac_count_frames(_flac_bytes(path))
        return sr, ch, n
    fmt, ch, sr, bits, data_off, data_len = _parse_wav_header(path)
    return sr, ch, data_len // (ch * (bits // 8))


def read(path: str):
    """Decode a file to float32 [frames, channels] and its sample rate."""
    kind = _sniff(path)
    if kind == "flac" and _sf is None:
        return _read_flac(path)
    if kind == "wav" or path.lower().endswith(".wav"):
        return _read_wav(path)
    if _sf is None:
        raise AudioFormatError(f"cannot decode {os.path.basename(path)}: libsndfile (soundfile) "
                               "is not installed; provide a WAV file")
    x, sr = _sf.read(path, dtype="float32", always_2d=True)
    return np.ascontiguousarray(x, np.float32), sr


def write(path: str, data: np.ndarray, sr: int, fmt: str = "FLAC", subtype: str = "PCM_24"):
    """Encode ``data`` ([frames, ch] float) to ``path`` (FLAC via libsndfile, or WAV)."""
    data = np.asarray(data)
    if data.ndim == 1:
        data = data[:, None]
    if fmt.upper() == "WAV":
        _write_wav(path, data, sr, subtype)
        return
    if _sf is None:
        if fmt.upper() != "FLAC":
            raise AudioFormatError(f"format {fmt} needs libsndfile (soundfile), not installed")
        _write_flac(path, data, sr, subtype)
        return
    _sf.write(path, data, sr, format=fmt, subtype=subtype)


def write_with_fallback(out_path: str, data: np.ndarray, sr: int, log=print):
    """FLAC PCM_24, else WAV PCM_24 at ``out_path.replace('.flac', '.wav')``.

    Mirrors src/process_tomatis.py:242-251.  Returns (written_path, is_flac).
    """
    try:
        write(out_path, data, sr, "FLAC", "PCM_24")
        log("[OK] 输出格式: FLAC 24-bit")
        return out_path, True
    except Exception as e:
        log(f"[WARN] FLAC 写入失败: {e}")
        wav_path = out_path.replace(".flac", ".wav")
        write(wav_path, data, sr, "WAV", "PCM_24")
        log("[OK] 输出格式: WAV 24-bit (稍后需转换为 FLAC)")
        return wav_path, False


# ---------------------------------------------------------------------------
# RIFF/WAVE
# ---------------------------------------------------------------------------

def _parse_wav_header(path: str):
    with open(path, "rb") as f:
        head = f.read(12)
        if len(head) < 12 or head[:4] not in (b"RIFF", b"RF64") or head[8:12] != b"WAVE":
            raise AudioFormatError(f"{path}: not a RIFF/WAVE file")
        fmt = ch = sr = bits = None
        while True:
            hdr = f.read(8)
            if len(hdr) < 8:
                raise AudioFormatError(f"{path}: no data chunk")
            cid, size = hdr[:4], struct.unpack("<I", hdr[4:])[0]
            if cid == b"fmt ":
                body = f.read(size)
                fmt, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
                if fmt == WAVE_FORMAT_EXTENSIBLE and size >= 40:
                    fmt = struct.unpack("<H", body[24:26])[0]
                if size % 2:
                    f.read(1)
            elif cid == b"data":
                if fmt is None:
                    raise AudioFormatError(f"{path}: data before fmt chunk")
                off = f.tell()
                f.seek(0, os.SEEK_END)
                avail = f.tell() - off
                return fmt, ch, sr, bits, off, min(size, avail) if size != 0xFFFFFFFF else avail
            else:
                f.seek(size + (size % 2), os.SEEK_CUR)


def _read_wav(path: str):
    fmt, ch, sr, bits, off, nbytes = _parse_wav_header(path)
    bps = bits // 8
    n = nbytes // (ch * bps)
    raw = np.fromfile(path, dtype=np.uint8, count=n * ch * bps, offset=off)
    if fmt == WAVE_FORMAT_IEEE_FLOAT:
        if bits == 32:
            x = raw.view("<f4").astype(np.float32)
        elif bits == 64:
            x = raw.view("<f8").astype(np.float32)
        else:
            raise AudioFormatError(f"{path}: float{bits} WAV not supported")
    elif fmt == WAVE_FORMAT_PCM:
        if bits == 8:
            x = (raw.astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = raw.view("<i2").astype(np.float32) / np.float32(32768.0)
        elif bits == 24:
            b = raw.reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / np.float32(8388608.0)
        elif bits == 32:
            x = (raw.view("<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
        else:
            raise AudioFormatError(f"{path}: PCM{bits} WAV not supported")
    else:
        raise AudioFormatError(f"{path}: WAV format tag {fmt:#x} not supported")
    return np.ascontiguousarray(x.reshape(n, ch)), sr


def _write_wav(path: str, data: np.ndarray, sr: int, subtype: str = "PCM_24"):
    n, ch = data.shape
    st = subtype.upper()
    if st == "PCM_24":
        v = np.rint(np.asarray(data, np.float64) * 8388607.0)
        v = np.clip(v, -8388608, 8388607).astype(np.int32).reshape(-1)
        b = np.empty((v.size, 3), np.uint8)
        b[:, 0] = v & 0xFF
        b[:, 1] = (v >> 8) & 0xFF
        b[:, 2] = (v >> 16) & 0xFF
        payload, fmt, bits = b.tobytes(), WAVE_FORMAT_PCM, 24
    elif st == "PCM_16":
        v = np.clip(np.rint(np.asarray(data, np.float64) * 32767.0), -32768, 32767)
        payload, fmt, bits = v.astype("<i2").tobytes(), WAVE_FORMAT_PCM, 16
    elif st == "FLOAT":
        payload, fmt, bits = np.asarray(data, "<f4").tobytes(), WAVE_FORMAT_IEEE_FLOAT, 32
    else:
        raise AudioFormatError(f"WAV subtype {subtype} not supported")
    ba = ch * bits // 8
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 36 + len(payload)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<IHHIIHH", 16, fmt, ch, sr, sr * ba, ba, bits))
        f.write(b"data" + struct.pack("<I", len(payload)))
        f.write(payload)
