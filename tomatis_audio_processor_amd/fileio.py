"""Streaming file ingest and egress for the device pipeline.

The reference decodes with libsndfile in 10-s blocks and writes FLAC PCM_24
chunk by chunk (src/process_tomatis.py:225-251,433-457).  Here a file goes
straight between the native FLAC codec and HBM:

ingest   FLAC bytes -> K byte ranges decoded on host threads into one
         page-locked int32 block (``tomatis_flac_decode_bytes``); each range's
         samples are DMA'd to HBM on a copy stream while the next range
         decodes; int -> float32 (libsndfile's 2^(bps-1) rule) on the device.
egress   float32 -> PCM_24 on the device (``tomatis_float_to_pcm``), FLAC
         frames encoded on the device (``tomatis_flacd_plan`` / ``_write``:
         per 4096-sample block plan and exact size, host prefix sum of the
         sizes, frames written at their offsets), then the compressed bytes
         D2H in pieces through two page-locked buffers while the file is
         written.  Shapes the device encoder declines: segments of 2^22 frames
         D2H, encoded on host threads (``tomatis_flac_enc_push``) while the next
         one is in flight, written by a writer thread.  Both paths give the
         bytes of a whole-buffer host encode.

WAV files (and any format when libsndfile is importable) go through
``audio_io`` on the host as before; the reference's FLAC -> WAV fallback on an
encoder failure is kept.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

from . import audio_io
from ._lib import check, lib, ptr, stream_handle

SEG_FRAMES = 4096 * 1024     # egress segment (a whole number of FLAC blocks)
IN_RANGES = 8                # ingest byte ranges


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("device file I/O needs a ROCm GPU (MI355X)")
    return torch


def _flac():
    h = audio_io._flac()
    if not getattr(h, "_tm_stream_sigs", False):
        P, I32, I64 = C.c_void_p, C.c_int32, C.c_int64
        h.tomatis_flac_enc_open.argtypes = [I32, I32, I32, C.POINTER(P)]
        h.tomatis_flac_enc_push.argtypes = [P, P, I64]
        h.tomatis_flac_enc_finish.argtypes = [P, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(I64)]
        h.tomatis_flac_enc_close.argtypes = [P]
        h.tomatis_flac_enc_close.restype = None
        h.tomatis_flac_enc_take.argtypes = [P, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(I64)]
        h.tomatis_flac_enc_header.argtypes = [P, P]
        h.tomatis_flac_first_frame.argtypes = [P, I64]
        h.tomatis_flac_first_frame.restype = I64
        h.tomatis_flac_decode_bytes.argtypes = [P, I64, I64, I64, P, I64, C.POINTER(I64),
                                                C.POINTER(I64)]
        h._tm_stream_sigs = True
    return h


def _err(rc, what):
    if rc:
        raise audio_io.AudioFormatError(f"{what}: {audio_io._FLAC_ERR.get(rc, rc)}")


class Timer(dict):
    """Wall-clock phases of one file (seconds), for the e2e bench."""

    def add(self, k, t0):
        self[k] = self.get(k, 0.0) + time.perf_counter() - t0


def read_device(path: str, timer: Timer | None = None):
    """(x float32 cuda tensor [n*ch] interleaved, n, ch, sr) of an audio file."""
    torch = _torch()
    kind = audio_io._sniff(path)
    if kind == "flac" and not audio_io.have_soundfile():
        return _read_flac_device(path, timer)
    t0 = time.perf_counter()
    x, sr = audio_io.read(path)
    if timer is not None:
        timer.add("decode", t0)
    t0 = time.perf_counter()
    n, ch = x.shape
    xd = torch.from_numpy(np.ascontiguousarray(x).reshape(-1)).cuda()
    if timer is not None:
        torch.cuda.synchronize()
        timer.add("h2d", t0)
    return xd, n, ch, sr


def _read_flac_device(path, timer=None):
    """The file is memory-mapped (no host copy: the decode threads read the page
    cache directly); byte ranges decode into one page-locked int32 block, each
    range DMA'd to HBM on a copy stream while the next one decodes."""
    import mmap
    torch = _torch()
    h = _flac()
    t0 = time.perf_counter()
    with open(path, "rb") as f:
        if os.fstat(f.fileno()).st_size == 0:
            raise audio_io.AudioFormatError(f"{path}: empty file")
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    try:
        mv = np.frombuffer(mm, np.uint8)
        skip = audio_io.id3v2_size(bytes(mm[:10]))
        buf, size = mv.ctypes.data + skip, len(mm) - skip
        if timer is not None:
            timer.add("read", t0)
        r = _decode_flac_on_device(h, torch, mv[skip:], buf, size, timer)
        if r is None:
            x, n, ch, sr = _decode_flac_ranges(h, torch, buf, size, path, timer)
        else:
            x, n, ch, sr = r
        del mv
    finally:
        t1 = time.perf_counter()
        try:
            mm.close()
        except BufferError:  # an export is still alive: the map goes with it
            pass
        if timer is not None:
            timer.add("unmap", t1)
    return x, n, ch, sr


UP_PARTS = 8                 # host threads copying the mapped file into page-locked memory
# k_fdd_scan reports frame number x this for fixed-blocksize frames; a power of
# two above any block size, so the frame number comes back exactly
FLAC_NOMINAL_GUESS = 1 << 20


def _decode_flac_on_device(h, torch, src, buf, size, timer=None):
    """The FLAC stream src (uint8 numpy view of the mapped file, at address buf)
    decoded on the device (tomatis_flacd_*): the bytes go up through a
    page-locked block (host threads copy slices of the mapping, each slice DMA'd
    as soon as it is in), candidate frames are found and verified there, and
    the verified frames must tile the stream -- first frame at the first frame
    offset, each next one where the previous ended, consecutive samples to the
    STREAMINFO total, the last one ending at the end of the file.  Returns
    (x float32 [n*ch], n, ch, sr), or None for the host decoder (other shapes,
    a stream of unknown length, trailing bytes, anything that does not chain)."""
    import concurrent.futures as cf
    L = lib()
    sr_, ch_, bps_, n_ = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    if h.tomatis_flac_info(buf, size, C.byref(sr_), C.byref(ch_), C.byref(bps_), C.byref(n_)):
        return None
    sr, ch, bps, n = sr_.value, ch_.value, bps_.value, n_.value
    if not (1 <= ch <= 2 and 4 <= bps <= 24) or n <= 0:
        return None
    first = int(h.tomatis_flac_first_frame(buf, size))
    if first < 0:
        return None
    t0 = time.perf_counter()
    hs = stream_handle()
    dev = torch.empty((size + 8 + 3) // 4 * 4, dtype=torch.uint8, device="cuda")
    dev[size:].zero_()
    pin = torch.empty(max(1, size), dtype=torch.uint8, pin_memory=True)
    pin_np = pin.numpy()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    edges = np.linspace(0, size, UP_PARTS + 1).astype(np.int64)

    def part(k):
        a, b = int(edges[k]), int(edges[k + 1])
        np.copyto(pin_np[a:b], src[a:b])
        return k

    with cf.ThreadPoolExecutor(max_workers=UP_PARTS) as ex:
        for k in ex.map(part, range(UP_PARTS)):   # in order: DMA slice k once it is in
            a, b = int(edges[k]), int(edges[k + 1])
            if b > a:
                with torch.cuda.stream(cs):
                    dev[a:b].copy_(pin[a:b], non_blocking=True)
    torch.cuda.current_stream().wait_stream(cs)
    if timer is not None:
        torch.cuda.synchronize()
        timer.add("upload", t0)
    t0 = time.perf_counter()
    cap = n // 16 + 4096
    cand = torch.empty(cap, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    check(L.tomatis_flacd_find(ptr(dev), size, first, ch, bps, ptr(cand), cap, ptr(cnt), hs),
          "flacd_find")
    nc = int(cnt.item())
    if nc == 0 or nc > cap:
        return None
    cand = torch.sort(cand[:nc]).values
    info = torch.empty(4 * nc, dtype=torch.int64, device="cuda")
    check(L.tomatis_flacd_scan(ptr(dev), size, ptr(cand), nc, ch, bps, FLAC_NOMINAL_GUESS, ptr(info),
                               hs), "flacd_scan")
    inf = info.view(nc, 4).cpu().numpy()
    offs = cand.cpu().numpy()
    ok = inf[:, 0] > 0
    fo, fb, fs, fn, fv = offs[ok], inf[ok, 0], inf[ok, 1], inf[ok, 2], inf[ok, 3]
    if len(fo) == 0 or not (np.all(fv == fv[0])):
        return None
    # one fixed block size (the nominal one of every frame but the last) or
    # the coded sample numbers; the scan took frame numbers x the guess
    nominal = int(fn[0])
    chain = (fo[0] == first and np.array_equal(fo[1:], fo[:-1] + fb[:-1]) and
             int(fo[-1] + fb[-1]) == size)
    if not chain:
        return None
    fixed = fv[0] == 0
    if fixed and not (np.all(fn[:-1] == nominal) and fn[-1] <= nominal):
        return None
    start = fs // FLAC_NOMINAL_GUESS * nominal if fixed else fs
    if not (start[0] == 0 and np.array_equal(start[1:], start[:-1] + fn[:-1]) and
            int(start[-1] + fn[-1]) >= n):
        return None
    frames = torch.from_numpy(np.ascontiguousarray(fo)).to("cuda")
    pcm = torch.empty(max(1, n * ch), dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    check(L.tomatis_flacd_decode(ptr(dev), size, ptr(frames), len(fo), ch, bps,
                                 nominal if fixed else 0, ptr(pcm), n, ptr(err), hs),
          "flacd_decode")
    x = torch.empty(max(1, n * ch), dtype=torch.float32, device="cuda")
    check(L.tomatis_pcm_to_float(ptr(pcm), n * ch, bps, ptr(x), hs), "pcm_to_float")
    if int(err.item()):
        return None
    if timer is not None:
        timer.add("decode", t0)
    return x[:n * ch], n, ch, sr


def _decode_flac_ranges(h, torch, buf, size, path, timer):
    sr_, ch_, bps_, n_ = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    _err(h.tomatis_flac_info(buf, size, C.byref(sr_), C.byref(ch_), C.byref(bps_), C.byref(n_)),
         "FLAC")
    sr, ch, bps, n = sr_.value, ch_.value, bps_.value, n_.value
    if n == 0:   # unknown total in STREAMINFO: count by decoding without storing
        got_ = C.c_int64()
        _err(h.tomatis_flac_decode(buf, size, None, 0, C.byref(got_)), "FLAC decode failed")
        n = got_.value
    pin = torch.empty(max(1, n * ch), dtype=torch.int32, pin_memory=True)
    dev = torch.empty(max(1, n * ch), dtype=torch.int32, device="cuda")
    cs = torch.cuda.Stream()
    first = int(h.tomatis_flac_first_frame(buf, size))
    if first < 0:
        raise audio_io.AudioFormatError(f"{path}: not a FLAC stream")
    edges = np.linspace(first, size, IN_RANGES + 1).astype(np.int64)
    s_lo, s_hi = C.c_int64(), C.c_int64()
    got = 0
    t0 = time.perf_counter()
    for k in range(IN_RANGES):
        if h.tomatis_flac_decode_bytes(buf, size, int(edges[k]), int(edges[k + 1]),
                                       pin.data_ptr(), n, C.byref(s_lo), C.byref(s_hi)):
            got = -1   # a damaged range: the whole-buffer decoder decides
            break
        a, b = s_lo.value, s_hi.value
        if b > a:
            if a != got:   # frames missing / out of order: the whole-buffer decoder decides
                got = -1
                break
            with torch.cuda.stream(cs):   # DMA while the next range decodes
                dev[a * ch:b * ch].copy_(pin[a * ch:b * ch], non_blocking=True)
            got = b
    if got != n:
        # a gap, or fewer samples than STREAMINFO's total: a truncated stream
        # (the whole-buffer decoder returns the frames it holds) or a damaged
        # frame (it raises) -- let it decide, with its result
        cs.synchronize()
        got_ = C.c_int64()
        _err(h.tomatis_flac_decode(buf, size, pin.data_ptr(), n, C.byref(got_)),
             "FLAC decode failed")
        n = got_.value
        dev[:n * ch].copy_(pin[:n * ch])
    torch.cuda.current_stream().wait_stream(cs)
    x = torch.empty(max(1, n * ch), dtype=torch.float32, device="cuda")
    check(lib().tomatis_pcm_to_float(ptr(dev), n * ch, bps, ptr(x), stream_handle()),
          "pcm_to_float")
    if timer is not None:
        torch.cuda.synchronize()
        timer.add("decode+h2d", t0)
    cs.synchronize()   # the page-locked block may be reused once the copies have landed
    return x[:n * ch], n, ch, sr


class _EncBuf:
    """Bytes taken from the streaming encoder: a zero-copy view until free()."""

    def __init__(self, h, p, n):
        self.h, self.p, self.n = h, p, n

    def view(self):
        return memoryview((C.c_uint8 * self.n).from_address(C.addressof(self.p.contents)))

    def free(self):
        if self.p:
            self.h.tomatis_flac_free(self.p)
            self.p = None


def _encode_segments(y, n, ch, sr, bps, sink, timer=None):
    """Quantise on the device, then per segment of SEG_FRAMES frames: D2H into
    one of two page-locked buffers on a copy stream while the host encodes the
    previous one; every segment's frame bytes go to ``sink``.  Returns the
    42-byte stream header (STREAMINFO)."""
    torch = _torch()
    h = _flac()
    t0 = time.perf_counter()
    yi = torch.empty(max(1, n * ch), dtype=torch.int32, device="cuda")
    check(lib().tomatis_float_to_pcm(ptr(y), n * ch, bps, ptr(yi), stream_handle()),
          "float_to_pcm")
    enc = C.c_void_p()
    _err(h.tomatis_flac_enc_open(ch, sr, bps, C.byref(enc)), "FLAC encode failed")
    try:
        seg = SEG_FRAMES
        K = (n + seg - 1) // seg
        pins = [torch.empty(seg * ch, dtype=torch.int32, pin_memory=True)
                for _ in range(min(2, max(1, K)))]
        evs = [torch.cuda.Event() for _ in pins]
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())

        def issue(k):
            a, b = k * seg, min(n, (k + 1) * seg)
            with torch.cuda.stream(cs):
                pins[k % 2][:(b - a) * ch].copy_(yi[a * ch:b * ch], non_blocking=True)
                evs[k % 2].record(cs)

        if K:
            issue(0)
        out = C.POINTER(C.c_uint8)()
        ln = C.c_int64()
        for k in range(K):
            if k + 1 < K:
                issue(k + 1)          # its buffer's previous segment was pushed at k - 1
            evs[k % 2].synchronize()
            a, b = k * seg, min(n, (k + 1) * seg)
            _err(h.tomatis_flac_enc_push(enc, pins[k % 2].data_ptr(), b - a),
                 "FLAC encode failed")
            _err(h.tomatis_flac_enc_take(enc, C.byref(out), C.byref(ln)), "FLAC encode failed")
            if ln.value:   # the sink owns the encoder buffer (frees it with tomatis_flac_free)
                sink(_EncBuf(h, out, ln.value))
                out = C.POINTER(C.c_uint8)()
        hdr = (C.c_uint8 * 42)()
        _err(h.tomatis_flac_enc_header(enc, hdr), "FLAC encode failed")
    finally:
        h.tomatis_flac_enc_close(enc)
    if timer is not None:
        timer.add("d2h+encode", t0)
    return bytes(hdr)


FLAC_BLOCK = 4096             # tm_flac.cpp kBlock / tm_flacenc.hip kFdBlock
D2H_CHUNK = 1 << 26          # device-encoded bytes per D2H copy while the file is written


def _streaminfo_header(frames, ch, sr, bps, min_fs, max_fs, min_bs, max_bs) -> bytes:
    """"fLaC" + the STREAMINFO block tm_flac.cpp writes (MD5 zero)."""
    if frames == 0:
        min_fs = max_fs = 0
        min_bs = max_bs = FLAC_BLOCK
    fields = [(FLAC_BLOCK if frames > FLAC_BLOCK else max(16, min_bs), 16),
              (max(16, max_bs), 16), (min_fs, 24), (max_fs, 24), (sr, 20), (ch - 1, 3),
              (bps - 1, 5), (frames >> 32, 4), (frames & 0xFFFFFFFF, 32)]
    acc = 0
    for v, nb in fields:
        acc = (acc << nb) | (v & ((1 << nb) - 1))
    return b"fLaC" + bytes([0x80, 0, 0, 34]) + acc.to_bytes(18, "big") + bytes(16)


def _device_frames(yi, n: int, ch: int, bps: int):
    """FLAC frames of device int32 PCM yi [n*ch] encoded on the device
    (tomatis_flacd_*, byte-identical to the host encoder): (uint8 device
    tensor of the frames, total bytes, (min_fs, max_fs, min_bs, max_bs)), or
    None when the device encoder declines (shape, or a block it cannot hold)."""
    torch = _torch()
    L, hs = lib(), stream_handle()
    if not (1 <= ch <= 2 and 4 <= bps <= 24) or n == 0:
        return None
    nblk = (n + FLAC_BLOCK - 1) // FLAC_BLOCK
    ws = torch.empty(int(L.tomatis_flacd_workspace_bytes(n, ch)), dtype=torch.uint8,
                     device="cuda")
    sizes = torch.empty(nblk, dtype=torch.int32, device="cuda")
    check(L.tomatis_flacd_plan(ptr(yi), n, ch, bps, ptr(ws), ptr(sizes), hs), "flacd_plan")
    sz = sizes.cpu().numpy().view(np.uint32).astype(np.int64)   # synchronises
    if (sz >= 0xFFFFFFFE).any():
        return None
    off = np.zeros(nblk, np.int64)
    np.cumsum(sz[:-1], out=off[1:])
    total = int(off[-1] + sz[-1])
    out = torch.zeros((total + 7) // 4 * 4, dtype=torch.uint8, device="cuda")
    off_d = torch.from_numpy(off).to("cuda")
    check(L.tomatis_flacd_write(ptr(yi), n, ch, bps, ptr(ws), ptr(off_d), ptr(out), hs),
          "flacd_write")
    bs_last = n - (nblk - 1) * FLAC_BLOCK
    stats = (int(sz.min()), int(sz.max()), min(FLAC_BLOCK, bs_last), FLAC_BLOCK if nblk > 1 else bs_last)
    return out, total, stats


def encode_flac_device_frames(y, n: int, ch: int, sr: int, bps: int = 24):
    """The FLAC stream of device float32 samples y [n*ch] encoded on the device,
    as (header bytes, uint8 device tensor of the frames, frame bytes), or None
    when the device encoder declines (the host encoder then applies)."""
    torch = _torch()
    yi = torch.empty(max(1, n * ch), dtype=torch.int32, device="cuda")
    check(lib().tomatis_float_to_pcm(ptr(y), n * ch, bps, ptr(yi), stream_handle()),
          "float_to_pcm")
    r = _device_frames(yi, n, ch, bps)
    if r is None:
        return None
    out, total, (min_fs, max_fs, min_bs, max_bs) = r
    return _streaminfo_header(n, ch, sr, bps, min_fs, max_fs, min_bs, max_bs), out, total


def encode_flac_device(y, n: int, ch: int, sr: int, bps: int = 24, timer=None,
                       device_encoder: bool = True) -> bytes:
    """FLAC stream of the device float32 samples y [n*ch] at ``bps`` bits
    (encoded on the device when it takes the shape, else on host threads; the
    bytes are the same)."""
    if device_encoder:
        t0 = time.perf_counter()
        r = encode_flac_device_frames(y, n, ch, sr, bps)
        if r is not None:
            hdr, out, total = r
            b = hdr + out[:total].cpu().numpy().tobytes()
            if timer is not None:
                timer.add("encode+d2h", t0)
            return b
    parts = []

    def take(b):
        try:
            parts.append(bytes(b.view()))
        finally:
            b.free()

    hdr = _encode_segments(y, n, ch, sr, bps, take, timer)
    return hdr + b"".join(parts)


def _write_device_frames(f, y, n, ch, sr, timer=None) -> bool:
    """Device-encoded FLAC into the open file f: header, then the frames in
    D2H_CHUNK pieces through two page-locked buffers (the copy of piece k + 1
    overlaps the write of piece k).  False when the device encoder declines."""
    torch = _torch()
    t0 = time.perf_counter()
    r = encode_flac_device_frames(y, n, ch, sr, 24)
    if r is None:
        return False
    hdr, out, total = r
    if timer is not None:
        torch.cuda.synchronize()
        timer.add("encode", t0)
    t0 = time.perf_counter()
    f.write(hdr)
    K = (total + D2H_CHUNK - 1) // D2H_CHUNK
    pins = [torch.empty(min(D2H_CHUNK, max(1, total)), dtype=torch.uint8, pin_memory=True)
            for _ in range(min(2, max(1, K)))]
    evs = [torch.cuda.Event() for _ in pins]
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())

    def issue(k):
        a, b = k * D2H_CHUNK, min(total, (k + 1) * D2H_CHUNK)
        with torch.cuda.stream(cs):
            pins[k % 2][:b - a].copy_(out[a:b], non_blocking=True)
            evs[k % 2].record(cs)

    if K:
        issue(0)
    for k in range(K):
        evs[k % 2].synchronize()
        a, b = k * D2H_CHUNK, min(total, (k + 1) * D2H_CHUNK)
        view = pins[k % 2][:b - a].numpy()
        if k + 1 < K:
            # the other buffer's previous piece was written at k - 1
            issue(k + 1)
        f.write(memoryview(view))
    if timer is not None:
        timer.add("d2h+write", t0)
    return True


def write_device(out_path: str, y, n: int, ch: int, sr: int, log=print, timer=None,
                 device_encoder: bool = True):
    """FLAC PCM_24 of device samples y [n*ch], else the reference's WAV fallback
    at ``out_path.replace('.flac', '.wav')`` (src/process_tomatis.py:242-251).
    As in the reference, only a failure to *open* the FLAC output (the file or
    the encoder) falls back to WAV; an error while encoding or writing (a device
    error in the quantiser, a full disk) removes the partial file and raises.
    FLAC frames are encoded on the device (``tomatis_flacd_*``) and copied out
    while the file is written; shapes the device encoder declines go through
    the host encoder, whose frame bytes a writer thread writes while later
    segments encode (the header over a placeholder at the end).  Both give the
    same bytes.  Returns (written_path, is_flac)."""
    if audio_io.have_soundfile():
        return audio_io.write_with_fallback(out_path, y.cpu().numpy().reshape(n, ch), sr, log=log)
    import queue
    import threading
    h = _flac()
    t_open = time.perf_counter()
    try:
        enc = C.c_void_p()
        _err(h.tomatis_flac_enc_open(ch, sr, 24, C.byref(enc)), "FLAC encoder")
        h.tomatis_flac_enc_close(enc)
        f = open(out_path, "wb")
        if timer is not None:
            timer.add("open", t_open)
    except Exception as e:
        log(f"[WARN] FLAC 写入失败: {e}")
        wav_path = out_path.replace(".flac", ".wav")
        audio_io.write(wav_path, y.cpu().numpy().reshape(n, ch), sr, "WAV", "PCM_24")
        log("[OK] 输出格式: WAV 24-bit (稍后需转换为 FLAC)")
        return wav_path, False
    try:
        with f:
            if device_encoder and _write_device_frames(f, y, n, ch, sr, timer):
                t_close = time.perf_counter()
                f.close()
                if timer is not None:
                    timer.add("close", t_close)
                log("[OK] 输出格式: FLAC 24-bit")
                return out_path, True
            f.seek(0)
            f.truncate()
            f.write(b"\0" * 42)
            q = queue.Queue(maxsize=4)
            err = []

            def writer():
                while True:
                    b = q.get()
                    if b is None:
                        return
                    try:
                        if not err:
                            f.write(b.view())
                    except Exception as e:  # reported after the encode
                        err.append(e)
                    finally:
                        b.free()

            th = threading.Thread(target=writer, daemon=True)
            th.start()
            try:
                hdr = _encode_segments(y, n, ch, sr, 24, q.put, timer)
            finally:
                q.put(None)
                th.join()
            if err:
                raise err[0]
            t0 = time.perf_counter()
            f.seek(0)
            f.write(hdr)
    except BaseException:
        try:
            os.remove(out_path)
        except OSError:
            pass
        raise
    if timer is not None:
        timer.add("write", t0)
    log("[OK] 输出格式: FLAC 24-bit")
    return out_path, True


def requantize_device(y, n: int, ch: int, bps: int = 24):
    """Device float32 samples as a PCM_``bps`` file written from y reads back
    (libsndfile's float -> int rule, then int / 2^(bps-1)): the input of the
    reference's second pass over its own output (src/layer2_apply_eq.py:220-231)."""
    torch = _torch()
    yi = torch.empty(max(1, n * ch), dtype=torch.int32, device="cuda")
    check(lib().tomatis_float_to_pcm(ptr(y), n * ch, bps, ptr(yi), stream_handle()),
          "float_to_pcm")
    out = torch.empty(max(1, n * ch), dtype=torch.float32, device="cuda")
    check(lib().tomatis_pcm_to_float(ptr(yi), n * ch, bps, ptr(out), stream_handle()),
          "pcm_to_float")
    return out[:n * ch]


def device_stream_set(x, n: int, ch: int, sr: int):
    """One-stream ``engine.StreamSet`` over a device buffer from read_device."""
    from . import engine
    return engine.StreamSet(x=x, offs=[0], lens=[n], ch=ch, sr=sr)


__all__ = ["read_device", "write_device", "encode_flac_device", "encode_flac_device_frames",
           "requantize_device", "device_stream_set", "Timer"]
