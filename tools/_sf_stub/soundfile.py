"""In-memory stand-in for the ``soundfile`` package (golden generation only).

``soundfile`` (libsndfile) is not installed in the build container.  The
reference hot-path modules import it at top level only for file I/O, so
``tools/make_goldens.py`` puts this module on ``sys.path`` first.  It serves
input arrays from ``STORE`` and captures every written chunk as float
(*before* PCM_24 quantisation), which is what the parity fixtures need.  It
replaces no arithmetic of the reference.

``GUARD_BYPASS``: when true, ``samplerate``/``channels`` are returned as an
``int`` subclass whose ``!=`` is always False, so the reference's
48 kHz / stereo guards pass while all arithmetic uses the true value
("Out-of-domain configs").
"""
import numpy as np

STORE = {}        # path -> (array [N, ch] float32, sr)
WRITES = {}       # path -> list of written chunks (as given)
GUARD_BYPASS = False


class _LooseInt(int):
    def __ne__(self, other):
        return False

    def __eq__(self, other):
        return True if GUARD_BYPASS else int.__eq__(self, other)

    __hash__ = int.__hash__


def _wrap(v):
    return _LooseInt(v) if GUARD_BYPASS else int(v)


class _Info:
    def __init__(self, arr, sr):
        self.samplerate = int(sr)
        self.channels = arr.shape[1]
        self.frames = arr.shape[0]
        self.duration = arr.shape[0] / sr
        self.subtype = "PCM_24"
        self.format = "FLAC"


class SoundFile:
    def __init__(self, path, mode="r", samplerate=None, channels=None,
                 format=None, subtype=None, **kw):
        self.path, self.mode = path, mode
        if "r" in mode:
            if path in STORE:
                arr, sr = STORE[path]
            else:                      # read back something written earlier
                chunks = WRITES[path]
                arr = np.concatenate([np.asarray(c, np.float32).reshape(len(c), -1)
                                      for c in chunks])
                sr = WRITES[path + "#sr"]
            self._arr = np.asarray(arr, np.float32)
            self.samplerate = _wrap(sr)
            self.channels = _wrap(self._arr.shape[1])
            self.frames = self._arr.shape[0]
            self._pos = 0
        else:
            WRITES[path] = []
            WRITES[path + "#sr"] = samplerate
            self.samplerate, self.channels = samplerate, channels

    def read(self, frames=-1, dtype="float32", always_2d=False):
        n = self.frames - self._pos if frames < 0 else min(frames, self.frames - self._pos)
        out = self._arr[self._pos:self._pos + n].astype(dtype)
        self._pos += n
        if not always_2d and out.shape[1] == 1:
            out = out[:, 0]
        return out

    def write(self, data):
        WRITES[self.path].append(np.array(data, copy=True))

    def seek(self, pos):
        self._pos = pos

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def read(path, dtype="float32", always_2d=False, **kw):
    with SoundFile(path) as f:
        data = f.read(-1, dtype=dtype, always_2d=always_2d)
        return data, int(f.samplerate)


def write(path, data, samplerate, subtype=None, **kw):
    WRITES[path] = [np.array(data, copy=True)]
    WRITES[path + "#sr"] = samplerate


def info(path):
    arr, sr = STORE[path]
    return _Info(arr, sr)
