"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer build of the host FLAC
codec (csrc/tm_flac.cpp) under a corruption sweep (tools/flac_sanitize.cpp).

The codec parses untrusted bytes on every CLI ingest, in place of libsndfile
behind the reference's sf.read / sf.write (src/process_tomatis.py:225-251).
The sweep flips bits in every header / metadata byte, in the first bytes of
every frame (frame, subframe and residual-partition headers), around every
multi-thread decode range boundary of a stream large enough for a 4-thread
decode, and at pseudo-random body positions, and truncates streams at frame
boundaries and random lengths -- on streams from the C encoder (1-6 channels,
8-32 bits) and from the independent Python writer of test_flac_codec.py (LPC,
escape-coded and Rice2 partitions, wasted bits, side/right and mid/side).
Every corruption inside an audio frame must return an error status; no
sanitizer report may occur (the build aborts on the first one).  Host code
only: nothing here touches a GPU.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _independent_streams(d):
    from tests.test_flac_codec import py_flac
    out = []
    for assign in (9, 10):
        rng = np.random.default_rng(100 + assign)
        frames = []
        for n in (256, 200, 256, 128, 256):
            t = np.arange(n)
            base = (np.sin(t * 0.05) * 3e6).astype(np.int64)
            L = base + rng.integers(-50, 50, n)
            R = base // 2 + rng.integers(-50, 50, n)
            if assign == 10:
                R = L - 4 * ((L - R) // 4)
            frames.append(np.stack([L, R], 1))
        path = os.path.join(d, f"indep_{assign}.flac")
        with open(path, "wb") as f:
            f.write(py_flac(frames, 48000, 24, assign))
        out += [path, str(sum(len(f) for f in frames)), "2"]
    return out


@pytest.mark.timeout(900)
def test_flac_codec_sanitizers(tmp_path):
    cxx = shutil.which(os.environ.get("CXX", "g++"))
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "flac_sanitize")
    cmd = [cxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
           "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tomatis_audio_processor_amd", "csrc", "tm_flac.cpp"),
           os.path.join(ROOT, "tools", "flac_sanitize.cpp"), "-o", exe, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "asan" in (r.stderr or "").lower():
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, TOMATIS_FLAC_THREADS="4",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    args = [exe] + _independent_streams(str(tmp_path))
    r = subprocess.run(args, capture_output=True, text=True, env=env, timeout=850)
    tail = (r.stderr or "")[-3000:]
    assert r.returncode == 0, tail
    assert "failures 0" in tail, tail
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, tail
