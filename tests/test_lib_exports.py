"""The C-ABI library loads and exports every entry point include/tomatis_hip.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tomatis_hip.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tomatis_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_abi():
    names = declared()
    assert "tomatis_stft_ola" in names and "tomatis_levels" in names
    assert len(names) >= 14


def test_library_exports_all_symbols():
    from tomatis_audio_processor_amd import _lib
    path = _lib.lib_path()
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: run __graft_entry__.build() first")
    h = ctypes.CDLL(path)
    missing = [n for n in declared() if not hasattr(h, n)]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(declared())
    assert h.tomatis_abi_version() == _lib.ABI_VERSION == 11
    h.tomatis_status_string.restype = ctypes.c_char_p
    assert h.tomatis_status_string(-2).decode().startswith("configuration")


def test_header_constants_match_binding():
    from tomatis_audio_processor_amd import _lib
    src = open(HEADER).read()
    defs = dict(re.findall(r"#define (TOMATIS_[A-Z0-9_]+) \(?(-?\d+)u?\)?", src))
    for name, val in [("TOMATIS_ABI_VERSION", _lib.ABI_VERSION),
                      ("TOMATIS_GATE_SEGMENT", _lib.GATE_SEGMENT),
                      ("TOMATIS_GATE_NONE", _lib.GATE_NONE),
                      ("TOMATIS_ERR_LIMITER_WAIT", _lib.ERR_LIMITER_WAIT),
                      ("TOMATIS_ERR_PAIR_BARRIER", _lib.ERR_PAIR_BARRIER),
                      ("TOMATIS_OPT_FUSE_LIMITER", _lib.OPT_FUSE_LIMITER),
                      ("TOMATIS_OPT_LIMITER_SPIN", _lib.OPT_LIMITER_SPIN),
                      ("TOMATIS_OPT_MINHOLD_SERIAL", _lib.OPT_MINHOLD_SERIAL)]:
        assert int(defs[name]) == val, name


def test_struct_layout_matches_header():
    from tomatis_audio_processor_amd import _lib
    # 10 int64/float/int32 fields ... verified against the C compiler below
    import subprocess, tempfile
    c = r'''
#include <stdio.h>
#include <stddef.h>
#include "tomatis_hip.h"
int main(){printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(TomatisStream), offsetof(TomatisStream,t_on),
 offsetof(TomatisStream,frame_base), sizeof(TomatisPlanDesc), offsetof(TomatisStream,on_exc),
 sizeof(TomatisGateCand), offsetof(TomatisGateCand,up_delay));return 0;}
'''
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "s.c")
        open(src, "w").write(c)
        exe = os.path.join(d, "s")
        subprocess.run(["gcc", "-I" + os.path.join(ROOT, "include"), src, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    S = _lib.TomatisStream
    G = _lib.TomatisGateCand
    got = [ctypes.sizeof(S), S.t_on.offset, S.frame_base.offset,
           ctypes.sizeof(_lib.TomatisPlanDesc), S.on_exc.offset, ctypes.sizeof(G),
           G.up_delay.offset]
    import numpy as np
    assert np.dtype(_lib.GATE_CAND_DTYPE).itemsize == ctypes.sizeof(G)
    assert [int(v) for v in out] == got


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    from tomatis_audio_processor_amd import _lib
    monkeypatch.setenv("TOMATIS_HIP_LIB", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_LIB", None)
    with pytest.raises(_lib.TomatisLibraryError):
        _lib.lib()
