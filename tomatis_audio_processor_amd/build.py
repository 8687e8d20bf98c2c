"""Build ``libtomatis_hip.so`` in-tree with hipcc for gfx950 (no cmake/ninja needed)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "tm_kernels.hip")
DEPS = [SRC, os.path.join(HERE, "csrc", "tm_common.h"), os.path.join(HERE, "csrc", "tm_fft.h"),
        os.path.join(ROOT, "include", "tomatis_hip.h")]
OUT = os.path.join(HERE, "libtomatis_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC", "-shared",
         "-I" + os.path.join(ROOT, "include")]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
