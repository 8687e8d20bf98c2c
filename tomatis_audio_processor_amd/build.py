"""Build ``libtomatis_hip.so`` in-tree with hipcc for gfx950 (no cmake/ninja needed).

Six translation units, compiled in parallel and linked into one C-ABI library:

* ``tm_kernels.hip``   levels, gate, limiter, plan and the ``extern "C"`` entry points;
* ``tm_transform.hip`` the fused transform kernels (FMA contraction on;
  ``TOMATIS_TRANSFORM_SCHED`` selects another LLVM machine scheduler for
  experiments — measured within 1 % of the default);
* ``tm_analysis.hip``  analysis spectra for the validators / calibration tools
  (SURVEY.md §8 rows f3/f4);
* ``tm_flacenc.hip``   FLAC frames encoded on the device (row f1's egress);
* ``tm_flacdec.hip``   FLAC frames decoded on the device (row f1's ingest).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
# machine scheduler of the transform unit ("" = LLVM's default, occupancy-aware)
SCHED = os.environ.get("TOMATIS_TRANSFORM_SCHED", "")
UNITS = {  # source -> extra flags
    "tm_kernels.hip": [],
    # FMA contraction in the transform unit only (-2 % kernel time, measured): the
    # spectral path has a 1e-4 tolerance, the level / gate unit stays
    # -ffp-contract=off for its bit-exact r
    "tm_transform.hip": ["-ffp-contract=fast"] +
                        (["-mllvm", f"-amdgpu-sched-strategy={SCHED}"] if SCHED else []),
    "tm_analysis.hip": [],
    "tm_flacenc.hip": [],
    "tm_flacdec.hip": [],
}
DEPS = [os.path.join(CSRC, f) for f in (*UNITS, "tm_common.h", "tm_fft.h", "tm_shared.h",
                                        "tm_lds_fft.h", "tm_host_dsp.h", "tm_gate.h")] + \
       [os.path.join(ROOT, "include", "tomatis_hip.h"), os.path.abspath(__file__)]
OUT = os.path.join(HERE, "libtomatis_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "--offload-arch=gfx950"
FLAGS = [ARCH, "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC",
         "-I" + os.path.join(ROOT, "include")]


def _unit_cmd(src: str, fl, extra, obj: str):
    return [HIPCC, *FLAGS, *fl, *extra, "-c", "-o", obj + ".tmp", os.path.join(CSRC, src)]


def _unit_hash(src: str, cmd) -> str:
    """Content hash of a unit: its full command line (minus the output path),
    its source and every shared header -- an object whose recorded hash
    differs is rebuilt (flags changed, or an edit landed during a build)."""
    import hashlib
    h = hashlib.sha256(" ".join(cmd[:-3] + cmd[-1:]).encode())
    for d in [os.path.join(CSRC, src)] + [d for d in DEPS if not d.endswith(".hip")]:
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(obj: str, src: str, cmd) -> bool:
    """A unit recompiles when its object is missing or its recorded hash
    (objects and hashes are kept next to the library) differs."""
    if not os.path.exists(obj) or not os.path.exists(obj + ".hash"):
        return True
    with open(obj + ".hash") as f:
        return f.read().strip() != _unit_hash(src, cmd)


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    return any(_stale(f"{out}.{src}.o", src, _unit_cmd(src, fl, (), f"{out}.{src}.o"))
               for src, fl in UNITS.items())


def build(force: bool = False, verbose: bool = True, out: str = OUT, extra=()) -> str:
    """Compile the C-ABI library; ``out``/``extra`` build experiment variants."""
    if out == OUT and not extra and not force and not needs_build():
        return OUT
    objs, procs = [], []
    for src, fl in UNITS.items():
        obj = f"{out}.{src}.o"
        objs.append(obj)
        cmd = _unit_cmd(src, fl, extra, obj)
        if not force and not extra and not _stale(obj, src, cmd):
            continue
        digest = _unit_hash(src, cmd)  # of the inputs as compiled (before the compile)
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), obj, digest))
    rcs = [p.wait() for p, _, _ in procs]
    if any(rcs):
        raise subprocess.CalledProcessError(max(rcs), "hipcc")
    for _, obj, digest in procs:
        os.replace(obj + ".tmp", obj)
        with open(obj + ".hash", "w") as f:
            f.write(digest + "\n")
    link = [HIPCC, ARCH, "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    if extra or out != OUT:
        for o in objs:
            os.remove(o)
            if os.path.exists(o + ".hash"):
                os.remove(o + ".hash")
    return out


FLAC_SRC = os.path.join(CSRC, "tm_flac.cpp")
FLAC_OUT = os.path.join(HERE, "libtomatis_flac.so")


def build_flac(force: bool = False, verbose: bool = True) -> str:
    """Host FLAC codec: plain C++, built with g++."""
    deps = [FLAC_SRC, os.path.join(ROOT, "include", "tomatis_flac.h"), os.path.abspath(__file__)]
    if (not force and os.path.exists(FLAC_OUT)
            and all(os.path.getmtime(d) <= os.path.getmtime(FLAC_OUT) for d in deps)):
        return FLAC_OUT
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-shared", "-fPIC",
           "-o", FLAC_OUT + ".tmp", FLAC_SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(FLAC_OUT + ".tmp", FLAC_OUT)
    return FLAC_OUT


if __name__ == "__main__":
    # python -m tomatis_audio_processor_amd.build [--force] [--out PATH -- extra hipcc flags]
    a = sys.argv[1:]
    extra = a[a.index("--") + 1:] if "--" in a else []
    out = a[a.index("--out") + 1] if "--out" in a else OUT
    build(force="--force" in a, out=out, extra=extra)
    build_flac(force="--force" in a)
