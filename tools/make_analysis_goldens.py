#!/usr/bin/env python3
"""Generate the analysis-spectrum golden fixtures (``tests/golden/an_*.npz``) by
running the REFERENCE's own functions (``/root/reference/src``) on the seeded
inputs of ``tests/golden/an_cases.py``:

  compare_audio.power_mono + compare_audio.stft_mag_avg
  layer2_analyze_eq.stft_logpower_median
  validate_layer1.compute_conditional_spectrum

Build-container only.  The modules import ``soundfile`` at top level (absent
here): ``tools/_sf_stub`` satisfies the import; none of these functions touch
files.  Fixtures hold only parameters and the reference's outputs.

Usage:  MPLBACKEND=Agg python tools/make_analysis_goldens.py [--missing]
(--missing: only cases without a fixture, leaving committed ones untouched)
"""
from __future__ import annotations

import importlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF_SRC = "/root/reference/src"
sys.path.insert(0, os.path.join(HERE, "_sf_stub"))
sys.path.insert(0, REPO)
os.environ.setdefault("MPLBACKEND", "Agg")
from tests.golden.an_cases import AN_CASES, an_inputs  # noqa: E402


def ref(mod):
    if REF_SRC not in sys.path:
        sys.path.insert(1, REF_SRC)
    return importlib.import_module(mod)


def main():
    missing = "--missing" in sys.argv[1:]
    for c in AN_CASES:
        p = os.path.join(REPO, "tests", "golden", c["name"] + ".npz")
        if missing and os.path.exists(p):
            continue
        x, y, states = an_inputs(c)
        out = {"meta": np.array(json.dumps(c))}
        if c["fn"] == "stft_mag_avg":
            m = ref("compare_audio")
            mono = m.power_mono(x)
            out["mag"] = m.stft_mag_avg(mono, c["sr"], c["n_fft"], c["hop"])
        elif c["fn"] == "stft_logpower_median":
            m = ref("layer2_analyze_eq")
            freqs, med, used = m.stft_logpower_median(x, c["sr"], c["n_fft"], c["hop"],
                                                      c["music_dbfs"])
            out.update(freqs=freqs, med=med, used=np.array(used))
        else:
            m = ref("validate_layer1")
            freqs, c1, c2, n1, n2 = m.compute_conditional_spectrum(
                x, y, c["sr"], states, c["n_fft"], c["hop"], c["level_threshold"])
            out.update(freqs=freqs, c1_db=c1, c2_db=c2, n1=np.array(n1), n2=np.array(n2))
        np.savez_compressed(p, **out)
        print(c["name"], {k: (v.shape, v.dtype) for k, v in out.items() if k != "meta"},
              {k: int(v) for k, v in out.items() if k in ("used", "n1", "n2")})


if __name__ == "__main__":
    main()
