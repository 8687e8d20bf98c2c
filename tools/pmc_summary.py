#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel.

Per kernel: mean over dispatches of each counter, plus derived metrics:
  VALU busy   = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES  (per-wave issue share)
  HBM bytes   = 2 * FETCH_SIZE(KB) * 1024 + WRITE_SIZE(KB) * 1024
(MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced streaming read; WRITE_SIZE is exact for 16-B-per-lane stores.)
Usage: tools/pmc_summary.py gpurun_out/pmc [kernel-substring] [--json out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    data = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            data[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = dict(vgpr=r["VGPR_Count"], agpr=r.get("Accum_VGPR_Count"),
                           lds=r["LDS_Block_Size"], grid=r["Grid_Size"], wg=r["Workgroup_Size"])
    return data, meta


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    data, meta = load(d)
    out = {}
    for k, cs in data.items():
        if sub and sub not in k:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["HBM_BYTES_corrected"] = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                      "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in m:
                    m[c + "/WAVE_CYCLES"] = m[c] / m["SQ_WAVE_CYCLES"]
        out[k] = dict(meta=meta.get(k), counters=m)
        print(f"== {k[:110]}\n   {meta.get(k)}")
        for c in sorted(m):
            print(f"   {c:34s} {m[c]:.6g}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
