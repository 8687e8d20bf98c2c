#!/usr/bin/env python3
"""Write profiles/pmc_traffic.json from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Usage: tools/pmc_traffic.py PMC_DIR WORKLOAD [--kernel k_stft_ola] [--alg-bytes B]
                            [--base BASE_DIR [--base-kernel K]]

PMC_DIR holds the per-pass rocprofv3 outputs of tools/pmc.sh or
tools/pmc_fetch.sh (p*/run_counter_collection.csv).  For the fused kernel the
per-dispatch counters are averaged over its dispatches and converted to bytes
the way MI355X_MICROARCH.md (HBM / rocprofv3 section) prescribes:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so reads = 2 x FETCH_SIZE.  The
kernel's input loads are 8-byte-per-lane buffer loads, a width the guide lists
as uncalibrated, so the uncorrected figure is kept beside the corrected one.
bench.py reads "hbm_bytes_per_launch" for its roofline.traffic field.

--base: a pipelined launch reads its own input (8-B lanes) and the previous
batch's limited blocks (16-B lanes, the partner rescale).  BASE_DIR is the
same kernel's run with no chunk over the limit (bench --input-gain 0.05): its
FETCH_SIZE is the input part, taken as reported; the excess over it is the
partner part, corrected x2 (the guide's factor for 16-B streaming reads).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    a = sys.argv[1:]
    d, workload = a[0], a[1]
    kern = a[a.index("--kernel") + 1] if "--kernel" in a else "k_stft_ola"
    alg = float(a[a.index("--alg-bytes") + 1]) if "--alg-bytes" in a else None
    # reads: "raw" = FETCH_SIZE as reported (8-B-per-lane loads; calibrated on the
    # limiter-inactive run, whose FETCH_SIZE is 1.08x the input bytes read once),
    # "x2" = the guide's gfx950 factor for 16-B-per-lane streaming reads
    reads = a[a.index("--reads") + 1] if "--reads" in a else "raw"
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
        sys.exit(f"no FETCH_SIZE/WRITE_SIZE dispatches of {kern} under {d}")
    fetch_kib = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write_kib = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
    rd = (2.0 if reads == "x2" else 1.0) * fetch_kib * 1024.0
    base_kib = None
    if "--base" in a:
        bv = []
        # (--base-kernel: the base is another instantiation, e.g. the same
        # run's first, unpipelined pass)
        bk = a[a.index("--base-kernel") + 1] if "--base-kernel" in a else kern
        for f in sorted(glob.glob(os.path.join(a[a.index("--base") + 1], "p*",
                                               "run_counter_collection.csv"))):
            for r in csv.DictReader(open(f)):
                if bk in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                    bv.append(float(r["Counter_Value"]))
        if "--base-first" in a:  # only the base run's first N dispatches (e.g. the
            # pipeline's first, unpipelined passes, not bench.py's one-file passes)
            bv = bv[:int(a[a.index("--base-first") + 1])]
        if not bv:
            sys.exit(f"no FETCH_SIZE dispatches of {kern} under the base run")
        base_kib = sum(bv) / len(bv)
        rd = (base_kib + 2.0 * max(0.0, fetch_kib - base_kib)) * 1024.0
        reads = "base+2x"
    wr = write_kib * 1024.0
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "profiles", "pmc_traffic.json")
    try:
        doc = json.load(open(out_path))
    except (OSError, ValueError):
        doc = {}
    rec = {"kernel": kern, "dispatches": len(vals["FETCH_SIZE"]),
           "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
           "read_bytes": rd, "write_bytes": wr,
           "hbm_bytes_per_launch": rd + wr,
           "hbm_bytes_x2_reads": 2.0 * fetch_kib * 1024.0 + wr,
           "source": os.path.relpath(d),
           "reads": reads,
           "correction": ("reads = FETCH_SIZE: the kernel's input loads are 8 B/lane, a width "
                          "MI355X_MICROARCH.md leaves uncalibrated; calibrated on the "
                          "limiter-inactive run (bench --input-gain 0.05), where FETCH_SIZE is "
                          "1.08x the input bytes (each input byte once + warm-up halos)"
                          if reads == "raw" else
                          "reads = FETCH_SIZE of the no-limit run (input, 8-B lanes, as "
                          "reported) + 2 x the excess (the partner rescale's 16-B reads)"
                          if reads == "base+2x" else
                          "reads = 2 x FETCH_SIZE (gfx950, 16-B/lane streaming-read factor)")}
    if base_kib is not None:
        rec["base_fetch_size_kib"] = base_kib
    if alg:
        rec["alg_bytes_per_launch"] = alg
        rec["traffic_over_alg"] = (rd + wr) / alg
    doc[workload] = rec
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
