#!/usr/bin/env python3
"""Kernel timeline of the last step in a rocprofv3 --kernel-trace CSV (diagnostic).

usage: python tools/timeline.py <kernel_trace.csv> [first-kernel-substring]

The last step is taken to start at the earliest of the last burst (within
3 ms) of dispatches whose name contains the substring (default
k_absmax_streams, the adaptive step's first kernel, one per stream group);
prints start/end/duration in
us relative to that step's first dispatch, the queue, and the kernel name.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "k_absmax_streams"
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r.get("Queue_Id", "?"), r["Kernel_Name"]))
    rows.sort()
    firsts = [i for i, r in enumerate(rows) if key in r[3]]
    if not firsts:
        raise SystemExit(f"no kernel matching {key}")
    # the step's first kernel dispatches come in a burst (one per stream group)
    tl = rows[firsts[-1]][0]
    t0 = min(rows[i][0] for i in firsts if tl - rows[i][0] < 3_000_000)
    print(f"{'start':>9} {'end':>9} {'dur':>8}  queue  kernel   (us from the step's first {key})")
    for s, e, q, n in rows:
        if s < t0 - 100_000:
            continue
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:<5} {n[:90]}")


if __name__ == "__main__":
    main()
