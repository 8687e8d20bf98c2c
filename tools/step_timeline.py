#!/usr/bin/env python3
"""Kernel timeline around the last dispatches of a kernel in a rocprofv3
--kernel-trace CSV (diagnostic): start / end / duration in us relative to the
second-to-last dispatch of the key kernel.

usage: python tools/step_timeline.py <kernel_trace.csv> [key=k_stft_ola] [before=8]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "k_stft_ola"
    before = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70])
                  for r in csv.DictReader(open(path, newline="")))
    idx = [i for i, r in enumerate(rows) if key in r[2]]
    if len(idx) < 2:
        raise SystemExit(f"fewer than two dispatches matching {key}")
    t0 = rows[idx[-2]][0]
    for s, e, n in rows[max(0, idx[-2] - before):idx[-1] + 4]:
        print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {n}")


if __name__ == "__main__":
    main()
