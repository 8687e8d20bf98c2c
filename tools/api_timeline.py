#!/usr/bin/env python3
"""One steady-state adaptive (C3) step from a rocprofv3 --hip-trace --kernel-trace
run (diagnostic): kernels and the host API calls around them, in us from the
step's first k_absmax_streams, plus the step's host API time by function.

usage: python tools/api_timeline.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv> [step from the end, default 3]
"""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ks = {}
    for r in csv.DictReader(open(glob.glob(d + "/*_kernel_trace.csv")[0])):
        ks[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
    kl = sorted(ks.values())
    starts = []
    for s, e, n in kl:
        if "k_absmax_streams" in n and (not starts or s - starts[-1] > 3_000_000):
            starts.append(s)
    t0, t1 = starts[-back], starts[-back + 1]
    api = []
    for r in csv.DictReader(open(glob.glob(d + "/*_hip_api_trace.csv")[0])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 500_000 <= s < t1:
            api.append((s, e, r["Function"], r["Correlation_Id"]))
    tot, cnt = collections.Counter(), collections.Counter()
    for s, e, f, c in api:
        if t0 <= s < t1:
            tot[f] += e - s
            cnt[f] += 1
    print(f"step {(t1 - t0) / 1e3:.1f} us; host API time in the step by function:")
    for f, v in tot.most_common(8):
        print(f"  {f:28s} {cnt[f]:4d} calls {v / 1e3:9.1f} us")
    ev = [(s, e, "K " + n) for s, e, n in kl if t0 <= s < t1]
    for s, e, f, c in api:
        if f in ("hipLaunchKernel", "hipMemcpyAsync", "hipEventSynchronize", "hipStreamWaitEvent",
                 "hipEventRecord"):
            tgt = ks.get(c)
            ev.append((s, e, "A " + f + (" -> " + tgt[2][:60] if tgt else "")))
    ev.sort()
    print(f"{'start':>9} {'end':>9} {'dur':>8}  (us from the step's first k_absmax_streams)")
    for s, e, n in ev:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n[:100]}")


if __name__ == "__main__":
    main()
