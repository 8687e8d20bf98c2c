#!/usr/bin/env python3
"""Print bench JSON highlights and kernel stats for a gpu_check TAG."""
import csv, json, sys
tag = sys.argv[1]
try:
    print(open(f"gpurun_out/tests_{tag}.log").read().strip().splitlines()[-2:])
except OSError:
    pass
for line in open(f"gpurun_out/bench_{tag}.log"):
    if line.startswith("{"):
        d = json.loads(line)
        print("value", d["value"], d["unit"], "ms/step", d["ms_per_step"])
        print("roofline", {k: d["roofline"][k] for k in ("achieved", "frac", "kernel_ms", "traffic")})
        print("compute", d["compute"]["achieved"], d["compute"]["frac"], "cpu", d["cpu_baseline"] and d["cpu_baseline"]["value"])
try:
    rows = list(csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_stats.csv")))
    for r in rows[:9]:
        print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>3} {r['Name'][:80]}")
except OSError:
    pass
