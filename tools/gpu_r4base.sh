#!/bin/bash
# round-4 baseline on a fresh box: C2 limited + quiet, C5x, C3 (current tree)
set -o pipefail
D=gpurun_out/r4base; mkdir -p $D
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 > $D/c2.log 2>&1 || { tail -20 $D/c2.log; exit 1; }
echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $D/c2.log) $(grep -o '"kernel_ms": [0-9.]*' $D/c2.log)"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 --input-gain 0.05 > $D/c2q.log 2>&1 || { tail -20 $D/c2q.log; exit 1; }
echo "c2q $(grep -o '"ms_per_step": [0-9.]*' $D/c2q.log) $(grep -o '"kernel_ms": [0-9.]*' $D/c2q.log)"
for w in c5x c4; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/$w.log 2>&1 || { tail -20 $D/$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/$w.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$w.log)"
done
