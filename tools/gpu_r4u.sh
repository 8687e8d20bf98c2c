#!/bin/bash
# round 4: C5x launch shapes via dev options (no rebuild)
set -o pipefail
D=gpurun_out/r4u; mkdir -p $D
for rep in 1 2; do
  for v in "" "--dev WG=256" "--dev WG=512" "--dev RUN_ROUNDS=2"; do
    n=$(echo "x$v" | tr -c 'A-Za-z0-9' '_')
    timeout -k 10 200 python -u bench.py --workload c5x --steps 10 --warmup 3 --cpu-sample-s 0 $v > $D/$n.$rep.log 2>&1 || { tail -20 $D/$n.$rep.log; exit 1; }
    echo "$rep [$v] $(grep -o '"ms_per_step": [0-9.]*' $D/$n.$rep.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.$rep.log)"
  done
done
