#!/bin/bash
# round 4: limiter rounds x fused levels on C4 / C2 (same box)
set -o pipefail
D=gpurun_out/r4h; mkdir -p $D
for w in c4 c2; do
  for V in "" "--dev LIMITER_ROUNDS=2" "--dev FUSED_LEVELS=0" "--dev FUSED_LEVELS=0 --dev LIMITER_ROUNDS=2"; do
    n=$(echo "$w$V" | tr -c 'a-zA-Z0-9' '_')
    timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --cpu-sample-s 0 $V > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
    echo "$w [$V] $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log)"
  done
done
