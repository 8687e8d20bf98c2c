#!/bin/bash
# round 3: C3 kernel timelines, min-hold bisection auto (first group speculative) vs serial
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-r3p}; mkdir -p $D
for m in auto serial; do
  TOMATIS_MH_MODE=$m TOMATIS_C3_GROUPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/tr_$m -o c3 -- python3 bench.py --workload c3 --steps 3 --warmup 2 --cpu-sample-s 0 > $D/tr_$m.log 2>&1 || { tail -20 $D/tr_$m.log; exit 1; }
  f=$(find $D/tr_$m -name '*kernel_trace.csv' | head -1)
  python3 tools/timeline.py "$f" > $D/timeline_$m.txt
  grep -o '"ms_per_step": [0-9.]*' $D/tr_$m.log
done
