#!/bin/bash
# round 3: level-stats aggregated histograms + min-hold states in LDS — adaptive tests, C3 timelines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-r3q}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_level_stats.py tests/test_gpu_parity.py -k "adapt or level or minhold" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for g in 2 1 4; do
  TOMATIS_C3_GROUPS=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/tr_g$g -o c3 -- python3 bench.py --workload c3 --steps 3 --warmup 2 --cpu-sample-s 0 > $D/tr_g$g.log 2>&1 || { tail -20 $D/tr_g$g.log; exit 1; }
  f=$(find $D/tr_g$g -name '*kernel_trace.csv' | head -1)
  python3 tools/timeline.py "$f" > $D/timeline_g$g.txt
  echo "g$g traced $(grep -o '"ms_per_step": [0-9.]*' $D/tr_g$g.log)"
done
for g in 2 1 4; do
  TOMATIS_C3_GROUPS=$g timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --cpu-sample-s 0 > $D/c3_g$g.log 2>&1 || { tail -20 $D/c3_g$g.log; exit 1; }
  echo "g$g $(grep -o '"ms_per_step": [0-9.]*' $D/c3_g$g.log) $(grep -o '"kernel_ms": [0-9.]*' $D/c3_g$g.log)"
done
