#!/bin/bash
# round 3: min-hold probes split over workgroups — adaptive tests, C3 bench + timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-r3t}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_level_stats.py tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_gpu_compositions.py tests/test_gpu_anysize.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2; do
  TOMATIS_C3_GROUPS=2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample-s 0 --workload c3 > $D/c3_g2_$i.log 2>&1 || { tail -20 $D/c3_g2_$i.log; exit 1; }
  echo "g2 $(grep -o '"ms_per_step": [0-9.]*' $D/c3_g2_$i.log) $(grep -o '"kernel_ms": [0-9.]*' $D/c3_g2_$i.log)"
done
TOMATIS_C3_GROUPS=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample-s 0 --workload c3 > $D/c3_g1.log 2>&1 || { tail -20 $D/c3_g1.log; exit 1; }
echo "g1 $(grep -o '"ms_per_step": [0-9.]*' $D/c3_g1.log)"
TOMATIS_C3_GROUPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/tr_g2 -o c3 -- python3 bench.py --workload c3 --steps 3 --warmup 2 --cpu-sample-s 0 > $D/tr_g2.log 2>&1 || { tail -20 $D/tr_g2.log; exit 1; }
python3 tools/timeline.py $(find $D/tr_g2 -name '*kernel_trace.csv' | head -1) > $D/timeline_g2.txt
