#!/bin/bash
# round 3: k_mh_probe without the last arriver's cache-wide acquire — adaptive tests, C3 x3
set -o pipefail
D=gpurun_out/${1:-r3aa}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_level_stats.py tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_gpu_anysize.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --cpu-sample-s 0 > $D/c3_$i.log 2>&1 || { tail -20 $D/c3_$i.log; exit 1; }
  echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $D/c3_$i.log) $(grep -o '"device_error": [0-9]*' $D/c3_$i.log)"
done
