#!/bin/bash
# round 3: min-hold bisection mode per stream group (first group speculative)
set -o pipefail
D=gpurun_out/${1:-r3o}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_level_stats.py tests/test_gpu_robustness.py tests/test_gpu_compositions.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
BA="--workload c3"
b c3_g2_auto TOMATIS_C3_GROUPS=2
b c3_g2_ser TOMATIS_C3_GROUPS=2 TOMATIS_MH_MODE=serial
b c3_g4_auto TOMATIS_C3_GROUPS=4
b c3_g4_ser TOMATIS_C3_GROUPS=4 TOMATIS_MH_MODE=serial
b c3_g2_auto_b TOMATIS_C3_GROUPS=2
b c3_g2_ser_b TOMATIS_C3_GROUPS=2 TOMATIS_MH_MODE=serial
b c3_g4_auto_b TOMATIS_C3_GROUPS=4
