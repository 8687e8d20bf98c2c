#!/bin/bash
# round 3: full GPU suite on the consolidated build, C2 limiter rescale order A/B
set -o pipefail
D=gpurun_out/${1:-r3l}; mkdir -p $D
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
BA=""
b c2_rev0 TOMATIS_LIM_REV=0
b c2_rev1 TOMATIS_LIM_REV=1
b c2_rev0b TOMATIS_LIM_REV=0
b c2_rev1b TOMATIS_LIM_REV=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
