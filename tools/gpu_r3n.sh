#!/bin/bash
# round 3: speculative min-hold bisection — GPU suite, C3 serial vs speculative x groups, analysis bench
set -o pipefail
D=gpurun_out/${1:-r3n}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
BA="--workload c3"
b c3_g2_spec TOMATIS_C3_GROUPS=2
b c3_g2_ser TOMATIS_C3_GROUPS=2 TOMATIS_MH_SERIAL=1
b c3_g4_spec TOMATIS_C3_GROUPS=4
b c3_g4_ser TOMATIS_C3_GROUPS=4 TOMATIS_MH_SERIAL=1
b c3_g8_spec TOMATIS_C3_GROUPS=8
timeout -k 10 300 python -u tools/bench_analysis.py > $D/bench_analysis.log 2>&1 || { tail -20 $D/bench_analysis.log; exit 1; }
grep -o '"fn": "[a-z_]*"\|"ms": [0-9.]*\|"spec_kernel_ms": [0-9.]*' $D/bench_analysis.log | paste -sd' '
