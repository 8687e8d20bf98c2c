#!/bin/bash
# round 3: C3 stream-group count sweep, analysis bench after the any-n_fft change
set -o pipefail
D=gpurun_out/${1:-r3m}; mkdir -p $D
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
BA="--workload c3"
b c3_g2 TOMATIS_C3_GROUPS=2
b c3_g3 TOMATIS_C3_GROUPS=3
b c3_g4 TOMATIS_C3_GROUPS=4
b c3_g1 TOMATIS_C3_GROUPS=1
timeout -k 10 300 python -u tools/bench_analysis.py > $D/bench_analysis.log 2>&1 || { tail -20 $D/bench_analysis.log; exit 1; }
tail -8 $D/bench_analysis.log
