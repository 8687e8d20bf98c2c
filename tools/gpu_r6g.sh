#!/bin/bash
# Side-stream gate look-back: its tests, then the C2 / C4 bench with and without
# it (--serial-lookback) on one box.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6g}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipelined.py tests/test_gpu_as_benched.py tests/test_lib_exports.py -x -v --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -n 1 $D/tests.log
for i in 1 2; do
  for v in "" "--serial-lookback"; do
    for w in c2 c4; do
      timeout -k 10 300 python -u bench.py --workload $w --cpu-sample-s 0 --single-steps 0 $v > $D/b_${w}_${i}${v:+_serial}.log 2>&1 || { tail -20 $D/b_${w}_${i}${v:+_serial}.log; exit 1; }
      echo "$w ${v:-side} $(grep -o '"ms_per_step": [0-9.]*' $D/b_${w}_${i}${v:+_serial}.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/b_${w}_${i}${v:+_serial}.log)"
    done
  done
done
