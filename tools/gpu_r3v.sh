#!/bin/bash
# round 3: double-buffered batches (levels + gate of pass k+1 during pass k's transform)
set -o pipefail
D=gpurun_out/${1:-r3v}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compositions.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
b() {
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 "$@" > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
b c2_b1 --batches 1
b c2_b2 --batches 2
b c2_b1b --batches 1
b c2_b2b --batches 2
b c4_b1 --workload c4 --batches 1
b c4_b2 --workload c4 --batches 2
b c5x_b2 --workload c5x --batches 2
