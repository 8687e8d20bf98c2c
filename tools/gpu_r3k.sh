#!/bin/bash
# round 3: half-frame n_fft 4096 kernel (two P = 64 waves per frame): tests + C5x/C5 benches
set -o pipefail
D=gpurun_out/${1:-r3k}; mkdir -p $D
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"frac": [0-9.]*' $D/$n.log | head -1) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
TOMATIS_HALF4096=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_anysize.py tests/test_gpu_parity.py tests/test_gpu_compositions.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
BA="--workload c5x"
b c5x_half TOMATIS_HALF4096=1
b c5x_p128 TOMATIS_HALF4096=0
BA="--workload c5"
b c5_half TOMATIS_HALF4096=1
b c5_p128 TOMATIS_HALF4096=0
