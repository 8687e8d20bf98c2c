#!/bin/bash
# round 3: balanced work-list rounds vs static runs (C2 limited / quiet, C3, C4)
set -o pipefail
D=gpurun_out/${1:-r3j}; mkdir -p $D
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_runs.py tests/test_gpu_robustness.py > $D/quick.log 2>&1 || { tail -30 $D/quick.log; exit 1; }
tail -1 $D/quick.log
BA=""
b l_static TOMATIS_DYN=0
b l_list TOMATIS_DYN=1
b l_list_128 TOMATIS_RUN_FRAMES=128
b l_list_t16 TOMATIS_RUN_TAIL=16
b l_list_t32 TOMATIS_RUN_TAIL=32
b l_list_lag2 TOMATIS_RESCALE_LAG=2
b l_list_48 TOMATIS_RUN_FRAMES=48
BA="--input-gain 0.05"
b q_static TOMATIS_DYN=0
b q_list TOMATIS_DYN=1
b q_list_128 TOMATIS_RUN_FRAMES=128
BA="--workload c3"
b c3_static TOMATIS_DYN=0
b c3_list TOMATIS_DYN=1
BA="--workload c4"
b c4_static TOMATIS_DYN=0
b c4_list TOMATIS_DYN=1
