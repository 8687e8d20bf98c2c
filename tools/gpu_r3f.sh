#!/bin/bash
# round 3: dynamic work list (runs + rescale slices) A/B on C2 (limited / quiet),
# run-length variants, C3/C4, then the full GPU suite
set -o pipefail
D=gpurun_out/${1:-r3f}; mkdir -p $D
b() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_runs.py > $D/quick.log 2>&1 || { tail -30 $D/quick.log; exit 1; }
tail -1 $D/quick.log
BA="" b c2_dyn TOMATIS_DYN=1
BA="" b c2_static TOMATIS_DYN=0
BA="--input-gain 0.05" b c2q_dyn TOMATIS_DYN=1
BA="--input-gain 0.05" b c2q_static TOMATIS_DYN=0
BA="" b c2_dyn_150_24 TOMATIS_RUN_FRAMES=150
BA="" b c2_dyn_96_16 TOMATIS_RUN_TAIL=16
BA="" b c2_dyn_64_16 TOMATIS_RUN_FRAMES=64 TOMATIS_RUN_TAIL=16
BA="" b c2_dyn_lag2 TOMATIS_RESCALE_LAG=2
BA="" b c2_dyn_200_32 TOMATIS_RUN_FRAMES=200 TOMATIS_RUN_TAIL=32
BA="" b c2_dyn_s64 TOMATIS_SLICE_KB=64
BA="--workload c3" b c3_dyn TOMATIS_DYN=1
BA="--workload c4" b c4_dyn TOMATIS_DYN=1
BA="--workload c4" b c4_static TOMATIS_DYN=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
