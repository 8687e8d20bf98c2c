#!/bin/bash
# round 3: full GPU suite; C3 min-hold probe workgroups per probe (TOMATIS_MH_PARTS) sweep
set -o pipefail
D=gpurun_out/${1:-r3z}; mkdir -p $D
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
for p in ${PARTS:-0 3 14 0 3 14}; do
  TOMATIS_MH_PARTS=$p timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --cpu-sample-s 0 > $D/c3_p$p.log 2>&1 || { tail -20 $D/c3_p$p.log; exit 1; }
  echo "parts $p $(grep -o '"ms_per_step": [0-9.]*' $D/c3_p$p.log) $(grep -o '"device_error": [0-9]*' $D/c3_p$p.log)"
done
