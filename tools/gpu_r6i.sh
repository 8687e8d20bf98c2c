#!/bin/bash
# c5x / c5: fused 4096 levels + gate + alpha vs the two-pass chain (--dev
# FUSED_LEVELS=0), same box, twice each; then the 4096 tests.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6i}
D=gpurun_out/$TAG; mkdir -p $D
for i in 1 2; do
  for v in "" "--dev FUSED_LEVELS=0"; do
    for w in c5x ${W2:-}; do
      f=$D/b_${w}_${i}${v:+_twopass}.log
      timeout -k 10 300 python -u bench.py --workload $w --cpu-sample-s 0 --single-steps 0 $v > $f 2>&1 || { tail -20 $f; exit 1; }
      echo "$w ${v:-fused} $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) $(grep -o '"kernel_ms": [0-9.]*' $f) $(grep -o '"gate_fallbacks": [0-9]*' $f)"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_levels_4096.py -x -q --timeout 300 --timeout-method thread > $D/t4096.log 2>&1 || { tail -60 $D/t4096.log; exit 1; }
tail -n 1 $D/t4096.log
