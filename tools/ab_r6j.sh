#!/bin/bash
# c5x: fused 4096 gate variants (timing only: no gate stores / no alpha / no
# level code) vs fused and two-pass, same box.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6j}
D=gpurun_out/$TAG; mkdir -p $D
B=abx/libx_gx_base.so
for i in 1 2; do
  for L in $B abx/libx_gx_NOLV.so; do
    n=$(basename $L .so)
    TOMATIS_HIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload c5x --steps 20 --warmup 3 --cpu-sample-s 0 --single-steps 0 > $D/${n}_$i.log 2>&1 || { tail -20 $D/${n}_$i.log; exit 1; }
    echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/${n}_$i.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/${n}_$i.log)"
  done
  TOMATIS_HIP_LIB=$PWD/$B timeout -k 10 200 python -u bench.py --workload c5x --steps 20 --warmup 3 --cpu-sample-s 0 --single-steps 0 --dev FUSED_LEVELS=0 > $D/twopass_$i.log 2>&1 || { tail -20 $D/twopass_$i.log; exit 1; }
  echo "twopass $(grep -o '"ms_per_step": [0-9.]*' $D/twopass_$i.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/twopass_$i.log)"
done
