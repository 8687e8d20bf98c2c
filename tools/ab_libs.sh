#!/bin/bash
# A/B the C2 bench over library variants: tools/ab_libs.sh TAG lib1.so lib2.so ...
# Each variant first runs smoke() (states bit-exact, samples vs the oracle) unless
# NOSMOKE=1, then the bench; logs -> gpurun_out/TAG/<lib>.log
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG; mkdir -p $D
for L in "$@"; do
  n=$(basename $L .so)
  if [ -z "${NOSMOKE:-}" ]; then
    TOMATIS_HIP_LIB=$PWD/$L timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/$n.smoke 2>&1 || { echo "$n smoke FAILED"; tail -3 $D/$n.smoke; continue; }
  fi
  TOMATIS_HIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 ${BENCH_ARGS:-} > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"frac": [0-9.]*' $D/$n.log | head -1) $(tail -1 $D/$n.smoke 2>/dev/null | grep -o 'max|err|=[0-9.e+-]*')"
  grep tm_profile $D/$n.log | tail -2
done
true
