#!/bin/bash
# Instruction-fetch / issue counters of the fused kernel (diagnostic): lists the
# SQ/SQC counters the box offers, then one pass over a few of them.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=${PMC_OUT:-$R/gpurun_out/pmc_if}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o -E "\b(SQC?_[A-Z0-9_]+)" $OUT/avail.txt | sort -u > $OUT/sq_names.txt || true
ARGS="bench.py --steps 2 --warmup 1 --cpu-sample-s 0 ${BENCH_ARGS:-}"
i=0
for C in "${@}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C -d $OUT/p$i -o run --output-format csv -- python3 $ARGS > $OUT/p$i.log 2>&1 || echo "pass $i ($C) failed"
done
echo pmc_ifetch done
