#!/bin/bash
# One FETCH_SIZE + one WRITE_SIZE pass (rocprofv3 --pmc) of bench.py: tools/pmc_fetch.sh TAG
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/pmcf_$1
mkdir -p $OUT
ARGS="bench.py --steps 2 --warmup 1 --cpu-sample-s 0 ${BENCH_ARGS:-}"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/p1 -o run --output-format csv -- python3 $ARGS > $OUT/p1.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/p2 -o run --output-format csv -- python3 $ARGS > $OUT/p2.log 2>&1 || { echo "write pass failed"; exit 1; }
echo pmcf done
