#!/bin/bash
# GPU check: parity tests, bench, kernel-trace stats.  Usage: tools/gpu_check.sh TAG
set -u
TAG=${1:-run}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $R/gpurun_out/tests_$TAG.log 2>&1; echo "tests rc=$?" >> $R/gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $R/gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-sample-s 0 ${BENCH_ARGS:-} > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo prof failed; exit 1; }
echo ok
