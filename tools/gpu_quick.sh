#!/bin/bash
# Quick GPU check: the GPU tests, then bench lines for the given workloads.
set -o pipefail
TAG=${1:-quick}; shift
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log) $(grep -o '"frac": [0-9.]*' $D/bench_$w.log | head -1)"
done
