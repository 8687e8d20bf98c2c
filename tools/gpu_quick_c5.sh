#!/bin/bash
# full GPU suite, then C2 / c5x / c5x-quiet / c5 benches (no CPU legs)
set -o pipefail
TAG=${1:-q5}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
for w in "c2" "c5x" "c5x --input-gain 0.05" "c5"; do
  n=$(echo $w | tr -d ' -' | cut -c1-16)
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_$n.log 2>&1 || { tail -20 $D/bench_$n.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$n.log) $(grep -o '"frac": [0-9.]*' $D/bench_$n.log | head -1)"
done
