#!/bin/bash
# c5x / c5 pipelined vs not, c5x quiet (no limiter engaged)
set -o pipefail
TAG=${1:-c5ab}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipelined.py -x -q --timeout 240 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for w in "c5x" "c5x --no-pipeline" "c5x --input-gain 0.05" "c5" "c5 --no-pipeline"; do
  n=$(echo $w | tr -d ' -' | cut -c1-20)
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_$n.log 2>&1 || { tail -20 $D/bench_$n.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$n.log) $(grep -o '"frac": [0-9.]*' $D/bench_$n.log | head -1) $(grep -o '"device_error": [0-9]*' $D/bench_$n.log)"
done
