#!/bin/bash
# round-6 lease D: adaptive tests with the min-hold hipGraph, C3 A/B (graph on / off) -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6d}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_level_stats.py tests/test_gpu_pipelined.py tests/test_gpu_robustness.py tests/test_gpu_as_benched.py tests/test_gpu_cli.py -m gpu -x -q -k "adaptive or c3 or minhold or level or Adaptive" --timeout 400 --timeout-method thread > $D/adaptive_tests.log 2>&1 || { tail -60 $D/adaptive_tests.log; exit 1; }
tail -1 $D/adaptive_tests.log
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-sample-s 0 --single-steps 0 --dev NO_GRAPHS=$v > $D/bench_c3_g$v.$i.log 2>&1 || { tail -20 $D/bench_c3_g$v.$i.log; exit 1; }
    echo "c3 NO_GRAPHS=$v run $i $(grep -o '"ms_per_step": [0-9.]*' $D/bench_c3_g$v.$i.log | head -1)"
  done
done
