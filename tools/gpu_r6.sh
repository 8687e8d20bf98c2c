#!/bin/bash
# round-6 lease: the new / changed GPU tests first, then the whole suite, smoke
# and the default bench (+ the whole-batch C4 workloads) -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipelined.py tests/test_gpu_fused_levels.py tests/test_gpu_as_benched.py tests/test_gpu_cli.py -m gpu -x -v --timeout 400 --timeout-method thread > $D/new_tests.log 2>&1 || { tail -60 $D/new_tests.log; exit 1; }
tail -1 $D/new_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 600 python -u bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-600
for w in c4 c4all c4allh; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log) $(grep -o '"gate_fallbacks": [0-9]*' $D/bench_$w.log)"
done
