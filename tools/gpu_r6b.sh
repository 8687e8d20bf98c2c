#!/bin/bash
# round-6 lease B: gate / transform tests first, the whole suite, smoke,
# bench (C2 + workloads), the multi-file batch file->file timing -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6b}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_levels.py tests/test_gpu_pipelined.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/first_tests.log 2>&1 || { tail -60 $D/first_tests.log; exit 1; }
tail -1 $D/first_tests.log
timeout -k 10 600 python -u bench.py --cpu-sample-s 0 > $D/bench_nocpu.log 2>&1 || { tail -20 $D/bench_nocpu.log; exit 1; }
echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $D/bench_nocpu.log | head -2 | tr '\n' ' ') $(grep -o '"kernel_ms": [0-9.]*' $D/bench_nocpu.log) $(grep -o '"achievable_peak": [0-9.]*' $D/bench_nocpu.log)"
timeout -k 10 300 python -u bench.py --input-gain 0.05 --cpu-sample-s 0 --single-steps 0 > $D/bench_quiet.log 2>&1 || { tail -20 $D/bench_quiet.log; exit 1; }
echo "c2 quiet $(grep -o '"ms_per_step": [0-9.]*' $D/bench_quiet.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_quiet.log)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
for w in c4 c4h c3 c5x; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log | head -2 | tr '\n' ' ') $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log) $(grep -o '"gate_fallbacks": [0-9]*' $D/bench_$w.log)"
done
df -h ${TMPDIR:-/tmp} | tail -1
BATCH_FILES=64 BATCH_SECS=300 BATCH_GB=1 timeout -k 10 600 python -u tools/bench_batch.py > $D/bench_batch.log 2>&1 || { tail -20 $D/bench_batch.log; exit 1; }
tail -1 $D/bench_batch.log
