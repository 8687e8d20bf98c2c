#!/bin/bash
# Final evidence, lease part 1: tools/gpu_final.sh TAG tests  (full GPU suite +
# smoke) or tools/gpu_final.sh TAG bench (the default bench with its CPU legs,
# every other workload, quiet / unpipelined C2, the file->file benches).
# -> gpurun_out/TAG
set -o pipefail
TAG=${1:-final}
PART=${2:-tests}
D=gpurun_out/$TAG; mkdir -p $D
if [ "$PART" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
  tail -n 1 $D/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
  tail -n 1 $D/smoke.log
  exit 0
fi
timeout -k 10 600 python -u bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -n 1 $D/bench.log | cut -c1-300
for w in c3 c4 c4h c4all c4allh c5x c5 c2ts; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log | head -2 | tr '\n' ' ') $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log) $(grep -o '"frac": [0-9.]*' $D/bench_$w.log | head -1) $(grep -o '"gate_fallbacks": [0-9]*' $D/bench_$w.log)"
done
timeout -k 10 300 python -u bench.py --input-gain 0.05 --cpu-sample-s 0 --single-steps 0 > $D/bench_quiet.log 2>&1 || { tail -20 $D/bench_quiet.log; exit 1; }
echo "c2 quiet $(grep -o '"ms_per_step": [0-9.]*' $D/bench_quiet.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_quiet.log)"
timeout -k 10 300 python -u bench.py --no-pipeline --cpu-sample-s 0 > $D/bench_nopipe.log 2>&1 || { tail -20 $D/bench_nopipe.log; exit 1; }
echo "c2 unpipelined $(grep -o '"ms_per_step": [0-9.]*' $D/bench_nopipe.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_nopipe.log)"
timeout -k 10 400 python -u tools/bench_file.py > $D/bench_file.log 2>&1 || { tail -20 $D/bench_file.log; exit 1; }
tail -n 1 $D/bench_file.log | cut -c1-300
BATCH_FILES=64 BATCH_SECS=300 BATCH_GB=1 timeout -k 10 600 python -u tools/bench_batch.py > $D/bench_batch.log 2>&1 || { tail -20 $D/bench_batch.log; exit 1; }
tail -n 1 $D/bench_batch.log
