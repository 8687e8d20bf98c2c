#!/bin/bash
# Confirmation on the round's last code: full GPU suite, smoke, the default
# bench (CPU legs included) and C3.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-final2}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -n 1 $D/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -n 1 $D/smoke.log
timeout -k 10 600 python -u bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -n 1 $D/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --workload c3 --cpu-sample-s 0 > $D/bench_c3.log 2>&1 || { tail -20 $D/bench_c3.log; exit 1; }
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $D/bench_c3.log | head -2 | tr '\n' ' ')"
