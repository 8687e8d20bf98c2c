#!/bin/bash
# n_fft 4096 in-kernel levels / gate / alpha: new tests, then the suites that
# touch the gated and cross-fade paths, then c5x / c5 bench.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6h}
D=gpurun_out/$TAG; mkdir -p $D
[ -n "${SKIP_SMOKE:-}" ] || timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
[ -n "${SKIP_4096:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_levels_4096.py -x -v --timeout 300 --timeout-method thread > $D/t4096.log 2>&1 || { tail -60 $D/t4096.log; exit 1; }
tail -n 1 $D/t4096.log
timeout -k 10 900 python -u -m pytest ${SUITE:-tests/test_gpu_parity.py tests/test_gpu_fused_levels.py} tests/test_gpu_pipelined.py tests/test_gpu_as_benched.py tests/test_gpu_robustness.py -x -v --timeout 400 --timeout-method thread > $D/tsuite.log 2>&1 || { tail -60 $D/tsuite.log; exit 1; }
tail -n 1 $D/tsuite.log
for w in c5x c5 c2; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample-s 0 --single-steps 0 > $D/b_$w.log 2>&1 || { tail -20 $D/b_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/b_$w.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/b_$w.log) $(grep -o '"frac": [0-9.]*' $D/b_$w.log | head -1) $(grep -o '"gate_fallbacks": [0-9]*' $D/b_$w.log)"
done
