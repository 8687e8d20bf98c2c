#!/bin/bash
# round 3: any-size GPU tests, then kernel stats for C3 / C5x / C5 chain and the
# SQ + traffic PMC passes of the n_fft 4096 kernel (c5x)
set -o pipefail
D=gpurun_out/${1:-r3e}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_anysize.py tests/test_gpu_parity.py > $D/anysize.log 2>&1 || { tail -30 $D/anysize.log; exit 1; }
tail -2 $D/anysize.log
export TMPDIR=/tmp
for w in c3 c5x c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$w -o $w -- python3 bench.py --workload $w --steps 5 --warmup 2 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log)"
done
PMC_OUT=$D/pmc_c5x BENCH_ARGS="--workload c5x" bash tools/pmc.sh > $D/pmc_c5x.log 2>&1 || { tail -20 $D/pmc_c5x.log; exit 1; }
echo pmc ok
