#!/bin/bash
# round 4: n_fft 4096 exchange swizzle — 4096 parity, C5x / C5 bench, C5x PMC
set -o pipefail
D=gpurun_out/r4f; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "4096 or c5 or C5 or xfade" tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_gpu_compositions.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for w in c5x c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PMC_OUT=$D/pmc_c5x BENCH_ARGS="--workload c5x" bash tools/pmc.sh > $D/pmc_c5x.log 2>&1 || { tail -20 $D/pmc_c5x.log; exit 1; }
python3 tools/pmc_summary.py $D/pmc_c5x k_stft_ola | grep "==\|BANK\|IDX_ACTIVE\|VALU/WAVE\|WAIT_ANY/"
