#!/bin/bash
# After the two-wave trade's priority change (n_fft 4096 kernels only): full
# GPU suite + smoke, the C5 workloads, rocprofv3 stats and PMC of c5x.
# -> gpurun_out/TAG
set -o pipefail
TAG=${1:-final4}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -n 1 $D/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -n 1 $D/smoke.log
for w in c5x c5; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log | head -2 | tr '\n' ' ') $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c5x -o c5x -- python3 bench.py --workload c5x --cpu-sample-s 0 > $D/prof_c5x.log 2>&1 || { tail -20 $D/prof_c5x.log; exit 1; }
PMC_OUT=$D/pmc_c5x BENCH_ARGS="--steps 4 --workload c5x" bash tools/pmc.sh > $D/pmc_c5x.log 2>&1 || { tail -20 $D/pmc_c5x.log; exit 1; }
echo prof ok
