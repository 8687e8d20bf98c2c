#!/bin/bash
# One measurement pass on the GPU box (gpurun): GPU tests, smoke, the bench
# lines, rocprofv3 kernel stats, PMC passes (limiter-active and quiet input),
# the file->file bench.  Everything under gpurun_out/$TAG.
set -o pipefail
TAG=${1:-round}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 600 python -u bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-300
for w in c3 c4 c5x c5 c2ts; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log) $(grep -o '"frac": [0-9.]*' $D/bench_$w.log | head -1)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
PMC_OUT=$D/pmc bash tools/pmc.sh > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
PMC_OUT=$D/pmc_quiet BENCH_ARGS="--input-gain 0.05" bash tools/pmc.sh > $D/pmc_quiet.log 2>&1 || { tail -20 $D/pmc_quiet.log; exit 1; }
echo pmc ok
timeout -k 10 400 python -u tools/bench_file.py > $D/bench_file.log 2>&1 || { tail -20 $D/bench_file.log; exit 1; }
tail -1 $D/bench_file.log
