#!/bin/bash
# round 4: per-wave xfade alpha passes — xfade / C5 tests, C5x / C5 bench, kernel stats
set -o pipefail
D=gpurun_out/r4g; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "xfade or c5 or C5 or alpha" tests/ -m gpu > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for w in c5x c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c5x -o c5x -- python3 bench.py --workload c5x --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof_c5x.log 2>&1 || { tail -20 $D/prof_c5x.log; exit 1; }
find $D/prof_c5x -name "*kernel_stats.csv" | head -1 | xargs head -12 | cut -d, -f1-4 | cut -c1-150
