#!/bin/bash
# round 4: two-round limiter -- new tests, parity tests, C2 bench (limited + quiet), C4
set -o pipefail
D=gpurun_out/r4a; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_limiter_rounds.py tests/test_gpu_parity.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 > $D/c2.log 2>&1 || { tail -20 $D/c2.log; exit 1; }
echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $D/c2.log) $(grep -o '"kernel_ms": [0-9.]*' $D/c2.log) $(grep -o '"device_error": [0-9]*' $D/c2.log)"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 --input-gain 0.05 > $D/c2q.log 2>&1 || { tail -20 $D/c2q.log; exit 1; }
echo "c2q $(grep -o '"ms_per_step": [0-9.]*' $D/c2q.log) $(grep -o '"kernel_ms": [0-9.]*' $D/c2q.log)"
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 3 --cpu-sample-s 0 > $D/c4.log 2>&1 || { tail -20 $D/c4.log; exit 1; }
echo "c4 $(grep -o '"ms_per_step": [0-9.]*' $D/c4.log) $(grep -o '"kernel_ms": [0-9.]*' $D/c4.log)"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs head -8
