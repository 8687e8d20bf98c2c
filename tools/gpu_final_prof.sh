#!/bin/bash
# Final evidence, lease part 2: rocprofv3 kernel stats (C2 default bench
# command without the CPU legs, C5x) and PMC passes (C2 limited / quiet, C5x;
# 4 timed passes so the steady-state pipelined launch dominates)
set -o pipefail
TAG=${1:-final}
D=gpurun_out/$TAG; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --cpu-sample-s 0 > $D/prof_c2.log 2>&1 || { tail -20 $D/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c5x -o c5x -- python3 bench.py --workload c5x --cpu-sample-s 0 > $D/prof_c5x.log 2>&1 || { tail -20 $D/prof_c5x.log; exit 1; }
PMC_OUT=$D/pmc BENCH_ARGS="--steps 4" bash tools/pmc.sh > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
PMC_OUT=$D/pmc_quiet BENCH_ARGS="--steps 4 --input-gain 0.05" bash tools/pmc.sh > $D/pmc_quiet.log 2>&1 || { tail -20 $D/pmc_quiet.log; exit 1; }
PMC_OUT=$D/pmc_c5x BENCH_ARGS="--steps 4 --workload c5x" bash tools/pmc.sh > $D/pmc_c5x.log 2>&1 || { tail -20 $D/pmc_c5x.log; exit 1; }
echo prof ok
