#!/bin/bash
# kernel stats (C2, C5x) and PMC passes (C2 loud / quiet, C5x)
set -o pipefail
TAG=${1:-prof}
D=gpurun_out/$TAG; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c5x -o c5x -- python3 bench.py --workload c5x --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof_c5x.log 2>&1 || { tail -20 $D/prof_c5x.log; exit 1; }
PMC_OUT=$D/pmc bash tools/pmc.sh > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
PMC_OUT=$D/pmc_quiet BENCH_ARGS="--input-gain 0.05" bash tools/pmc.sh > $D/pmc_quiet.log 2>&1 || { tail -20 $D/pmc_quiet.log; exit 1; }
PMC_OUT=$D/pmc_c5x BENCH_ARGS="--workload c5x" bash tools/pmc.sh > $D/pmc_c5x.log 2>&1 || { tail -20 $D/pmc_c5x.log; exit 1; }
echo pmc ok
