#!/bin/bash
# round 4: kernel stats of the final code (C2, C4)
set -o pipefail
D=gpurun_out/r4s; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c4 -o c4 -- python3 bench.py --workload c4 --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof_c4.log 2>&1 || { tail -20 $D/prof_c4.log; exit 1; }
tail -1 $D/prof.log | cut -c1-200
