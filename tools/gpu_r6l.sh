#!/bin/bash
# C2 bench + rocprofv3 kernel stats (look-back duration check).  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6l}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 200 python -u bench.py --cpu-sample-s 0 --single-steps 0 > $D/b_c2.log 2>&1 || { tail -20 $D/b_c2.log; exit 1; }
echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $D/b_c2.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/b_c2.log)"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 20 --cpu-sample-s 0 --single-steps 0 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
echo prof ok
