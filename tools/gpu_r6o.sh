#!/bin/bash
# look-back fast walk with 16-byte loads: gate tests, C2 / C4 bench, look-back
# duration (rocprofv3) on loud and quiet input.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6o}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused_levels.py tests/test_gpu_fused_levels_4096.py tests/test_gpu_pipelined.py tests/test_gpu_as_benched.py -x -q --timeout 400 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -n 1 $D/tests.log
for w in c2 c4 c4allh; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample-s 0 --single-steps 0 > $D/b_$w.log 2>&1 || { tail -20 $D/b_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/b_$w.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/b_$w.log) $(grep -o '"gate_fallbacks": [0-9]*' $D/b_$w.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in 1.0 0.3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$g -o run -- python3 bench.py --steps 20 --cpu-sample-s 0 --single-steps 0 --input-gain $g > $D/prof_$g.log 2>&1 || { tail -20 $D/prof_$g.log; exit 1; }
done
echo prof ok
