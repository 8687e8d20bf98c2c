#!/bin/bash
# round 3: C3 first transform waits for every group's statistics (vs chain), groups 2/4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-r3r}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_robustness.py tests/test_gpu_compositions.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
TOMATIS_C3_GROUPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/tr_g2 -o c3 -- python3 bench.py --workload c3 --steps 3 --warmup 2 --cpu-sample-s 0 > $D/tr_g2.log 2>&1 || { tail -20 $D/tr_g2.log; exit 1; }
python3 tools/timeline.py $(find $D/tr_g2 -name '*kernel_trace.csv' | head -1) > $D/timeline_g2.txt
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample-s 0 --workload c3 > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log) $(grep -o '"device_error": [0-9]*' $D/$n.log)"
}
b g2_first TOMATIS_C3_GROUPS=2
b g2_chain TOMATIS_C3_GROUPS=2 TOMATIS_C3_SYNC=chain
b g4_first TOMATIS_C3_GROUPS=4
b g3_first TOMATIS_C3_GROUPS=3
b g2_first_b TOMATIS_C3_GROUPS=2
b g2_chain_b TOMATIS_C3_GROUPS=2 TOMATIS_C3_SYNC=chain
b g4_first_b TOMATIS_C3_GROUPS=4
