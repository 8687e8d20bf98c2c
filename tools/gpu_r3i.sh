#!/bin/bash
# round 3: work-list overheads on quiet input (no chunk limited)
set -o pipefail
D=gpurun_out/${1:-r3i}; mkdir -p $D
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 $BA > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log)"
}
BA="--input-gain 0.05"
b q_static TOMATIS_DYN=0
b q_list TOMATIS_DYN=1
b q_list_nofuse TOMATIS_FUSE_LIMITER=0
b q_list_151 TOMATIS_RUN_FRAMES=151 TOMATIS_RUN_TAIL=151
b q_list_151_nofuse TOMATIS_RUN_FRAMES=151 TOMATIS_RUN_TAIL=151 TOMATIS_FUSE_LIMITER=0
b q_list_96_96_nofuse TOMATIS_RUN_FRAMES=96 TOMATIS_RUN_TAIL=96 TOMATIS_FUSE_LIMITER=0
b q_static_nofuse TOMATIS_DYN=0 TOMATIS_FUSE_LIMITER=0
BA=""
b l_static TOMATIS_DYN=0
b l_list_lag3 TOMATIS_RESCALE_LAG=3
b l_list_lag2_s256 TOMATIS_RESCALE_LAG=2 TOMATIS_SLICE_KB=256
