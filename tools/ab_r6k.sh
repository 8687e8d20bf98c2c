#!/bin/bash
# gate look-back prefetch depth (TM_GC_PFD 4 / 8 / 16) on C2 and C4, same box,
# with rocprofv3 kernel stats of k_gate_carry.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6k}
D=gpurun_out/$TAG; mkdir -p $D
B=tomatis_audio_processor_amd/libtomatis_hip.so
BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_pfd8.so abx/libx_pfd16.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_pfd8.so abx/libx_pfd16.so || exit 1
NOSMOKE=1 BENCH_ARGS="--workload c4 --single-steps 0" bash tools/ab_libs.sh $TAG/c4 $B abx/libx_pfd8.so abx/libx_pfd16.so || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in $B abx/libx_pfd8.so abx/libx_pfd16.so; do
  n=$(basename $L .so)
  TOMATIS_HIP_LIB=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$n -o run -- python3 bench.py --steps 20 --cpu-sample-s 0 --single-steps 0 > $D/prof_$n.log 2>&1 || { tail -20 $D/prof_$n.log; exit 1; }
  f=$(find $D/prof_$n -name "*kernel_stats.csv" | head -1)
  echo "$n $(grep k_gate_carry $f | cut -d, -f2-4)"
done
