#!/bin/bash
# look-back prefetch depth 2 vs 4 (b64 walk): C2 bench and rocprofv3 look-back
# duration, loud and quiet input, same box.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6p}
D=gpurun_out/$TAG; mkdir -p $D
B=tomatis_audio_processor_amd/libtomatis_hip.so
BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_pfd2.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_pfd2.so || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in $B abx/libx_pfd2.so; do
  n=$(basename $L .so)
  for g in 1.0 0.05; do
    TOMATIS_HIP_LIB=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_${n}_$g -o run -- python3 bench.py --steps 20 --cpu-sample-s 0 --single-steps 0 --input-gain $g > $D/prof_${n}_$g.log 2>&1 || { tail -20 $D/prof_${n}_$g.log; exit 1; }
  done
done
echo prof ok
