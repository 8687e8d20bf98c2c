#!/bin/bash
# Round-6 experiment A/B on one box (tools/ab_libs.sh per variant):
#  libx_rev  : partner blocks rescaled in reverse list order (correct results)
#  libx_b128 : 16-byte frame loads / stores without the permutation (timing only)
# then FETCH_SIZE passes of base vs rev (C2 limited, c5x).  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6e}
B=tomatis_audio_processor_amd/libtomatis_hip.so
bash tools/ab_libs.sh $TAG/c2 $B abx/libx_rev.so || exit 1
NOSMOKE=1 bash tools/ab_libs.sh $TAG/c2 abx/libx_b128.so $B abx/libx_rev.so abx/libx_b128.so || exit 1
NOSMOKE=1 BENCH_ARGS="--input-gain 0.05" bash tools/ab_libs.sh $TAG/quiet $B abx/libx_b128.so $B abx/libx_b128.so || exit 1
NOSMOKE=1 BENCH_ARGS="--workload c5x" bash tools/ab_libs.sh $TAG/c5x $B abx/libx_rev.so $B abx/libx_rev.so || exit 1
for L in $B abx/libx_rev.so; do
  n=$(basename $L .so)
  TOMATIS_HIP_LIB=$PWD/$L BENCH_ARGS="--steps 4" bash tools/pmc_fetch.sh ${TAG}_c2_$n || exit 1
  TOMATIS_HIP_LIB=$PWD/$L BENCH_ARGS="--steps 4 --workload c5x" bash tools/pmc_fetch.sh ${TAG}_c5x_$n || exit 1
done
echo ab done
