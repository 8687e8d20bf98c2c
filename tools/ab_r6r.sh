#!/bin/bash
# s_setprio around the in-kernel gate (level 2 / 3) and from the gate through
# the forward FFT, C2 limited / quiet and C4, same box.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6r}
B=tomatis_audio_processor_amd/libtomatis_hip.so
V="abx/libx_prio_G2.so abx/libx_prio_G3.so abx/libx_prio_GF.so"
BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B $V || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B $V || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0 --input-gain 0.05" bash tools/ab_libs.sh $TAG/quiet $B $V || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0 --workload c4" bash tools/ab_libs.sh $TAG/c4 $B $V || exit 1
echo ab done
