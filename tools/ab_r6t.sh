#!/bin/bash
# the inverse FFT's LDS transpose at raised priority (n_fft 2048 kernels), same box.
set -o pipefail
TAG=${1:-r6t}
B=tomatis_audio_processor_amd/libtomatis_hip.so
BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_prio_ix.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_prio_ix.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0 --workload c4" bash tools/ab_libs.sh $TAG/c4 $B abx/libx_prio_ix.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0 --workload c3" bash tools/ab_libs.sh $TAG/c3 $B abx/libx_prio_ix.so || exit 1
echo ab done
