#!/bin/bash
# n_fft 4096 level-fusion cost (TM_EXP_LV4096, results unchanged: the extra level
# arithmetic only feeds a never-taken row override) on c5x, same box.
set -o pipefail
TAG=${1:-r6f}
B=tomatis_audio_processor_amd/libtomatis_hip.so
BENCH_ARGS="--workload c5x" bash tools/ab_libs.sh $TAG/c5x $B abx/libx_lv4096.so || exit 1
NOSMOKE=1 BENCH_ARGS="--workload c5x" bash tools/ab_libs.sh $TAG/c5x $B abx/libx_lv4096.so $B abx/libx_lv4096.so || exit 1
NOSMOKE=1 BENCH_ARGS="--workload c5x --input-gain 0.05" bash tools/ab_libs.sh $TAG/c5xq $B abx/libx_lv4096.so $B abx/libx_lv4096.so || exit 1
echo ab done
