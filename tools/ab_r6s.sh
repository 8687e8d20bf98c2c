#!/bin/bash
# wave-priority follow-ups: the 4096 two-wave trade at priority 2 (c5x), and the
# C2 gate priority held through the inverse FFT; same box.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6s}
B=tomatis_audio_processor_amd/libtomatis_hip.so
BENCH_ARGS="--single-steps 0 --workload c5x" bash tools/ab_libs.sh $TAG/c5x $B abx/libx_prio_trade.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0 --workload c5x" bash tools/ab_libs.sh $TAG/c5x $B abx/libx_prio_trade.so || exit 1
BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_prio_wide.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_prio_wide.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0 --workload c4" bash tools/ab_libs.sh $TAG/c4 $B abx/libx_prio_wide.so || exit 1
echo ab done
