#!/bin/bash
# s_setprio experiments on the C2 interior loop (memory-issue phase / gate
# latency chain at priority 2), same box, limited and quiet input.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6q}
B=tomatis_audio_processor_amd/libtomatis_hip.so
BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_prio_MEM.so abx/libx_prio_GATE.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0" bash tools/ab_libs.sh $TAG/c2 $B abx/libx_prio_MEM.so abx/libx_prio_GATE.so || exit 1
NOSMOKE=1 BENCH_ARGS="--single-steps 0 --input-gain 0.05" bash tools/ab_libs.sh $TAG/quiet $B abx/libx_prio_MEM.so abx/libx_prio_GATE.so || exit 1
echo ab done
