#!/bin/bash
# round 4: A/B of the two-round limiter variants (C2 limited, then quiet), kernel stats
set -o pipefail
D=gpurun_out/r4b; mkdir -p $D
bash tools/ab_libs.sh r4b tomatis_audio_processor_amd/libtomatis_hip.so variants/lib_tailonly.so || exit 1
BENCH_ARGS="--input-gain 0.05" NOSMOKE=1 bash tools/ab_libs.sh r4b_q tomatis_audio_processor_amd/libtomatis_hip.so || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-200
