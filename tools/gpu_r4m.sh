#!/bin/bash
# round 4: level-code variants of the fused C2 kernel -- parity first, then A/B
set -o pipefail
D=gpurun_out/r4m; mkdir -p $D
V=${V:-variants/v1.so}
TOMATIS_HIP_LIB=$PWD/$V timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused_levels.py > $D/fused_tests.log 2>&1 || { tail -30 $D/fused_tests.log; exit 1; }
tail -1 $D/fused_tests.log
bash tools/ab_libs.sh r4m/loud variants/base.so variants/v1.so $V || exit 1
NOSMOKE=1 BENCH_ARGS="--input-gain 0.05" bash tools/ab_libs.sh r4m/quiet variants/base.so variants/v1.so $V || exit 1
NOSMOKE=1 bash tools/ab_libs.sh r4m/loud2 $V variants/v1.so variants/base.so
