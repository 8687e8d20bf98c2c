#!/bin/bash
# round 4: v3 (rsq sqrt + per-frame lane addresses) vs v1 -- parity, then A/B
set -o pipefail
D=gpurun_out/r4p; mkdir -p $D
TOMATIS_HIP_LIB=$PWD/variants/v3.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused_levels.py > $D/fused_tests.log 2>&1 || { tail -30 $D/fused_tests.log; exit 1; }
tail -1 $D/fused_tests.log
bash tools/ab_libs.sh r4p/loud variants/v1.so variants/v3.so || exit 1
NOSMOKE=1 BENCH_ARGS="--input-gain 0.05" bash tools/ab_libs.sh r4p/quiet variants/v1.so variants/v3.so || exit 1
NOSMOKE=1 bash tools/ab_libs.sh r4p/loud2 variants/v3.so variants/v1.so
NOSMOKE=1 BENCH_ARGS="--input-gain 0.05" bash tools/ab_libs.sh r4p/quiet2 variants/v3.so variants/v1.so
