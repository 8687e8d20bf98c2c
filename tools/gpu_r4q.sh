#!/bin/bash
# round 4: fast look-back walk in k_gate_carry (gc1) vs gc0 -- parity, kernel stats, A/B
set -o pipefail
D=gpurun_out/r4q; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TOMATIS_HIP_LIB=$PWD/variants/gc2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused_levels.py > $D/fused_tests.log 2>&1 || { tail -30 $D/fused_tests.log; exit 1; }
tail -1 $D/fused_tests.log
for v in gc1 gc2; do
  TOMATIS_HIP_LIB=$PWD/variants/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$v -o c2 -- python3 bench.py --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof_$v.log 2>&1 || { tail -20 $D/prof_$v.log; exit 1; }
  echo "$v $(grep -h k_gate_carry $D/prof_$v/*kernel_stats.csv | cut -d, -f3-4)"
done
NOSMOKE=1 bash tools/ab_libs.sh r4q/ab2 variants/gc0.so variants/gc2.so variants/gc1.so variants/gc0.so variants/gc2.so
