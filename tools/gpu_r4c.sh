#!/bin/bash
# round 4: fused levels + gate (tomatis_stft_ola_gated) — parity, then C2 A/B
set -o pipefail
D=gpurun_out/r4c; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused_levels.py > $D/fused.log 2>&1 || { tail -40 $D/fused.log; exit 1; }
tail -3 $D/fused.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_limiter_rounds.py tests/test_gpu_runs.py > $D/parity.log 2>&1 || { tail -40 $D/parity.log; exit 1; }
tail -2 $D/parity.log
for V in "" "--dev FUSED_LEVELS=0"; do
  for G in 1.0 0.05; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 --input-gain $G $V > $D/b.log 2>&1 || { tail -20 $D/b.log; exit 1; }
    echo "[$V g=$G] $(grep -o '"ms_per_step": [0-9.]*' $D/b.log) $(grep -o '"kernel_ms": [0-9.]*' $D/b.log) $(grep -o '"fused_levels": [a-z]*' $D/b.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --steps 10 --warmup 3 --cpu-sample-s 0 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -c1-220
