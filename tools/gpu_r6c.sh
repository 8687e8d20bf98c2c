#!/bin/bash
# round-6 lease C: level / parity tests on the new k_leaves, the host chain
# probe, C5x / C3 / C2 benches -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6c}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_level_stats.py tests/test_gpu_fused_levels.py tests/test_gpu_parity.py tests/test_gpu_anysize.py tests/test_gpu_runs.py tests/test_gpu_robustness.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/level_tests.log 2>&1 || { tail -60 $D/level_tests.log; exit 1; }
tail -1 $D/level_tests.log
python3 tools/pinned_probe.py > $D/pinned_probe.log 2>&1; cat $D/pinned_probe.log
for w in c5x c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log | head -2 | tr '\n' ' ') $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c5x -o c5x -- python3 bench.py --workload c5x --steps 10 --warmup 2 --cpu-sample-s 0 --single-steps 0 > $D/prof_c5x.log 2>&1 || { tail -20 $D/prof_c5x.log; exit 1; }
echo ok
