set -o pipefail
D=gpurun_out/r2v11; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
timeout -k 10 300 python -u tools/prof_c3.py > $D/prof_c3.log 2>&1 || { tail -20 $D/prof_c3.log; exit 1; }
tail -1 $D/prof_c3.log
TOMATIS_GAIN_LDS=0 timeout -k 10 300 python -u tools/prof_c3.py > $D/prof_c3_nolds.log 2>&1 || { tail -20 $D/prof_c3_nolds.log; exit 1; }
tail -1 $D/prof_c3_nolds.log
for w in c3 c5x c2; do timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }; tail -1 $D/bench_$w.log | cut -c1-400; done
