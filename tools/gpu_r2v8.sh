set -o pipefail
D=gpurun_out/r2v8; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_c3.log 2>&1 || { tail -20 $D/bench_c3.log; exit 1; }
tail -1 $D/bench_c3.log
timeout -k 10 400 python -u tools/bench_file.py > $D/bench_file.log 2>&1 || { tail -20 $D/bench_file.log; exit 1; }
tail -1 $D/bench_file.log
