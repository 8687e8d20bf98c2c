# round-3 quick check: full GPU suite + C2 bench line (device_error in the JSON)
set -o pipefail
D=gpurun_out/${1:-r3a}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --cpu-sample-s 0 > $D/bench_c2.log 2>&1 || { tail -20 $D/bench_c2.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"device_error": [0-9]*' $D/bench_c2.log
