set -o pipefail
D=gpurun_out/r2v13; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_timeshard.py tests/test_gpu_parity.py tests/test_gpu_fileio.py -x -q --timeout 120 --timeout-method thread -k "timeshard or fused or alpha_long or fileio or flac or std_48k" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
TOMATIS_RUN_ROUNDS=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timeshard.py -x -q --timeout 120 --timeout-method thread -k "fused or alpha_long or std_48k or bit_identical" >> $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
BENCH_ARGS="--workload c2 --steps 20" bash tools/ab.sh c2r "TOMATIS_RUN_ROUNDS=1" "TOMATIS_RUN_ROUNDS=2" "TOMATIS_RUN_ROUNDS=3" "TOMATIS_RUN_ROUNDS=4" || exit 1
BENCH_ARGS="--workload c3 --steps 10" bash tools/ab.sh c3r "TOMATIS_RUN_ROUNDS=1" "TOMATIS_RUN_ROUNDS=2" "TOMATIS_RUN_ROUNDS=4" "TOMATIS_RUN_ROUNDS=6" || exit 1
BENCH_ARGS="--workload c2ts --steps 20" bash tools/ab.sh c2ts "TOMATIS_RUN_ROUNDS=1" || exit 1
for f in gpurun_out/ab_c2r_*.log gpurun_out/ab_c3r_*.log gpurun_out/ab_c2ts_*.log; do echo "$f $(head -1 $f) $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f) $(grep -o '"frac": [0-9.]*' $f | head -1)"; done
timeout -k 10 400 python -u tools/bench_file.py > $D/bench_file.log 2>&1 || { tail -20 $D/bench_file.log; exit 1; }
tail -1 $D/bench_file.log
