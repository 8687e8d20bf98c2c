set -o pipefail
mkdir -p gpurun_out/r2v4
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_compositions.py tests/test_gpu_timeshard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2v4/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2v4/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2v4/gpu_tests.log
bash tools/ab.sh rounds "TOMATIS_ROUNDS=1" "TOMATIS_ROUNDS=2" "TOMATIS_ROUNDS=3" "TOMATIS_ROUNDS=4" "TOMATIS_ROUNDS=6" && \
bash tools/ab.sh exp "TOMATIS_HIP_LIB=exp/lib_nosync.so" "TOMATIS_HIP_LIB=exp/lib_compute.so" "TOMATIS_HIP_LIB=exp/lib_nosync_compute.so" "TOMATIS_FUSE_LIMITER=0 TOMATIS_ROUNDS=1" && \
BENCH_ARGS="--workload c4 --steps 5" bash tools/ab.sh c4 "TOMATIS_ROUNDS=1" "TOMATIS_ROUNDS=3"
for f in gpurun_out/ab_*.log; do echo "$f $(head -1 $f) $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f)"; done
