set -o pipefail
mkdir -p gpurun_out/r2v5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2v5/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|Error|error" gpurun_out/r2v5/gpu_tests.log | head -20
tail -3 gpurun_out/r2v5/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r2v5/bench.log 2>&1; tail -1 gpurun_out/r2v5/bench.log
