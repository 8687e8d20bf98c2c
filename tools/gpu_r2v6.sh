set -o pipefail
mkdir -p gpurun_out/r2v6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2v6/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|Error" gpurun_out/r2v6/gpu_tests.log | head -20
tail -3 gpurun_out/r2v6/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_file.py > gpurun_out/r2v6/bench_file.log 2>&1; tail -3 gpurun_out/r2v6/bench_file.log
