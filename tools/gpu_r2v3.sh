set -o pipefail
mkdir -p gpurun_out/r2v3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2v3/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r2v3/gpu_tests.log
exit $rc
