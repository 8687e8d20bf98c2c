#!/bin/bash
# round 4: FLAC device decode + encode tests
set -o pipefail
mkdir -p gpurun_out/r4n
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_flac_decode.py tests/test_gpu_flac_device.py > gpurun_out/r4n/flac_tests.log 2>&1 || { tail -30 gpurun_out/r4n/flac_tests.log; exit 1; }
tail -1 gpurun_out/r4n/flac_tests.log
