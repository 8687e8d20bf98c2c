#!/bin/bash
# round 4: device FLAC decoder — equality with the host decoder, then file -> file
set -o pipefail
D=gpurun_out/r4l; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_flac_decode.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 500 python -u tools/bench_file.py > $D/bench_file.log 2>&1 || { tail -20 $D/bench_file.log; exit 1; }
tail -1 $D/bench_file.log
