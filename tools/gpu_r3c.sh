#!/bin/bash
# round 3: layer-2 on the device file path (CLI test + file timing)
set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cli.py > gpurun_out/r3c/cli.log 2>&1; rc=$?; echo "cli rc=$rc"; tail -4 gpurun_out/r3c/cli.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_layer2_file.py > gpurun_out/r3c/bench_layer2_file.log 2>&1; echo "l2 rc=$?"; tail -2 gpurun_out/r3c/bench_layer2_file.log
