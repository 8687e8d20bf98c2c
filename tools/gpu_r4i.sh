#!/bin/bash
# round 4: device FLAC encoder — byte equality with the host encoder
set -o pipefail
D=gpurun_out/r4i; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_flac_device.py > $D/tests.log 2>&1; rc=$?
tail -30 $D/tests.log
exit $rc
