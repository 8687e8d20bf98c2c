#!/bin/bash
# round 3: any-size transform (Bluestein, HBM buffers, many channels) + parity suite
set -o pipefail
D=gpurun_out/${1:-r3d}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_anysize.py tests/test_gpu_parity.py > $D/anysize.log 2>&1; rc=$?
tail -5 $D/anysize.log; exit $rc
