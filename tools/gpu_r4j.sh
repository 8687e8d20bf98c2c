#!/bin/bash
# round 4: C2 file -> file with the device FLAC encoder
set -o pipefail
D=gpurun_out/r4j; mkdir -p $D
timeout -k 10 500 python -u tools/bench_file.py > $D/bench_file.log 2>&1 || { tail -20 $D/bench_file.log; exit 1; }
tail -1 $D/bench_file.log
