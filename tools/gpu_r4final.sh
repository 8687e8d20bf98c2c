#!/bin/bash
# round 4 final pass: GPU suite, smoke, every workload, file path, kernel stats, PMC
set -o pipefail
T=${1:-r4final}
bash tools/gpu_r4d.sh $T/suite || exit 1
timeout -k 10 500 python -u tools/bench_file.py > gpurun_out/$T/suite/bench_file.log 2>&1 || { tail -20 gpurun_out/$T/suite/bench_file.log; exit 1; }
tail -1 gpurun_out/$T/suite/bench_file.log | cut -c1-300
bash tools/gpu_r4e.sh $T/prof || exit 1
