set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2v2
timeout -k 10 120 rocprofv3 -L > gpurun_out/r2v2/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2v2/ktrace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-sample-s 0 > gpurun_out/r2v2/ktrace.log 2>&1 && \
bash tools/pmc.sh > gpurun_out/r2v2/pmc.log 2>&1
