set -o pipefail
mkdir -p gpurun_out/r2v1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2v1/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r2v1/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2v1/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample-s 0 > gpurun_out/r2v1/prof.log 2>&1
