#!/bin/bash
# round-6 profiling lease: rocprofv3 kernel stats / traces for C2, C5x, C3 and
# a host profile of the multi-file batch runner -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6prof}
D=gpurun_out/$TAG; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c2 -o c2 -- python3 bench.py --cpu-sample-s 0 --single-steps 0 > $D/prof_c2.log 2>&1 || { tail -20 $D/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c5x -o c5x -- python3 bench.py --workload c5x --cpu-sample-s 0 --single-steps 0 > $D/prof_c5x.log 2>&1 || { tail -20 $D/prof_c5x.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c3 -o c3 -- python3 bench.py --workload c3 --steps 10 --warmup 2 --cpu-sample-s 0 --single-steps 0 > $D/prof_c3.log 2>&1 || { tail -20 $D/prof_c3.log; exit 1; }
TOMATIS_LOG10_THREADS=2 timeout -k 10 300 python3 bench.py --workload c3 --steps 20 --warmup 3 --cpu-sample-s 0 --single-steps 0 > $D/bench_c3_log10t2.log 2>&1 || { tail -20 $D/bench_c3_log10t2.log; exit 1; }
timeout -k 10 300 python3 bench.py --workload c3 --steps 20 --warmup 3 --cpu-sample-s 0 --single-steps 0 > $D/bench_c3_base.log 2>&1 || { tail -20 $D/bench_c3_base.log; exit 1; }
echo "c3 base $(grep -o '"ms_per_step": [0-9.]*' $D/bench_c3_base.log | head -1) log10 x2 $(grep -o '"ms_per_step": [0-9.]*' $D/bench_c3_log10t2.log | head -1)"
python3 tools/log10_threads.py > $D/log10_threads.log 2>&1
BATCH_FILES=16 BATCH_SECS=300 BATCH_GB=0.5 timeout -k 10 600 python3 -m cProfile -s cumtime tools/bench_batch.py > $D/bench_batch_cprofile.log 2>&1 || { tail -20 $D/bench_batch_cprofile.log; exit 1; }
grep -m1 workload $D/bench_batch_cprofile.log | cut -c1-400
echo prof ok
