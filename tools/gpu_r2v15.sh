set -o pipefail
D=gpurun_out/r2v15; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_compositions.py -x -q --timeout 300 --timeout-method thread -k "c3" > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for w in c3; do timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --cpu-sample-s 0 > $D/bench_$w.log 2>&1 || { tail -20 $D/bench_$w.log; exit 1; }; echo "$w $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log) $(grep -o '"kernel_ms": [0-9.]*' $D/bench_$w.log) $(grep -o '"frac": [0-9.]*' $D/bench_$w.log | head -1)"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/tr -o c3 -- python3 bench.py --workload c3 --steps 3 --warmup 1 --cpu-sample-s 0 > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
echo traced
