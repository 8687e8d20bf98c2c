set -o pipefail
D=gpurun_out/r2v16; mkdir -p $D
timeout -k 10 120 python -u tools/log10_probe.py > $D/log10.log 2>&1 || { tail -20 $D/log10.log; exit 1; }
cat $D/log10.log
BENCH_ARGS="--workload c3 --steps 10" bash tools/ab.sh c3g "TOMATIS_C3_GROUPS=1" "TOMATIS_C3_GROUPS=2" "TOMATIS_C3_GROUPS=1 TOMATIS_RUN_ROUNDS=8" "TOMATIS_C3_GROUPS=1 TOMATIS_RUN_ROUNDS=12" "TOMATIS_C3_GROUPS=1 TOMATIS_RUN_ROUNDS=16" "TOMATIS_C3_GROUPS=1 TOMATIS_LOG10_THREADS=8" || exit 1
for f in gpurun_out/ab_c3g_*.log; do echo "$f $(head -1 $f) $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f)"; done
timeout -k 10 300 python -u tools/prof_c3.py > $D/prof_c3.log 2>&1 || { tail -20 $D/prof_c3.log; exit 1; }
tail -1 $D/prof_c3.log
