set -o pipefail
D=gpurun_out/r2v10; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_level_stats.py tests/test_gpu_parity.py tests/test_gpu_compositions.py -x -q --timeout 120 --timeout-method thread -k "level_stats or adapt or C3 or c3 or mixed" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 300 python -u tools/prof_c3.py > $D/prof_c3.log 2>&1 || { tail -20 $D/prof_c3.log; exit 1; }
tail -1 $D/prof_c3.log
TOMATIS_FUSE_LIMITER=0 timeout -k 10 300 python -u tools/prof_c3.py > $D/prof_c3_nofuse.log 2>&1 || { tail -20 $D/prof_c3_nofuse.log; exit 1; }
tail -1 $D/prof_c3_nofuse.log
