set -o pipefail
D=gpurun_out/r2v12; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compositions.py tests/test_gpu_level_stats.py -x -q --timeout 300 --timeout-method thread -k "minhold or adapt or gate_api or C3 or c3 or mixed or level_stats" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -3 $D/tests.log
timeout -k 10 300 python -u tools/prof_c3.py > $D/prof_c3.log 2>&1 || { tail -20 $D/prof_c3.log; exit 1; }
tail -1 $D/prof_c3.log
