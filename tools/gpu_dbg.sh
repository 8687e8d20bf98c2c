#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python -u tools/dbg_r2.py > gpurun_out/dbg.log 2>&1 || { tail -30 gpurun_out/dbg.log; exit 1; }

cat gpurun_out/dbg.log
