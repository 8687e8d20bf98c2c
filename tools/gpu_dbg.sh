#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python -u tools/dbg_fdd.py > gpurun_out/dbg.log 2>&1; rc=$?; tail -30 gpurun_out/dbg.log; exit $rc
