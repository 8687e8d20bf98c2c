#!/bin/bash
# PMC passes for the fused kernel (run on the GPU box from the repo root).
# Separate passes: SQ timing counters, LDS counters, FETCH_SIZE, WRITE_SIZE.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=${PMC_OUT:-$R/gpurun_out/pmc}
mkdir -p $OUT
ARGS="bench.py --steps 2 --warmup 1 --cpu-sample-s 0 ${BENCH_ARGS:-}"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C -d $OUT/p$i -o run --output-format csv -- python3 $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc done
