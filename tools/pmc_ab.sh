#!/bin/bash
# SQ / LDS / instruction-fetch counter passes of the fused kernel for library
# variants (diagnostic): tools/pmc_ab.sh TAG lib1.so lib2.so ...
# -> gpurun_out/TAG/<lib>/p*/ ; BENCH_ARGS as bench.py flags (e.g. --input-gain 0.05)
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=$1; shift
ARGS="bench.py --steps 2 --warmup 1 --cpu-sample-s 0 ${BENCH_ARGS:-}"
for L in "$@"; do
  n=$(basename $L .so)
  OUT=$R/gpurun_out/$TAG/$n; mkdir -p $OUT
  i=0
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQ_INST_LEVEL_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_IFETCH" \
           "SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH_LEVEL SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    TOMATIS_HIP_LIB=$R/$L timeout -k 10 120 rocprofv3 --pmc $C -d $OUT/p$i -o run --output-format csv -- python3 $ARGS > $OUT/p$i.log 2>&1 || { echo "$n pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  echo "$n pmc done"
done
