#!/bin/bash
# round 3: why is the dynamic kernel slower?  quiet-input variants + SQ counters
set -o pipefail
D=gpurun_out/${1:-r3g}; mkdir -p $D
b() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample-s 0 --input-gain 0.05 > $D/$n.log 2>&1 || { tail -20 $D/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $D/$n.log) $(grep -o '"kernel_ms": [0-9.]*' $D/$n.log)"
}
b q_dyn_151 TOMATIS_RUN_FRAMES=151 TOMATIS_RUN_TAIL=151
b q_dyn_nofuse TOMATIS_FUSE_LIMITER=0
b q_dyn TOMATIS_DYN=1
export TMPDIR=/tmp
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_FLAT"; do
  for m in 0 1; do
    i=$((i+1))
    TOMATIS_DYN=$m timeout -k 10 240 rocprofv3 --pmc $C -d $D/pmc$m/p$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-sample-s 0 --input-gain 0.05 > $D/pmc$m.p$i.log 2>&1 || { echo "pmc $m $i failed"; tail -5 $D/pmc$m.p$i.log; exit 1; }
  done
done
echo pmc ok
