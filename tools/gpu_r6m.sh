#!/bin/bash
# Spread and coverage runs: the C2 bench five times on one box, the torchrun
# path at N=1 (RCCL initialised, one rank), rocprofv3 kernel stats of C3 and
# C4.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6m}
D=gpurun_out/$TAG; mkdir -p $D
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --cpu-sample-s 0 --single-steps 0 > $D/c2_$i.log 2>&1 || { tail -20 $D/c2_$i.log; exit 1; }
  echo "c2 run $i $(grep -o '"ms_per_step": [0-9.]*' $D/c2_$i.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/c2_$i.log)"
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --cpu-sample-s 0 --single-steps 0 > $D/torchrun_n1.log 2>&1 || { tail -20 $D/torchrun_n1.log; exit 1; }
echo "torchrun n1 $(grep -o '"ms_per_step": [0-9.]*' $D/torchrun_n1.log | head -1) $(grep -o '"n_gpus": [0-9]*' $D/torchrun_n1.log)"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$w -o $w -- python3 bench.py --workload $w --steps 10 --cpu-sample-s 0 --single-steps 0 > $D/prof_$w.log 2>&1 || { tail -20 $D/prof_$w.log; exit 1; }
done
echo prof ok
