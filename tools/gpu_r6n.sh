#!/bin/bash
# look-back duration on loud vs quiet C2 input (rocprofv3 kernel stats), and
# the torchrun path at N=1 with the default step count.  -> gpurun_out/TAG
set -o pipefail
TAG=${1:-r6n}
D=gpurun_out/$TAG; mkdir -p $D
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --cpu-sample-s 0 --single-steps 0 > $D/torchrun_n1.log 2>&1 || { tail -20 $D/torchrun_n1.log; exit 1; }
echo "torchrun n1 $(grep -o '"ms_per_step": [0-9.]*' $D/torchrun_n1.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $D/torchrun_n1.log)"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in 1.0 0.05 0.3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$g -o run -- python3 bench.py --steps 20 --cpu-sample-s 0 --single-steps 0 --input-gain $g > $D/prof_$g.log 2>&1 || { tail -20 $D/prof_$g.log; exit 1; }
done
echo prof ok
