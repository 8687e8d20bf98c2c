set -o pipefail
D=gpurun_out/r2v9; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c3prof -o c3 -- python3 bench.py --workload c3 --steps 5 --warmup 2 --cpu-sample-s 0 > $D/c3prof.log 2>&1 || { tail -20 $D/c3prof.log; exit 1; }
find $D/c3prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
