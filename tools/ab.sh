#!/bin/bash
# A/B bench runs: tools/ab.sh TAG "ENV=a" "ENV=b" ...   (each: bench JSON -> gpurun_out/ab_TAG_i.log)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
i=0
for E in "$@"; do
  i=$((i+1))
  echo "$E" > $R/gpurun_out/ab_${TAG}_$i.log
  env $E timeout -k 10 200 python bench.py --cpu-sample-s 0 ${BENCH_ARGS:-} >> $R/gpurun_out/ab_${TAG}_$i.log 2>&1 || { echo "ab $i failed"; exit 1; }
done
echo ab done
