#!/bin/bash
# Quick fabric-step kernel timing on the GPU box: kernel trace + stats only.
# Usage: bash profiles/quick_fabric.sh <tag>
set -e
R=$(pwd)
TAG=${1:-q}
OUT=$R/gpurun_out/quick_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3 > $OUT/bench.json
cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
head -6 $OUT/kernel_stats.csv
