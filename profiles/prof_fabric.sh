#!/bin/bash
# Fabric step profile (runs on the GPU box from the repo root): kernel trace
# + stats, then one PMC pass per counter group (FETCH_SIZE, WRITE_SIZE).
# Usage: bash profiles/prof_fabric.sh <tag>   -> gpurun_out/prof_<tag>/final/
set -e
R=$(pwd)
TAG=${1:-r02}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT/final
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
  python3 $B --steps 20 --warmup 3 > $OUT/trace_bench.json
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o run --output-format csv -- \
  python3 $B --steps 3 --warmup 1 > $OUT/pmc_fetch.json
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o run --output-format csv -- \
  python3 $B --steps 3 --warmup 1 > $OUT/pmc_write.json
cd $R
python3 profiles/collect_pmc.py $OUT/pmc_fetch $OUT/pmc_write $OUT/final/pmc_traffic.json
cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/final/kernel_stats.csv
cp $OUT/trace_bench.json $OUT/final/trace_bench.json
