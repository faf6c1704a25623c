#!/bin/bash
# Round profile recipe for the host-driven sections (RouteDb rebuild, KSP2,
# all-nodes route table + route delta): kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE / WRITE_SIZE, as run_profiles.sh).
# Usage: bash profiles/run_profiles_routedb.sh <round-tag>
set -e
R=$(pwd)
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_rdb_$TAG
mkdir -p $OUT/final
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-wan --no-whatif"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
  python3 $B --steps 5 --warmup 2 > $OUT/trace_bench.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o run --output-format csv -- \
  python3 $B --steps 2 --warmup 1 > $OUT/pmc_fetch.json
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o run --output-format csv -- \
  python3 $B --steps 2 --warmup 1 > $OUT/pmc_write.json
cd $R
python3 profiles/collect_pmc.py $OUT/pmc_fetch $OUT/pmc_write $OUT/final/pmc_traffic.json
cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/final/kernel_stats.csv
cp $OUT/trace_bench.json $OUT/final/trace_bench.json
