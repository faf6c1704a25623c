set -o pipefail
# KSP2 heavy-trace tuning: budget sweep, then a kernel trace of the default
D=gpurun_out/r05x; mkdir -p $D
R=$(pwd)
timeout -k 10 400 python3 profiles/ksp2_budget_probe.py "OPENR_SPF_TRACE_HEAVY=0" "" "OPENR_SPF_TRACE_BUDGET=512" "OPENR_SPF_TRACE_BUDGET=1024" "OPENR_SPF_TRACE_BUDGET=4096" "OPENR_SPF_TRACE_STATS=1" > $D/sweep.json 2> $D/sweep.err || { tail -5 $D/sweep.err; exit 3; }
cat $D/sweep.json; grep "trace" $D/sweep.err | tail -6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/$D/trace -o run --output-format csv -- python3 $R/profiles/ksp2_budget_probe.py "" > $R/$D/trace.json 2>&1 || exit 4
cd $R
head -12 $(find $D/trace -name "*kernel_stats.csv" | head -1)
