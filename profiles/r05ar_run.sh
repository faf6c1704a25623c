set -o pipefail
# what-if WAN baseline: the few-source LDS-row pass on or off
D=gpurun_out/r05ar; mkdir -p $D
R=$(pwd)
timeout -k 10 200 python3 profiles/whatif_probe.py 5 > $D/probe_default.json 2> $D/probe_default.err || exit 3
OPENR_SPF_DSTEP_LDSROW=0 timeout -k 10 200 python3 profiles/whatif_probe.py 5 > $D/probe_noldsrow.json 2> $D/probe_noldsrow.err || exit 3
for f in default noldsrow; do python3 -c "import json; d=json.load(open('$D/probe_$f.json')); print('$f', {k: d.get(k) for k in ('ms','device_ms','value','parity_check')})"; done
cd /tmp && export TMPDIR=/tmp
OPENR_SPF_DSTEP_LDSROW=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/$D/trace -o run --output-format csv -- python3 $R/profiles/whatif_probe.py 3 > $R/$D/trace.json 2>&1 || exit 4
cd $R
head -12 $(find $D/trace -name "*kernel_stats.csv" | head -1)
