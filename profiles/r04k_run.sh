set -o pipefail
# round 4: price every config's dominant kernel at HEAD --
#  (1) PMC over the full 100k-source WAN pass (spf_dlds_kernel),
#  (2) kernel trace + PMC over the what-if batch alone (profiles/whatif_probe.py),
#  (3) PMC over the all-nodes route table alone (spf_route_table_kernel).
R=$(pwd); D=$R/gpurun_out/r04k; mkdir -p $D/final
cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $P -T -d $D/wan_$P -o run --output-format csv -- \
    python3 $R/profiles/quick_wan.py 100000 base > $D/wan_$P.log 2>&1 || exit 3
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $D/wi_trace -o run --output-format csv -- \
  python3 $R/profiles/whatif_probe.py 5 > $D/wi_trace.log 2>&1 || exit 4
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P -T -d $D/wi_$P -o run --output-format csv -- \
    python3 $R/profiles/whatif_probe.py 2 --batches-out $D/wi_batches.json > $D/wi_$P.log 2>&1 || exit 5
done
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $P -T -d $D/rt_$P -o run --output-format csv -- \
    python3 $R/profiles/route_table_probe.py > $D/rt_$P.log 2>&1 || exit 6
done
cd $R
python3 profiles/collect_pmc.py $D/wan_FETCH_SIZE $D/wan_WRITE_SIZE $D/pmc_wan.json &&
python3 profiles/collect_pmc.py $D/wi_FETCH_SIZE $D/wi_WRITE_SIZE $D/final/pmc_whatif.json &&
python3 profiles/collect_pmc.py $D/rt_FETCH_SIZE $D/rt_WRITE_SIZE $D/pmc_rt.json &&
python3 - <<PY
import json
D="$D"
wi=json.load(open(D+"/final/pmc_whatif.json")); wi["batches"]=json.load(open(D+"/wi_batches.json"))["batches"]
wi["what"]+="; what-if batch alone (profiles/whatif_probe.py 2: warm-up + 2 timed batches)"
json.dump(wi,open(D+"/final/pmc_whatif.json","w"),indent=1)
out={"what":"per-launch HBM bytes (2*FETCH_SIZE + WRITE_SIZE): spf_dlds_kernel from quick_wan.py 100000 base "
     "(the full 100,000-source WAN pass), route-table kernels from profiles/route_table_probe.py","kernels":{}}
for f,ks in (("pmc_wan.json",("spf_dlds_kernel","spf_dstep_kernel")),("pmc_rt.json",("spf_route_table_kernel","spf_route_table_diff_kernel"))):
    d=json.load(open(D+"/"+f))["kernels"]
    for k in ks:
        if k in d: out["kernels"][k]=d[k]
json.dump(out,open(D+"/final/pmc_traffic.json","w"),indent=1)
print(json.dumps(out)[:3000]); print(json.dumps(wi)[:3000])
PY
cp $(find $D/wi_trace -name "*kernel_stats.csv" | head -1) $D/final/whatif_kernel_stats.csv
tail -2 $D/wan_FETCH_SIZE.log $D/wi_trace.log $D/rt_FETCH_SIZE.log
