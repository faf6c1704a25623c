set -o pipefail
# round 4: PMC of the what-if plan after the repair, then the full bench at HEAD
D=gpurun_out/r04q; mkdir -p $D/final
R=$(pwd); cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P -T -d $R/$D/wi_$P -o run --output-format csv -- \
    python3 $R/profiles/whatif_probe.py 2 --batches-out $R/$D/wi_batches.json > $R/$D/wi_$P.log 2>&1 || exit 3
done
cd $R
python3 profiles/collect_pmc.py $D/wi_FETCH_SIZE $D/wi_WRITE_SIZE $D/final/pmc_whatif.json || exit 4
python3 - <<PY
import json
D="$D"
wi=json.load(open(D+"/final/pmc_whatif.json")); wi["batches"]=json.load(open(D+"/wi_batches.json"))["batches"]
wi["what"]+="; what-if batch alone after the repair (profiles/whatif_probe.py 2: warm-up + 2 timed batches)"
json.dump(wi,open(D+"/final/pmc_whatif.json","w"),indent=1)
PY
mkdir -p profiles/r04q && cp $D/final/pmc_whatif.json profiles/r04q/
timeout -k 10 900 python bench.py > $D/bench_full.json 2> $D/bench_full.err || exit 5
python - <<'PY'
import json
d=json.load(open('gpurun_out/r04q/bench_full.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k in ('wan_all_sources','ksp2_route_db','route_db_rebuild','route_db_link_flap','whatif_batch','all_nodes_route_table'):
    v=d.get(k) or {}
    print(k, {x: v.get(x) for x in ('ms','spf_ms','value','ms_median','build_ms_median','update_ms_median','parity_check','kernel','error')})
PY
