set -o pipefail
# round-6 HEAD after the what-if and route-shard changes: full bench, what-if
# plan PMC, smoke
R=$(pwd)
D=gpurun_out/r06y; mkdir -p $D
timeout -k 10 600 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 3; }
cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P -T -d $R/$D/wi_$P -o run --output-format csv -- \
    python3 $R/profiles/whatif_probe.py 2 --batches-out $R/$D/wi_batches.json > $R/$D/wi_$P.log 2>&1 || exit 4
done
cd $R
python3 profiles/collect_pmc.py $D/wi_FETCH_SIZE $D/wi_WRITE_SIZE $D/pmc_whatif.json || exit 5
python3 - <<PY
import json
D="$D"
wi=json.load(open(D+"/pmc_whatif.json")); wi["batches"]=json.load(open(D+"/wi_batches.json"))["batches"]
wi["what"]+="; what-if batch alone at round-6 HEAD (first-hop form, work list; profiles/whatif_probe.py 2: warm-up + 2 timed batches)"
json.dump(wi,open(D+"/pmc_whatif.json","w"),indent=1)
b=json.loads(open(D+"/bench_full.json").read().strip().splitlines()[-1])
print(b["value"], b["ms_per_step"], b["roofline"]["frac"], b.get("table_path",{}).get("value"))
for k in ("route_db_rebuild_lfa","route_db_rebuild","ksp2_route_db","route_db_link_flap","whatif_batch","wan_all_sources","grid_route_db"):
    v=b.get(k,{}); print(k, {x: v.get(x) for x in ("ms_median","build_ms_median","release_ms_median","ms","value","engine")})
PY
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 6; }
tail -1 $D/smoke.log
