set -o pipefail
# round-6 end state after the grid changes: full bench, GPU suite, smoke
D=gpurun_out/r06ba; mkdir -p $D
timeout -k 10 600 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 3; }
python3 - <<PY
import json
b=json.loads(open("$D/bench_full.json").read().strip().splitlines()[-1])
print(b["value"], b["ms_per_step"], b["roofline"]["frac"], b["roofline"].get("traffic_source"), b.get("table_path",{}).get("value"))
for k in ("route_db_rebuild_lfa","route_db_rebuild","ksp2_route_db","route_db_link_flap","whatif_batch","wan_all_sources","grid_route_db"):
    v=b.get(k,{}); print(k, {x: v.get(x) for x in ("ms_median","build_ms_median","release_ms_median","ms","value","engine")})
print(json.dumps(b["whatif_batch"].get("roofline"))[:400])
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 4; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 5; }
tail -1 $D/smoke.log
