set -o pipefail
# round 5: full GPU suite + smoke + full bench at HEAD (v2 next-hop pass,
# in-place link-flap graph update, persistent host pool)
D=gpurun_out/r05n; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -10 $D/smoke.log; exit 4; }
tail -1 $D/smoke.log
timeout -k 10 900 python bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 5; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r05n/bench_full.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_source'))
for k in ('wan_all_sources','ksp2_route_db','route_db_rebuild','route_db_link_flap','whatif_batch','all_nodes_route_table','grid_route_db'):
    v=d.get(k) or {}
    print(k, {x: v.get(x) for x in ('ms','spf_ms','value','ms_median','build_ms_median','update_ms_median','parity_check','kernel','error','engine','cpu_oracle')})
print(json.dumps(d.get('whatif_batch',{}).get('roofline')))
PY
