set -o pipefail
# round 4: the full bench at HEAD + the fabric-step profile (kernel trace and
# FETCH / WRITE passes) it prices its headline kernel against
D=gpurun_out/r04ap; mkdir -p $D


timeout -k 10 600 bash profiles/prof_fabric.sh r04ap > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 3; }
mkdir -p $D/prof && cp gpurun_out/prof_r04ap/final/* $D/prof/
timeout -k 10 900 python bench.py > $D/bench_full.json 2> $D/bench_full.err || exit 5
python - <<'PY'
import json
d=json.load(open('gpurun_out/r04ap/bench_full.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_source'))
for k in ('wan_all_sources','ksp2_route_db','route_db_rebuild','route_db_link_flap','whatif_batch','all_nodes_route_table'):
    v=d.get(k) or {}
    print(k, {x: v.get(x) for x in ('ms','spf_ms','value','ms_median','build_ms_median','update_ms_median','parity_check','kernel','error')})
PY
timeout -k 10 200 python3 profiles/route_table_probe.py --breakdown > $D/rt_breakdown.log 2>&1 || exit 6
tail -1 $D/rt_breakdown.log
