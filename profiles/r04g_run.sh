set -o pipefail
# round 4: full bench at HEAD (fabric byte masks, LDS-row WAN pass, cursor KSP2 traces)
D=gpurun_out/r04g; mkdir -p $D
timeout -k 10 900 python bench.py > $D/bench_full.json 2> $D/bench_full.err || exit 5
python - <<'PY'
import json
d=json.load(open('gpurun_out/r04g/bench_full.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k in ('wan_all_sources','ksp2_route_db','route_db_rebuild','whatif_batch'):
    v=d.get(k) or {}
    print(k, {x: v.get(x) for x in ('ms','spf_ms','value','ms_median','build_ms_median','loop_ms_median','parity_check','kernel')})
PY
