set -o pipefail
# round 5: persistent host pool A/B on the RouteDb loops (OPENR_HOST_POOL=0
# starts fresh threads per section, the round-4 behaviour), link-flap update
# phases, and the launched-kernel names of the what-if plan
D=gpurun_out/r05o; mkdir -p $D
for i in 1 2; do
for p in 1 0; do
OPENR_HOST_POOL=$p timeout -k 10 300 python3 profiles/route_db_probe.py 8 > $D/rdb.p$p.$i.json 2> $D/rdb.p$p.$i.err || { tail -5 $D/rdb.p$p.$i.err; exit 2; }
python3 -c "
import json; d=json.load(open('$D/rdb.p$p.$i.json'))
r=d['route_db_rebuild']; k=d['ksp2_route_db']
print('pool=$p', 'rebuild', r['ms_median'], r['build_ms_median'], r.get('release_ms_median'), 'ksp2', k['ms_median'], k['build_ms_median'])"
done
done
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 4; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
grep "spf_graph_update" $D/linkflap.err | tail -9
timeout -k 10 300 python3 profiles/whatif_probe.py 2 > $D/whatif.json 2> $D/whatif.err || { tail -5 $D/whatif.err; exit 5; }
python3 -c "import json; d=json.load(open('$D/whatif.json')); print(d['kernels_launched'], d['roofline'].get('traffic_note'))"
