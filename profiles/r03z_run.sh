set -o pipefail
D=gpurun_out/r03z; mkdir -p $D
timeout -k 10 300 python profiles/scaling_probe.py > $D/scaling_probe.json 2> $D/probe.err || exit 5
cat $D/scaling_probe.json | python -c "import json,sys; d=json.load(sys.stdin); [print(k, v['sources'], v['kernel'], v['ms'], v['stage_ms']) for k,v in d.items()]"
timeout -k 10 600 python -u -m pytest tests/test_routedb_golden_gpu.py -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -2 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "
import bench, json
from openr_amd import topologies as TP
topo = TP.fabric(10000)
for i in range(2):
    r = bench.ksp2_route_db(topo, 0)
    print(json.dumps({k: r[k] for k in ('ms_median','update_ms_median','build_ms_median','release_ms_median','parity_check')}), json.dumps({k: r['per_build'][k] for k in ('kth_memo_clear_us','route_prefetch_us','route_prefix_pool_us','route_label_us','route_merge_us')}))
" > $D/ksp2.json 2> $D/ksp2.err || exit 6
cat $D/ksp2.json
