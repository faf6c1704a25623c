set -o pipefail
# fused host fetch (spf_query_fetch_host): grid probes, fetch parity, engine
# parity and RouteDb goldens
D=gpurun_out/r06az; mkdir -p $D
timeout -k 10 200 python3 profiles/grid_run_probe.py 2000 > $D/run.json 2>/dev/null || exit 3
cat $D/run.json
OPENR_SPF_FETCH_STAGE=0 timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_off.json 2>/dev/null || exit 4
timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_on.json 2>/dev/null || exit 5
python3 -c "
import json
for t in ('off','on'):
    j=json.load(open('$D/grid_%s.json'%t)); e=j['engine']['per_build_us']
    print(t, j['engine']['ms_median'], e.get('decision.spf_batch_us'), 'oracle', j['cpu_oracle']['ms_median'])"
timeout -k 10 600 python3 -u -m pytest tests/test_abi_gpu.py tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 6; }
tail -1 $D/t.log
