set -o pipefail
# per-engine query cache (OPENR_LS_QUERY_CACHE) on top of the small-area
# MS-BFS plan: grid RouteDb A/B, GPU tests, bench
R=$(pwd)
D=gpurun_out/r06ap; mkdir -p $D
OPENR_LS_QUERY_CACHE=0 timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_off.json 2> $D/grid_off.err || exit 3
timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_on.json 2> $D/grid_on.err || exit 4
python3 - <<PY
import json
for t in ("off", "on"):
    j = json.load(open("$D/grid_%s.json" % t))
    e = j["engine"]["per_build_us"]
    print(t, j["engine"]["ms_median"], e.get("decision.spf_batch_us"), e.get("decision.spf_device_us"), e.get("decision.route_build_us"), "oracle", j["cpu_oracle"]["ms_median"])
PY
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 6; }
tail -2 $D/gpu_tests.log
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 7; }
python3 -c "
import json; j=json.loads(open('$D/bench.json').read().strip().splitlines()[-1]); print(j['value'], j['ms_per_step']); 
print({k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if 'ms' in kk or 'value' in kk}) for k, v in j.items() if k in ('grid_route_db','route_db','whatif','link_flap','ksp2')})
"
