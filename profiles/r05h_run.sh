set -o pipefail
# round 5: spf_graph_update (link flaps rebuild the device graph in place),
# its parity tests and the link-flap RouteDb loop; held vs v2 (order 3)
D=gpurun_out/r05h; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_graph_update_gpu.py tests/test_abi_lifetime_gpu.py tests/test_engine_parity_gpu.py -k "update or refused or link_flap or selective_memo or incremental or random_route_db" -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 4; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
for v in 0 1; do
OPENR_NL_V2=$v OPENR_NL_V2_ORDER=3 timeout -k 10 300 python3 $B > $D/fabric.v$v.$i.json 2> $D/fabric.v$v.$i.err || { tail -5 $D/fabric.v$v.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.v$v.$i.json')); print('v2=$v', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
done
