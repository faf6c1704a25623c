set -o pipefail
# round 5: C-ABI lifetime tests, the metric-raise link-flap test, the grid
# (config 1) RouteDb breakdown, and the fabric step baseline at HEAD
D=gpurun_out/r05a; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_lifetime_gpu.py tests/test_engine_parity_gpu.py -k "lifetime or refused or link_flap or selective_memo or incremental" -x -v --timeout 240 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -3 $D/gpu_tests.log
timeout -k 10 200 python -u profiles/grid_probe.py --iters 200 > $D/grid_probe.json 2> $D/grid_probe.err || { tail -20 $D/grid_probe.err; exit 4; }
cat $D/grid_probe.json
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
timeout -k 10 300 python3 $B > $D/fabric.$i.json 2> $D/fabric.$i.err || { tail -5 $D/fabric.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.$i.json')); print(d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
