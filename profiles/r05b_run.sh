set -o pipefail
# round 5: v2 held next-hop pass (solo items without the LDS staging chain,
# RSW groups sharing their neighbours' level words): A/B vs the held kernel,
# then the fabric / ABI parity tests with v2 on (the default)
D=gpurun_out/r05b; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
for v in 1 0; do
OPENR_NL_V2=$v timeout -k 10 300 python3 $B > $D/fabric.v$v.$i.json 2> $D/fabric.v$v.$i.err || { tail -5 $D/fabric.v$v.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.v$v.$i.json')); print('v2=$v', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
done
timeout -k 10 600 python -u -m pytest tests/test_config_sized_gpu.py tests/test_abi_gpu.py tests/test_zero_metric_plan.py tests/test_routedb_golden_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
