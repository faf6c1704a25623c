set -o pipefail
# round 5: v3 next-hop pass (scalar-loaded neighbour entries, one word loop
# not unrolled) x block order 0 / 1 / 3, with parity spot checks, then the
# all-sources parity tests
D=gpurun_out/r05g; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
for o in 0 1 3; do
OPENR_NL_V2_ORDER=$o timeout -k 10 300 python3 $B > $D/fabric.o$o.$i.json 2> $D/fabric.o$o.$i.err || { tail -5 $D/fabric.o$o.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.o$o.$i.json')); print('order=$o', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
done
for v in 1 4 5 6; do
OPENR_NL_V2_ORDER=3 OPENR_NL_V2_DBG=$v timeout -k 10 300 python3 $B > $D/fabric.d$v.json 2> $D/fabric.d$v.err || { tail -5 $D/fabric.d$v.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.d$v.json')); print('dbg=$v', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 120 python3 profiles/graph_create_probe.py > $D/create_probe.log 2>&1 || { tail -5 $D/create_probe.log; exit 4; }
cat $D/create_probe.log
timeout -k 10 600 python -u -m pytest tests/test_config_sized_gpu.py tests/test_abi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
