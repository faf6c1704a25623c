set -o pipefail
# round 4: held pass issues the source's own level word + distance-row store
# before the neighbour staging
D=gpurun_out/r04aq; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2 3; do
timeout -k 10 300 python3 $B > $D/fabric.$i.json 2> $D/fabric.$i.err || { tail -5 $D/fabric.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.$i.json')); print(d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
timeout -k 10 600 python -u -m pytest tests/test_abi_gpu.py tests/test_config_sized_gpu.py tests/test_all_sources_table_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -15 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
