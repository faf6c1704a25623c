set -o pipefail
# round 4: KMAX = 10 MS-BFS instance for the fabric (2 VGPR spills instead of 24) A/B
D=gpurun_out/r04ak; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
for g in 1 0; do
OPENR_MS_K10=$g timeout -k 10 300 python3 $B > $D/fabric_k10_$g.$i.json 2> $D/fabric_k10_$g.$i.err || { tail -5 $D/fabric_k10_$g.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric_k10_$g.$i.json')); print('k10=$g', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
done
timeout -k 10 600 python -u -m pytest tests/test_abi_gpu.py tests/test_config_sized_gpu.py tests/test_engine_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -15 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
